"""Diagnostic: per-parameter gradient error of the fp32 engine vs the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import ref_cpu
from smer_music_generation_amd.model import ScoreTransformer
from smer_music_generation_amd.train import Trainer
from smer_music_generation_amd.vocab import WordVocab
from smer_music_generation_amd.synth import synth_training_batch
d, H, F, B, S, T = [int(x) for x in sys.argv[1:7]]
v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
torch.manual_seed(1)
m = ScoreTransformer(309, d, H, 2, 2, F, 2400, 0.0, 0.0, precision=sys.argv[7] if len(sys.argv) > 7 else "fp32")
sd = {k: t.detach().clone() for k, t in m.state_dict().items()}
m = m.to("cuda")
b = synth_training_batch(11, v, B, S, T)
b["input"][1, S - 10:] = 0
b["input_pad_mask"] = b["input"] == 0
cfg = dict(d_model=d, nhead=H, num_encoder_layers=2, num_decoder_layers=2)
rl, parts, grads, logits = ref_cpu.train_step(sd, cfg, b, v.control_indices, 0.8, 8)
tr = Trainer(m, v)
loss = tr.step({k: torch.from_numpy(np.asarray(x)).to("cuda") for k, x in b.items()})
print("loss", loss.item(), float(rl))
for name, p in m.named_parameters():
    ref = grads[name].numpy(); g = p.grad.cpu().numpy()
    mx = np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-12)
    fro = np.linalg.norm(g - ref) / max(np.linalg.norm(ref), 1e-12)
    if True:
        i = np.unravel_index(np.argmax(np.abs(g - ref)), ref.shape)
        print("%-55s max %.1e fro %.1e" % (name[12:], mx, fro))
