"""Per-shape GEMM time of one C4 train step (weight gradients serialised on
the main stream so every launch's time is its own), from the live HIP-event
timer: which contractions stay bf16 in the fp8 step and what they cost.
    python tools/c4_shapes.py [fp8|bf16]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SMER_WGRAD_OVERLAP"] = "0"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smer_music_generation_amd import ops  # noqa: E402
from smer_music_generation_amd.synth import synth_training_batch  # noqa: E402
from smer_music_generation_amd.train import Trainer  # noqa: E402
from smer_music_generation_amd.vocab import WordVocab  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp8"
args = bench.parse_args([])
args.layers, args.d_model, args.nhead, args.seq, args.tgt = 12, 768, 12, 2048, 512
dev = torch.device("cuda", 0)
v = WordVocab(0, bench.CTRL)
m = bench.make_model(args, dev, prec)
tr = Trainer(m, v, lr=1e-4)
b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
for _ in range(3):
    tr.step(bt)
torch.cuda.synchronize()
timer = ops.KernelTimer()
ops.GEMM_TIMER = timer
tr.step(bt)
torch.cuda.synchronize()
ops.GEMM_TIMER = None
rows = sorted(timer.by_shape().items(), key=lambda kv: -kv[1][1])
tot = sum(r[1][1] for r in rows)
print("%s C4 step: %d GEMM launches, %.2f ms" % (prec, sum(r[1][0] for r in rows), tot))
for tag, (n, t, f) in rows:
    print("%-44s %4d  %8.3f ms  %7.1f TF/s" % (tag, n, t, f / (t * 1e-3) / 1e12 if t else 0))
