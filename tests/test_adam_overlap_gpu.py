"""Per-layer Adam overlapped with the backward (Trainer.step,
SMER_ADAM_OVERLAP, default on): each layer range's update runs on the
weight-gradient stream as soon as its gradients are final, behind the main
stream's reads of that layer's working weights.  Adam is elementwise, so
parameters, moments and the bf16 working copy must equal the single
end-of-step Adam bit for bit, step after step (train.py:786 optim.step())."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model_and_batch(precision):
    from smer_music_generation_amd.model import ScoreTransformer
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    torch.manual_seed(0)
    m = ScoreTransformer(309, 512, 8, 2, 2, 2048, 2400, 0.1, 0.1, precision=precision).to("cuda")
    b = synth_training_batch(77, v, 4, 1024, 256)
    return m, v, {k: torch.from_numpy(np.asarray(x)).to("cuda") for k, x in b.items()}


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_overlapped_adam_equals_end_of_step_adam(monkeypatch, precision):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from smer_music_generation_amd.train import Trainer
    m0, v, bt = _model_and_batch(precision)
    m1, _, _ = _model_and_batch(precision)
    t0, t1 = Trainer(m0, v, lr=1e-3), Trainer(m1, v, lr=1e-3)
    for k in range(3):
        monkeypatch.setenv("SMER_ADAM_OVERLAP", "0")
        l0 = t0.step(bt)
        monkeypatch.setenv("SMER_ADAM_OVERLAP", "1")
        l1 = t1.step(bt)
        torch.cuda.synchronize()
        assert torch.equal(l0, l1), k
        assert torch.equal(m0.flat_parameters(), m1.flat_parameters()), k
        assert torch.equal(t0.m, t1.m) and torch.equal(t0.v, t1.v), k
        if precision == "bf16":
            assert torch.equal(m0.engine._bf16, m1.engine._bf16), k
