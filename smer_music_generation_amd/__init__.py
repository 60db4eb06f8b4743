"""smer_music_generation_amd — MI355X-native SMER infilling engine.

Drop-in for the reference's hot path: `ScoreTransformer`
(model.py), `model_generate` / `generation_all` / `infill` (generation.py),
`WordVocab` (vocab.py), and a fused data-parallel `Trainer` (train.py),
all running hand-written gfx950 kernels from libsmer_hip.so (include/smer_hip.h).
"""
from .vocab import WordVocab  # noqa: F401

__all__ = ["WordVocab", "ScoreTransformer", "Trainer", "generation_all", "infill",
           "model_generate", "generation_batch"]


def __getattr__(name):  # lazy: importing torch-heavy modules only when used
    if name == "ScoreTransformer":
        from .model import ScoreTransformer
        return ScoreTransformer
    if name == "Trainer":
        from .train import Trainer
        return Trainer
    if name in ("generation_all", "infill", "model_generate", "generation_batch"):
        from . import generation
        return getattr(generation, name)
    raise AttributeError(name)
