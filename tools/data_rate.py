"""Host throughput of the training-data pipeline (pretraining items +
collate), one process.  With --reference (build container only) the
reference's dataset.py is timed on the same groups.

    python tools/data_rate.py [--seconds 5] [--mode 2] [--reference]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smer_music_generation_amd.data import measure_rate  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=5.0)
ap.add_argument("--mode", type=int, default=2)
ap.add_argument("--pretraining", type=int, default=1)
ap.add_argument("--reference", action="store_true")
a = ap.parse_args()
print("ours", measure_rate(a.seconds, a.mode, bool(a.pretraining)))
if a.reference:
    import types
    sys.path.insert(0, "/root/reference")
    for _m in ("pretty_midi", "music21", "coloredlogs"):
        sys.modules.setdefault(_m, types.ModuleType(_m))
    import dataset as ref_dataset  # reference (timing only)
    import vocab as ref_vocab
    t0 = time.time()
    print("reference", measure_rate(a.seconds, a.mode, bool(a.pretraining),
                                    dataset_cls=ref_dataset.ParallelLanguageDataset,
                                    collate=ref_dataset.collate_mlm_pretraining,
                                    vocab=ref_vocab.WordVocab(0, ['key', 'tensile', 'density',
                                                                  'polyphony', 'occupation'])))
