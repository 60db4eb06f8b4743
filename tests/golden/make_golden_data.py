"""Golden vectors for the training-data pipeline, generated
by running the REAL reference in this container.

RUN ONLY IN THE BUILD CONTAINER (needs /root/reference; never on the GPU box).
It imports the reference's `dataset.py` and `vocab.py` (absent MIDI / log
libraries stubbed as empty modules) and evaluates only the `stack_batches`
function of `load_dataset.py` (that module runs a corpus-build script at
import, so the function's definition is taken out of the source with `ast`
and executed alone, its pickle loads answered from memory).  Inputs are
synthetic SMER songs (smer_music_generation_amd.synth.synth_events, seeded),
so the fixture stores their seeds, not the songs.  Output: data only.

    python tests/golden/make_golden_data.py
"""
from __future__ import annotations

import ast
import copy
import json
import logging
import os
import random
import sys
import types
import zlib

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(OUT, "..", ".."))
sys.path.insert(0, REF)
for _m in ("pretty_midi", "music21", "coloredlogs"):
    sys.modules.setdefault(_m, types.ModuleType(_m))

import dataset as ref_dataset  # noqa: E402  (reference)
import vocab as ref_vocab      # noqa: E402  (reference)

from tests.golden.data_common import CASES, STACK_CASE, build_files, flatten_item  # noqa: E402


def ref_stack_batches():
    src = open(os.path.join(REF, "load_dataset.py")).read()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "stack_batches"][0]
    mod = ast.Module(body=[fn], type_ignores=[])
    store = {}

    class _Pickle:
        @staticmethod
        def load(f):
            return store[f.name]

    class _Opened:
        def __init__(self, name, mode):
            self.name = name

    ns = {"np": np, "re": __import__("re"), "random": random, "gc": __import__("gc"),
          "pickle": _Pickle, "open": _Opened, "vocab": ref_vocab,
          "logger": logging.getLogger("stack_batches")}
    exec(compile(mod, "load_dataset.py:stack_batches", "exec"), ns)
    return ns["stack_batches"], store


def main():
    stack, store = ref_stack_batches()
    out = {}
    meta = {"stack": None, "cases": []}

    # ---- stack_batches ----
    files = build_files(STACK_CASE["files"])
    names = []
    for k, evs in enumerate(files):
        store["f%d" % k] = evs
        names.append("f%d" % k)
    flat = [ev for evs in files for ev in evs]
    groups, lengths = stack(names, max_token_length=STACK_CASE["max_token_length"])
    where = {id(ev): i for i, ev in enumerate(flat)}
    meta["stack"] = {"groups": [[where[id(ev)] for ev in g] for g in groups],
                     "lengths": {str(k): v for k, v in lengths.items()}}

    # ---- dataset items ----
    for ci, case in enumerate(CASES):
        v = ref_vocab.WordVocab(0, case["controls"])
        files = build_files(case["files"])
        store.clear()
        names = []
        for k, evs in enumerate(files):
            store["f%d" % k] = evs
            names.append("f%d" % k)
        groups, lengths = stack(names, max_token_length=case["max_token_length"])
        np.random.seed(case["np_seed"])
        ds = ref_dataset.ParallelLanguageDataset(
            v, groups, lengths, case["batch_size"], total_mask_ratio=.15, logger=None,
            pretraining=case["pretraining"], bar_track_control=case["bar_track_control"],
            bar_control_at_end=case["bar_control_at_end"])
        items = [ds[i] for i in range(case["items"])]
        vals, struct = [], []
        for it in items:
            flatten_item(it, vals, struct)
        out["case%d_vals" % ci] = np.array(vals, dtype=np.int32)
        out["case%d_struct" % ci] = np.array(struct, dtype=np.int32)
        coll = ref_dataset.collate_mlm_pretraining(copy.deepcopy(items[:case["batch_size"]]))
        cmeta = {k: [list(t.shape), int(t.long().sum()), int(zlib.crc32(t.numpy().tobytes()))]
                 for k, t in coll.items()} if coll is not None else None
        state = [zlib.crc32(" ".join(ev).encode()) for g in groups for ev in g]
        meta["cases"].append({"collate": cmeta, "groups_after": state,
                              "next_random": random.random(), "next_np": float(np.random.random())})
        print("case", ci, case["name"], "items", len(items), "values", len(vals))
    np.savez_compressed(os.path.join(OUT, "data_golden.npz"), **out)
    json.dump(meta, open(os.path.join(OUT, "data_golden.json"), "w"))
    print("wrote data_golden.npz / data_golden.json")


if __name__ == "__main__":
    main()
