"""Golden vectors for the rest of the plugin wire surface:
`change_controls` (generation.py:698-877, both bar_track modes) and
`fill_empty_bars` (generation.py:230-245, including the 'a_0' placeholder
quirk Q9), produced by running the REFERENCE in the build container.

RUN ONLY IN THE BUILD CONTAINER (imports /root/reference; absent MIDI / log
libraries stubbed as empty modules).  Writes data only.

    python tests/golden/make_golden_wire.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(OUT, "..", ".."))
sys.path.insert(0, REF)
for _m in ("pretty_midi", "music21", "coloredlogs"):
    sys.modules.setdefault(_m, types.ModuleType(_m))

import encode as ref_encode        # noqa: E402  (reference)
import generation as ref_gen       # noqa: E402  (reference)

from smer_music_generation_amd.synth import synth_events  # noqa: E402


def controls_for(rng, n_tracks, n_bars, mode):
    c = {"bar_track": mode}
    for t in range(n_tracks):
        c["track_%d_c" % t] = {"density": int(rng.integers(10)), "polyphony": int(rng.integers(10)),
                               "occupation": int(rng.integers(10))}
    names = ["track_%d" % t for t in range(n_tracks)]
    if mode == 0:
        for key in ("bar_density", "bar_occupation", "bar_polyphony"):
            # value 10 = 'unk' (control left to the model)
            c[key] = {n: [int(x) for x in rng.integers(0, 11, n_bars)] for n in names}
    else:
        c["s_bar"] = int(rng.integers(0, n_bars))
        c["e_bar"] = int(rng.integers(c["s_bar"], n_bars))
        for n in names:
            c[n] = int(rng.integers(0, 2))
    return c


def change_controls_golden():
    recs = []
    rng = np.random.default_rng(17)
    for seed, nb, nt, ts in ((60, 3, 2, "4/4"), (61, 4, 3, "3/4"), (62, 2, 1, "6/8"),
                             (63, 5, 3, "4/4"), (64, 3, 2, "2/4")):
        for mode in (0, 1):
            ev = synth_events(seed, nb, nt, time_signature=ts, copy_controls=False)
            c = controls_for(rng, nt, nb, mode)
            out = ref_gen.change_controls(list(ev), json.loads(json.dumps(c)))
            recs.append({"events": ev, "controls": c, "out": [str(x) for x in out]})
    return recs


def fill_empty_bars_golden():
    recs = []
    for seed, nb, nt, ts, n_fill in ((70, 2, 2, "4/4", 1), (71, 3, 3, "3/4", 2),
                                     (72, 2, 1, "6/8", 1), (73, 1, 2, "2/4", 3)):
        ev = synth_events(seed, nb, nt, time_signature=ts)
        num, den = int(ev[0][0]), int(ev[0][2])
        # generation.py:470-475
        _, t2n, times, bar_dur = ref_encode.get_note_duration_dict(1.5 if den == 8 else 1, (num, den))
        out = ref_gen.fill_empty_bars(list(ev), n_fill, bar_dur, t2n, times)
        recs.append({"events": ev, "n_fill": n_fill, "out": [str(x) for x in out]})
    return recs


if __name__ == "__main__":
    with open(os.path.join(OUT, "wire_golden.json"), "w") as f:
        json.dump({"change_controls": change_controls_golden(),
                   "fill_empty_bars": fill_empty_bars_golden()}, f)
    print("written", os.path.join(OUT, "wire_golden.json"))
