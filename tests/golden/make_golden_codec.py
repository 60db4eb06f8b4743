"""Golden vectors for the MIDI <-> SMER codec's pure functions (SURVEY §8
row f4), produced by running the REFERENCE `encode.py` in the build
container on inputs that need no MIDI library:

* `to_category` (`encode.py:206-210`) on control values and bin edges;
* `note_density` / `bar_track_density` (`encode.py:13-50`) on per-bar
  token lists;
* `get_note_duration_dict` (`encode.py:213-277`) and `time2durations`
  (`encode.py:947-954`) over tempi and the four supported metres;
* `grid_notes` (`encode.py:900-936`) on notes given as plain attribute
  objects (start / end / pitch / velocity), including continued notes
  (velocity -1) and notes shorter than a grid step;
* `note_to_event_name` (`encode.py:939-944`);
* `bar_notes_to_event` (`encode.py:957-1141`) on bars whose notes end
  inside the bar, with continued notes from the previous bar as inputs;
* `bar_notes_to_event`'s cross-bar continuation branch
  (`encode.py:1028-1040,1109-1121`): notes running past the bar line.  That
  branch builds `pretty_midi.Note(pitch=, start=, end=, velocity=)` objects
  (pretty_midi is absent here), so the empty stub module gets a recorder
  class `Note` holding exactly those four attributes; the carried notes are
  recorded as [pitch, start, end, velocity].

RUN ONLY IN THE BUILD CONTAINER (imports /root/reference; the absent MIDI /
music libraries are stubbed as EMPTY modules, as in make_golden_wire.py).
Writes data only.

    python tests/golden/make_golden_codec.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
for _m in ("pretty_midi", "music21", "coloredlogs", "tension_calculation"):
    sys.modules.setdefault(_m, types.ModuleType(_m))



class _RecNote:
    """Recorder standing for pretty_midi.Note on the continuation branch:
    the four keyword attributes the reference passes and later reads."""

    def __init__(self, pitch, start, end, velocity):
        self.pitch, self.start, self.end, self.velocity = pitch, start, end, velocity


sys.modules["pretty_midi"].Note = _RecNote

import encode as ref_encode  # noqa: E402  (reference)

SIGS = ((4, 4), (3, 4), (2, 4), (6, 8))


class PlainNote:
    """Attribute container standing for a note object (the reference only
    reads and writes start / end / pitch / velocity on these paths)."""

    def __init__(self, pitch, start, end, velocity):
        self.pitch, self.start, self.end, self.velocity = pitch, start, end, velocity


def to_category_cases(rng):
    bins = np.arange(0, 1, 0.1)
    vals = list(rng.random(200)) + [0.0, 0.1, 0.0999999, 0.3, 0.5, 0.9, 0.95, 0.99999, 1.0, 2.5]
    return {"values": [float(v) for v in vals],
            "out": ref_encode.to_category(np.asarray(vals), bins)}


def _bar_tokens(rng, n):
    """A plausible bar of one track: pitch runs and duration / rest / sep tokens."""
    toks = []
    for _ in range(n):
        r = rng.random()
        if r < 0.5:
            toks += ["p_%d" % rng.integers(40, 90) for _ in range(int(rng.integers(1, 4)))]
            toks += ["quarter"] if rng.random() < 0.5 else ["eighth", "sixteenth"]
        elif r < 0.75:
            toks += ["rest", "half"]
        else:
            toks += ["sep", "eighth"]
    return toks


def density_cases(rng):
    recs = []
    for case in range(8):
        n_tracks, n_bars = int(rng.integers(1, 4)), int(rng.integers(1, 6))
        tracks = {"track_%d" % t: [_bar_tokens(rng, int(rng.integers(0, 8))) for _ in range(n_bars)]
                  for t in range(n_tracks)}
        length = int(rng.choice([12, 16, 24]))
        total = length * n_bars
        tot, per_bar = ref_encode.note_density(tracks, length, total)
        single = [ref_encode.bar_track_density([bar], length) for bar in tracks["track_0"]]
        recs.append({"tracks": tracks, "track_length": length, "total_length": total,
                     "total": [float(x) for x in tot],
                     "per_bar": {k: [float(x) for x in v] for k, v in per_bar.items()},
                     "bar_track_density": [float(x) for x in single]})
    return recs


def duration_cases(rng):
    recs = []
    for sig in SIGS:
        for beat in (0.5, 0.6, 1.0, 1.5, 0.4166666666666667):
            name_to_time, time_to_name, times, bar = ref_encode.get_note_duration_dict(beat, sig)
            probes = list(rng.random(40) * bar * 1.2) + [0.0, bar, name_to_time["sixteenth"] / 2]
            recs.append({"sig": list(sig), "beat": beat, "bar": float(bar),
                         "name_to_time": {k: float(v) for k, v in name_to_time.items()},
                         "times": [float(x) for x in times],
                         "probes": [float(x) for x in probes],
                         "durations": [ref_encode.time2durations(p, time_to_name, times) for p in probes]})
    return recs


def _grid(beat, sig):
    division = 6 if sig == (6, 8) else 4
    n_beats = int(4 * sig[0] / sig[1])
    beats = [beat * i for i in range(n_beats + 1)]
    return beats, division


def _random_notes(rng, bar_start, bar_end, n, step, allow_cont):
    notes = []
    for k in range(n):
        if allow_cont and k == 0 and rng.random() < 0.5:  # continued from the previous bar
            end = bar_start + step * int(rng.integers(1, 8)) + rng.normal(0, step / 10)
            notes.append([int(rng.integers(40, 80)), bar_start, float(min(end, bar_end - step)), -1])
            continue
        start = bar_start + rng.random() * (bar_end - bar_start - 2 * step)
        length = step * rng.choice([0.3, 1, 2, 3, 4, 6, 8])
        end = min(start + length + rng.normal(0, step / 8), bar_end - step)
        if end <= start:
            end = start + step * 0.4
        notes.append([int(rng.integers(40, 80)), float(start), float(end), int(rng.integers(30, 120))])
    # a chord: copies of one note with other pitches
    if n >= 2 and rng.random() < 0.6:
        p, s, e, v = notes[-1]
        notes.append([p + 4, s, e, v])
        notes.append([p + 7, s + step / 20, e - step / 20, v])
    return notes


def grid_cases(rng):
    recs = []
    for sig in SIGS:
        for beat in (0.5, 0.75):
            beats, division = _grid(beat, sig)
            name_to_time, _, _, _ = ref_encode.get_note_duration_dict(beat, sig)
            min_diff = name_to_time["sixteenth"] / 2
            for _ in range(4):
                raw = _random_notes(rng, 0.0, beats[-1], int(rng.integers(1, 10)), beat / division, True)
                notes = [PlainNote(*n) for n in raw]
                ref_encode.grid_notes(np.asarray(beats), notes, min_diff, grid_division=division)
                recs.append({"beats": beats, "division": division, "min_diff": min_diff, "notes": raw,
                             "out": [[float(n.start), float(n.end)] for n in notes]})
    return recs


def bar_event_cases(rng):
    recs = []
    for sig in SIGS:
        for beat in (0.5, 0.6):
            beats, division = _grid(beat, sig)
            name_to_time, time_to_name, times, bar = ref_encode.get_note_duration_dict(beat, sig)
            min_diff = name_to_time["sixteenth"] / 2
            for _ in range(6):
                n = int(rng.integers(0, 12))
                raw = _random_notes(rng, 0.0, bar, n, beat / division, True) if n else []
                notes = [PlainNote(*x) for x in raw]
                ev, carry = ref_encode.bar_notes_to_event(notes, 0.0, bar, np.asarray(beats), time_to_name,
                                                          times, min_diff, grid_division=division)
                assert not carry  # notes end inside the bar: no pretty_midi.Note was built
                tok = None
                if raw:
                    nt = PlainNote(*raw[0])
                    tok = list(ref_encode.note_to_event_name(nt, time_to_name, times))
                recs.append({"sig": list(sig), "beat": beat, "beats": beats, "division": division,
                             "min_diff": min_diff, "bar": float(bar), "notes": raw, "events": ev,
                             "note_to_event_name": tok})
    return recs


def _cross_notes(rng, bar, n, step):
    """Notes of one bar of which some run past the bar line (ties), chords
    of tied and untied notes, and a continued note from the previous bar."""
    notes = []
    if rng.random() < 0.5:  # continued from the previous bar, maybe tied on
        end = step * int(rng.integers(1, 8)) if rng.random() < 0.5 else bar + step * int(rng.integers(1, 12))
        notes.append([int(rng.integers(40, 80)), 0.0, float(end), -1])
    for _ in range(n):
        start = rng.random() * (bar - 2 * step)
        if rng.random() < 0.45:  # past the bar line
            end = bar + step * rng.choice([0.5, 1, 3, 8, 17])
        else:
            end = min(start + step * rng.choice([0.3, 1, 2, 4, 8]), bar - step)
            if end <= start:
                end = start + 0.4 * step
        notes.append([int(rng.integers(40, 80)), float(start), float(end), int(rng.integers(30, 120))])
    if notes and rng.random() < 0.7:  # a chord on the last note, some members tied
        p, s0, e0, v = notes[-1]
        notes.append([p + 3, s0, e0 if rng.random() < 0.5 else bar + 2 * step, v])
        notes.append([p + 7, s0 + step / 30, e0, v])
    if notes and rng.random() < 0.3:  # a duplicate pitch in a chord
        notes.append(list(notes[-1]))
    return notes


def cross_bar_cases(rng):
    recs = []
    for sig in SIGS:
        for beat in (0.5, 0.6):
            beats, division = _grid(beat, sig)
            name_to_time, time_to_name, times, bar = ref_encode.get_note_duration_dict(beat, sig)
            min_diff = name_to_time["sixteenth"] / 2
            for _ in range(10):
                raw = _cross_notes(rng, bar, int(rng.integers(1, 9)), beat / division)
                notes = [PlainNote(*x) for x in raw]
                ev, carry = ref_encode.bar_notes_to_event(notes, 0.0, bar, np.asarray(beats), time_to_name,
                                                          times, min_diff, grid_division=division)
                recs.append({"sig": list(sig), "beat": beat, "beats": beats, "division": division,
                             "min_diff": min_diff, "bar": float(bar), "notes": raw, "events": ev,
                             "carry": {str(p): [int(c.pitch), float(c.start), float(c.end), int(c.velocity)]
                                       for p, c in carry.items()}})
    assert sum(1 for r in recs if r["carry"]) >= len(recs) // 2
    return recs


if __name__ == "__main__":
    rng = np.random.default_rng(2024)
    out = {"to_category": to_category_cases(rng), "density": density_cases(rng),
           "durations": duration_cases(rng), "grid_notes": grid_cases(rng),
           "bar_notes_to_event": bar_event_cases(rng),
           "bar_notes_to_event_cross": cross_bar_cases(rng)}
    with open(os.path.join(OUT, "codec_golden.json"), "w") as f:
        json.dump(out, f)
    print("cases:", {k: len(v) if isinstance(v, list) else 1 for k, v in out.items()})
