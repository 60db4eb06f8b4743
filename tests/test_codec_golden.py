"""The codec's pure functions against the reference's
own `encode.py` outputs (tests/golden/make_golden_codec.py, run in the build
container with the absent MIDI libraries stubbed as empty modules).

Pinned here: `_category` (encode.py:206-210), `_density` (13-50),
`get_note_duration_dict` / `time2durations` (213-277, 947-954),
`_snap_to_grid` (900-936), `_note_tokens` (939-944) and `_bar_events`
(957-1141, bars whose notes end inside the bar, continued notes included)
and its cross-bar continuation branch (1028-1040, 1109-1121: a note running
past the bar line is cut there and carried to the next bar; the generator
records the reference's pretty_midi.Note objects with a stub class).
Still unpinned (they need pretty_midi objects the container lacks):
`event_2midi`, `midi_2event`,
`encode_midi` and the occupation / polyphony piano-roll statistics;
tests/test_codec.py checks those by properties."""
import json
import os

import numpy as np
import pytest

from smer_music_generation_amd import codec, durations, midi

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "codec_golden.json")))


def test_to_category():
    c = G["to_category"]
    assert codec._category(np.asarray(c["values"])) == c["out"]


@pytest.mark.parametrize("k", range(8))
def test_note_density(k):
    c = G["density"][k]
    total, per_bar = codec._density(c["tracks"], c["track_length"], c["total_length"])
    assert [float(x) for x in total] == c["total"]
    assert {t: [float(x) for x in v] for t, v in per_bar.items()} == c["per_bar"]
    # bar_track_density: one bar of track_0 at a time
    single = [codec._density({"t": [bar]}, c["track_length"], c["track_length"])[1]["t"][0]
              for bar in c["tracks"]["track_0"]]
    assert single == c["bar_track_density"]


@pytest.mark.parametrize("k", range(20))
def test_durations(k):
    c = G["durations"][k]
    n2t, t2n, times, bar = durations.get_note_duration_dict(c["beat"], tuple(c["sig"]))
    assert {a: float(b) for a, b in n2t.items()} == c["name_to_time"]
    assert [float(x) for x in times] == c["times"] and float(bar) == c["bar"]
    assert [durations.time2durations(p, t2n, times) for p in c["probes"]] == c["durations"]


def _notes(raw):
    return [midi.Note(v, p, s, e) for p, s, e, v in raw]


@pytest.mark.parametrize("k", range(32))
def test_grid_notes(k):
    c = G["grid_notes"][k]
    notes = _notes(c["notes"])
    codec._snap_to_grid(np.asarray(c["beats"]), notes, c["min_diff"], c["division"])
    assert [[float(n.start), float(n.end)] for n in notes] == c["out"]


@pytest.mark.parametrize("k", range(48))
def test_bar_notes_to_event(k):
    c = G["bar_notes_to_event"][k]
    _, t2n, times, bar = durations.get_note_duration_dict(c["beat"], tuple(c["sig"]))
    if c["note_to_event_name"] is not None:
        tok = codec._note_tokens(_notes(c["notes"][:1])[0], t2n, times)
        assert [tok[0], tok[1]] == c["note_to_event_name"]
    ev, carry = codec._bar_events(_notes(c["notes"]), 0.0, c["bar"], np.asarray(c["beats"]), t2n, times,
                                  c["min_diff"], c["division"])
    assert ev == c["events"]
    assert carry == {}


@pytest.mark.parametrize("k", range(len(G["bar_notes_to_event_cross"])))
def test_bar_notes_to_event_cross_bar(k):
    """Notes tied over the bar line (`encode.py:1028-1040,1109-1121`): the
    bar's events and the carried continuations (pitch, start = bar end, end,
    velocity -1) equal the reference's."""
    c = G["bar_notes_to_event_cross"][k]
    _, t2n, times, bar = durations.get_note_duration_dict(c["beat"], tuple(c["sig"]))
    ev, carry = codec._bar_events(_notes(c["notes"]), 0.0, c["bar"], np.asarray(c["beats"]), t2n, times,
                                  c["min_diff"], c["division"])
    assert ev == c["events"]
    got = {str(p): [int(n.pitch), float(n.start), float(n.end), int(n.velocity)] for p, n in carry.items()}
    assert got == c["carry"]
