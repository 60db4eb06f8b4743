"""MIDI <-> SMER event codec of the plugin path.

The plugin hands the model a MIDI clip and reads one back:

    DAW notes --note_midi--> PrettyMIDI --encode_midi--> SMER events + controls
      --change_controls / generation_all (wire.py, generation.py)--> events
      --event_2midi--> PrettyMIDI --midi2notes--> DAW notes

This module restates the reference's codec functions on the `midi` object
model (pretty_midi is absent here):

  reference (`encode.py`)                          here
  note_midi                 83-133                 note_midi
  occupation_polyphony_rate 155-203                _occupation_polyphony
  note_density / to_category 27-50, 206-210        _density, _category
  event_2midi               297-534                event_2midi
  grid_notes                900-936                _snap_to_grid
  time2durations / note_to_event_name 939-954      durations.time2durations
  bar_notes_to_event        957-1141               _bar_events
  midi_2event               1144-1314              midi_2event
  remove_continue_add_control_event 559-804        _add_controls
  encode_midi               1376-1505              encode_midi (the infill path:
                                                   key and tensile strains given)
  midi2notes / merge_pm     1317-1373              midi2notes, merge_pm

The constants are `vocab_control.py`'s (tempo / control bins, velocities,
the pitch range, key tokens).  Tension and key detection (`cal_tension`,
`tension_calculation.py`, music21's key analysers: `encode.py:1395-1470`)
are data preparation, out of scope: `encode_midi` needs the
key and the per-bar tensile strains from the caller, as the plugin's infill
call supplies them (`encode.py:1387-1399`).

Parity: the reference codec cannot run here (it constructs pretty_midi
objects), so this restatement is pinned by its own property tests
(tests/test_codec.py: grammar round trips, control recomputation, SMF I/O)
and not by reference outputs: parity unpinned.
"""
from __future__ import annotations

import math
import re

import numpy as np

from . import midi
from .durations import get_note_duration_dict, time2durations

# vocab_control.py
TRACK_0_RANGE = (21, 108)
TIME_SIGNATURE_MAX_CHANGE = 1
V0, V1 = 120, 100
TEMPO_BINS = np.array([0, 60, 90, 120, 150, 180, 200])
CONTROL_BINS = np.arange(0, 1, 0.1)
ALL_KEY_NAMES = ['C major', 'G major', 'D major', 'A major', 'E major', 'B major', 'F major', 'B- major',
                 'E- major', 'A- major', 'D- major', 'G- major', 'A minor', 'E minor', 'B minor', 'F# minor',
                 'C# minor', 'G# minor', 'D minor', 'G minor', 'C minor', 'F minor', 'B- minor', 'E- minor']
KEY_TO_TOKEN = {name: "k_%d" % i for i, name in enumerate(ALL_KEY_NAMES)}
CONTROL_TOKENS = frozenset(["s_%d" % i for i in range(12)] + ["d_%d" % i for i in range(10)] +
                           ["o_%d" % i for i in range(10)] + ["y_%d" % i for i in range(10)])
SUPPORTED_SIGNATURES = ((4, 4), (2, 4), (3, 4), (6, 8))
_PROGRAM = re.compile(r"i_\d")
_TRACK = re.compile(r"track_\d")


def _category(values, bins=CONTROL_BINS):
    """Index of the last bin edge <= value (`encode.py:206-210`)."""
    return [int(np.where((v - bins) >= 0)[0][-1]) for v in values]


def _tempo_of_token(tok):
    """Tempo of a 't_k' header token: the bin's midpoint, the last bin's edge."""
    k = int(tok[2])
    return float(TEMPO_BINS[k]) if k == len(TEMPO_BINS) - 1 else (TEMPO_BINS[k] + TEMPO_BINS[k + 1]) / 2


# ----------------------------------------------------------------------------
# SMER events -> MIDI
# ----------------------------------------------------------------------------
class _Writer:
    """Cursor state of event_2midi's walk: the current track and time, the
    pending pitches and duration tokens of one note group."""

    def __init__(self, pm, dur):
        self.pm, self.dur = pm, dur
        self.track, self.time, self.prev = 0, 0.0, 0.0
        self.bar_time = 0.0
        self.pitches, self.durs = [], []
        self.sep = self.cont = False

    def flush(self):
        """Close the pending group: its notes start at the cursor (one group
        back after 'sep'), or extend the notes they continue; the cursor then
        moves by the group's duration."""
        length = 0
        for d in self.durs:
            length += self.dur[d]
        if self.sep:
            self.time -= self.prev
        notes = self.pm.instruments[self.track].notes
        for p in self.pitches:
            if self.cont:
                for n in reversed(notes):
                    if math.isclose(n.end, self.time) and n.pitch == p:
                        n.end += length
                        break
            else:
                notes.append(midi.Note(V0 if self.track == 0 else V1, p, self.time, self.time + length))
        self.time += length
        self.prev = length
        self.pitches, self.durs = [], []
        self.sep = self.cont = False


def event_2midi(event_list, tempo=None):
    """SMER events -> PrettyMIDI (`encode.py:297-534`); None when the events
    do not decode (the reference returns None from its catch-all)."""
    try:
        return _event_2midi(list(event_list), tempo)
    except Exception:  # noqa: BLE001  (the reference's bare except, encode.py:532)
        return None


def _event_2midi(events, tempo):
    events = [e for e in events if e not in CONTROL_TOKENS]
    if not tempo:
        tempo = _tempo_of_token(events[1]) if events[1][0] == "t" else float(events[1])
    pm = midi.PrettyMIDI(initial_tempo=tempo)
    num, den = (int(x) for x in events[0].split("/"))
    pm.time_signature_changes = [midi.TimeSignature(num, den, 0)]
    programs = [e for e in events if _PROGRAM.match(e)]
    track_names = sorted(set(e for e in events if _TRACK.match(e)))
    track_index = {name: i for i, name in enumerate(track_names)}
    first_bar = events.index("bar")
    for k, prog in enumerate(programs):
        inst = midi.Instrument(program=int(prog.split("_")[-1]))
        inst.is_drum = track_names[k] == "track_4"
        pm.instruments.append(inst)
    # the beat grid of a 10-second clip (first instrument carries a long
    # placeholder note while the beats are taken), then a 10 ms placeholder
    # note in every instrument (midi2notes skips them)
    beats = None
    for k, inst in enumerate(pm.instruments):
        inst.notes.append(midi.Note(100, 1, 0, 10))
        if k == 0:
            beats = pm.get_beats()
        inst.notes.pop()
        inst.notes.append(midi.Note(100, 1, 0, 0.01))
    dur, _, _, bar_duration = get_note_duration_dict(beats[1] - beats[0], (num, den))
    bar_positions = [i for i, e in enumerate(events) if e == "bar"]
    pm.lyrics = [midi.Lyric("test", len(bar_positions) * bar_duration)]
    w = _Writer(pm, dur)
    grouping = False
    bar_num = 0
    for i, ev in enumerate(events[first_bar:]):
        if ev in dur:
            w.durs.append(ev)
            grouping = True
            if w.track >= len(programs):
                raise IndexError("track without a program")
            continue
        if grouping:
            w.flush()
            grouping = False
        m = re.search(r"p_(\d+)", ev)
        if m:
            w.pitches.append(int(m.group(1)))
        if ev == "sep":
            w.sep = True
        # (the reference compares the offset from the first bar with an
        # absolute bar position)
        if ev == "continue" and i > bar_positions[1]:
            w.cont = True
        if ev == "bar":
            w.bar_time = bar_num * bar_duration
            bar_num += 1
            continue
        if _TRACK.search(ev):
            w.time, w.prev = w.bar_time, 0
            w.track = track_index[ev]
        if w.track >= len(programs):
            raise IndexError("track without a program")
    if grouping:
        w.flush()
    return pm


# ----------------------------------------------------------------------------
# MIDI -> SMER events
# ----------------------------------------------------------------------------
def _snap_to_grid(beat_times, notes, min_diff, division):
    """Quantise note starts / ends in place to `division` steps per beat
    (`encode.py:900-936`).  A note shorter than one step grows by one; a
    continued note (velocity -1) is clipped to the grid's end."""
    grid = []
    for a, b in zip(beat_times[:-1], beat_times[1:]):
        for j in range(division):
            grid.append((b - a) / division * j + a)
    grid.append(beat_times[-1])
    grid = np.array(grid)
    last = len(grid) - 1
    for n in notes:
        s = int(np.argmin(np.abs(n.start - grid)))
        if n.velocity == -1 and n.end > grid[-1]:
            n.end = grid[-1]
        if n.end < grid[-1] + min_diff:
            e = int(np.argmin(np.abs(n.end - grid)))
            if s == e:
                if e != last:
                    e += 1
                elif s != 0:
                    s -= 1
                else:
                    n.start = n.end = -1
                    continue
            n.start, n.end = grid[s], grid[e]
        else:
            n.start = grid[s]


def _note_tokens(note, t2n, times):
    return "p_%d" % note.pitch, time2durations(note.end - note.start, t2n, times)


class _BarEncoder:
    """One bar of one track -> events (`encode.py:957-1141`).  Notes are
    grouped into chords (same start and end within min_diff, or same start
    when both run past the bar); a chord becomes its pitches and one
    duration, continued notes first behind 'continue'; the gap to the next
    chord is a 'rest' (after the chord's end) or 'sep' + offset (before it);
    notes past the bar line are cut there and handed to the next bar as
    continuations (velocity -1)."""

    def __init__(self, bar_end, t2n, times, min_diff):
        self.bar_end, self.t2n, self.times, self.min_diff = bar_end, t2n, times, min_diff
        self.out = []
        self.carry = {}
        self.in_cont = False
        self.dur = None  # the last chord's duration tokens (the reference reuses them)
        self.last = None  # the last note handled

    def _ordered(self, chord):
        cont = sorted((n for n in chord if n.velocity == -1), key=lambda n: n.pitch)
        rest = sorted((n for n in chord if n.velocity != -1), key=lambda n: n.pitch)
        return cont + rest

    @staticmethod
    def _dedup(chord):
        drop = [i for i in range(len(chord) - 1) if chord[i].pitch == chord[i + 1].pitch]
        for i in reversed(drop):
            chord.pop(i)

    def emit_chord(self, chord, final):
        chord = self._ordered(chord)
        if final:
            chord.sort(key=lambda n: n.pitch)
        self._dedup(chord)
        pending = []
        for n in chord:
            if n.velocity == -1:
                if not self.in_cont:
                    pending.append("continue")
                    self.in_cont = True
            elif self.in_cont:
                self.out.extend(pending)
                self.out.extend(self.dur)
                self.out.append("sep")
                self.in_cont = False
                pending = []
            if n.end > self.bar_end:
                self.carry[n.pitch] = midi.Note(-1, n.pitch, self.bar_end, n.end)
                tok, self.dur = _note_tokens(midi.Note(n.velocity, n.pitch, n.start, self.bar_end),
                                             self.t2n, self.times)
            else:
                tok, self.dur = _note_tokens(n, self.t2n, self.times)
            pending.append(tok)
            self.last = n
        return chord, pending


def _bar_events(notes, bar_start, bar_end, beats, t2n, times, min_diff, division=4):
    enc = _BarEncoder(bar_end, t2n, times, min_diff)
    if notes:
        _snap_to_grid(beats, notes, min_diff, division)
        notes.sort(key=lambda n: (n.start, n.end, n.pitch))
        lead = time2durations(notes[0].start - bar_start, t2n, times)
    else:
        lead = time2durations(bar_end - bar_start, t2n, times)
    if lead:
        enc.out.append("rest")
        enc.out.extend(lead)
    chord = []
    for n in notes:
        if not chord:
            chord.append(n)
            continue
        prev = chord[-1]
        if n.end > bar_end and abs(n.start - prev.start) < min_diff and abs(bar_end - prev.end) < min_diff:
            chord.append(n)
        elif abs(n.start - prev.start) < min_diff and abs(n.end - prev.end) < min_diff:
            chord.append(n)
        else:
            chord, pending = enc.emit_chord(chord, final=False)
            enc.out.extend(pending)
            enc.out.extend(enc.dur)
            enc.in_cont = False
            if n.start >= chord[-1].end:
                gap = time2durations(n.start - chord[-1].end, t2n, times)
                if gap:
                    enc.out.append("rest")
                    enc.out.extend(gap)
            else:
                enc.out.append("sep")
                enc.out.extend(time2durations(n.start - chord[-1].start, t2n, times))
            chord = [n]
    chord, pending = enc.emit_chord(chord, final=True)
    if pending:
        enc.out.extend(pending)
        enc.out.extend(enc.dur)
    if chord and enc.last.end < bar_end:
        tail = time2durations(bar_end - enc.last.end, t2n, times)
        if tail:
            enc.out.append("rest")
            enc.out.extend(tail)
    return enc.out, enc.carry


def midi_2event(pm, track_names=()):
    """PrettyMIDI -> (events, pm (notes quantised in place), tempo) over the
    first 16 bars, padded with 'unk' rest bars to 16 (`encode.py:1144-1314`);
    None for unsupported time signatures."""
    beats = np.unique(pm.get_beats(), axis=0)
    ts0 = pm.time_signature_changes[0]
    num, den = ts0.numerator, ts0.denominator
    tempo = pm.get_tempo_changes()[1][0]
    downs = np.unique(pm.get_downbeats(), axis=0)
    beats_per_bar = int(4 * num / den)
    if len(downs) == 1:
        downs = np.array([0.0, 4 * tempo / 60 * den / num])
    if beats[-1] >= downs[-1]:
        downs = np.append(downs, downs[-1] + downs[-1] - downs[-2])
    guard = 0
    while not abs(downs[-1] - beats[-1]) < 0.0001:
        beats = np.append(beats, beats[-1] + beats[-1] - beats[-2])
        guard += 1
        if guard > 100000:
            raise ValueError("midi_2event: the beat grid never meets the last downbeat")
    downs = downs[:16]
    down_idx = [int(np.argmin(np.abs(beats - d))) for d in downs]
    sigs = [(s.numerator, s.denominator) for s in pm.time_signature_changes]
    if pm.time_signature_changes[0].time != 0 or len(sigs) > TIME_SIGNATURE_MAX_CHANGE:
        return None
    if any(s not in SUPPORTED_SIGNATURES for s in sigs):
        return None
    tempi = pm.get_tempo_changes()[1]
    division = 6 if sigs[0] == (6, 8) else 4
    n_tracks = len(pm.instruments)
    for inst in pm.instruments:
        inst.notes.sort(key=lambda n: n.start)
    carry = [{} for _ in range(n_tracks)]
    sig = sigs[0]
    events = ["%d/%d" % sig, "%s" % tempi[0]]
    tempo = tempi[0]
    events += ["i_%d" % inst.program for inst in pm.instruments]
    beat_len = None
    bar_duration = None
    t2n = times = None
    for bar, bar_time in enumerate(downs):
        events.append("bar")
        bp = down_idx[bar]
        if bp + 1 < len(beats):
            beat_len = beats[bp + 1] - beats[bp]
        dur, t2n, times, bar_duration = get_note_duration_dict(beat_len, sig)
        min_diff = dur["sixteenth"] / 2
        bar_end = downs[bar + 1] if bar + 1 < len(downs) else downs[bar] + bar_duration
        for t in range(n_tracks):
            events.append(track_names[t])
            notes = [n for n in pm.instruments[t].notes
                     if bar_time - min_diff <= n.start < bar_end - min_diff
                     and TRACK_0_RANGE[0] <= n.pitch <= TRACK_0_RANGE[1]]
            if not notes:
                events.append("rest")
                events.extend(time2durations(bar_duration, t2n, times))
                continue
            if bar == 15:
                bar_beats = beats[down_idx[bar]:down_idx[bar] + beats_per_bar + 1]
            else:
                bar_beats = beats[down_idx[bar]:down_idx[bar + 1] + 1]
            if carry[t]:
                notes = list(carry[t].values()) + notes
            bar_ev, carry[t] = _bar_events(notes, bar_time, bar_end, bar_beats, t2n, times, min_diff, division)
            events.extend(bar_ev)
    for _ in range(16 - len(downs)):
        events += ["bar", "unk"]
        for t in range(n_tracks):
            events += ["track_%d" % t, "rest"] + time2durations(bar_duration, t2n, times)
    return events, pm, tempo


# ----------------------------------------------------------------------------
# controls
# ----------------------------------------------------------------------------
def _density(track_bars, sixteenths_per_bar, total_sixteenths):
    """Per track: chords (pitch runs) per sixteenth over the clip and per bar
    (`encode.py:27-50`)."""
    total, per_bar = [], {}
    for name, bars in track_bars.items():
        count = 0
        per_bar[name] = []
        for ev in bars:
            n = sum(1 for a, b in zip(ev[:-1], ev[1:]) if a[0] == "p" and b[0] != "p")
            count += n
            per_bar[name].append(n / sixteenths_per_bar)
        total.append(count / total_sixteenths)
    return total, per_bar


def _occupation_polyphony(pm, bar_sixteenths, sixteenth, n_bars):
    """Per instrument: the fraction of sixteenth steps sounding, and of those
    the fraction with more than one pitch; over the clip and per bar
    (`encode.py:155-203`; drums are rolled as pitched notes here)."""
    occ, poly, bar_occ, bar_poly = [], [], {}, {}
    for k, inst in enumerate(pm.instruments):
        if inst.is_drum:
            probe = midi.Instrument(inst.program, is_drum=False)
            probe.notes = inst.notes
            inst = probe
        roll = inst.get_piano_roll(fs=1 / sixteenth)
        sounding = np.any(roll, 0)
        occ.append(0 if roll.shape[1] == 0 else np.count_nonzero(sounding) / (n_bars * bar_sixteenths))
        ns = np.count_nonzero(sounding)
        poly.append(0 if ns == 0 else np.count_nonzero(np.count_nonzero(roll, 0) > 1) / ns)
        bar_occ[k], bar_poly[k] = [], []
        for b in range(n_bars):
            if roll.shape[1] < b * bar_sixteenths:
                bar_occ[k].append(0)
                bar_poly[k].append(0)
                continue
            part = roll[:, b * bar_sixteenths:(b + 1) * bar_sixteenths]
            on = np.count_nonzero(np.any(part, 0))
            if on == 0:
                bar_poly[k].append(0)
                bar_occ[k].append(0)
            else:
                bar_occ[k].append(on / bar_sixteenths)
                bar_poly[k].append(np.count_nonzero(np.count_nonzero(part, 0) > 1) / on)
    return occ, poly, bar_occ, bar_poly


def _split_bars(events, bars, track_names):
    """{track: [the events of that track in each bar]}."""
    out = {t: [] for t in track_names}
    edges = list(bars) + [len(events)]
    for a, b in zip(edges[:-1], edges[1:]):
        bar_ev = events[a:b]
        pos = [bar_ev.index(t) for t in track_names] + [len(bar_ev)]
        for k, t in enumerate(track_names):
            out[t].append(bar_ev[pos[k]:pos[k + 1]] if k + 1 < len(track_names) else bar_ev[pos[k]:])
    return out


def _add_controls(body, header, key, tensiles, pm):
    """Drop first-bar 'continue's, prepend the header, then insert the key,
    the clip-level track controls (d_/o_/y_ per track), a tensile strain per
    bar and the per-bar-track d_/o_/y_ controls; also returns the controls
    dict the plugin shows (`encode.py:559-804`)."""
    n_tracks = len(header[2:])
    bar_pos = [i for i, e in enumerate(body) if e == "bar"]
    ev = [e for i, e in enumerate(body) if not (e == "continue" and i < bar_pos[1])]
    ev = [str(h) for h in header] + ev
    controls = {"time_signature": ev[0], "tempo": ev[1][-1], "key": key}
    if "_" not in ev[1]:
        ev[1] = "t_%d" % int(np.where((float(ev[1]) - TEMPO_BINS) >= 0)[0][-1])
        controls["tempo"] = ev[1][-1]
    bar_pos = [i for i, e in enumerate(ev) if e == "bar"]
    beats_in_bar = int(str(header[0])[0])
    bar_sixteenths = beats_in_bar * 4 if beats_in_bar != 6 else int(beats_in_bar / 2 * 4)
    total_sixteenths = bar_sixteenths * len(bar_pos)
    track_names = sorted(set(e for e in ev if _TRACK.match(e)))
    track_bars = _split_bars(ev, bar_pos, track_names)
    total_density, bar_density = _density(track_bars, bar_sixteenths, total_sixteenths)
    density_cat = _category(total_density)
    for t in bar_density:
        bar_density[t] = _category(bar_density[t])
    beat = pm.get_beats()
    sixteenth = (beat[1] - beat[0]) / (4 if int(header[0][0]) != 6 else 6)
    occ, poly, bar_occ, bar_poly = _occupation_polyphony(pm, bar_sixteenths, sixteenth, len(bar_pos))
    if (len(next(iter(bar_density.values()))) != len(bar_pos) or len(next(iter(bar_occ.values()))) != len(bar_pos)
            or len(next(iter(bar_poly.values()))) != len(bar_pos)):
        return None
    occ_cat, poly_cat = _category(occ), _category(poly)
    if not (len(density_cat) == len(occ_cat) == len(poly_cat) == len(track_names)):
        return None
    d_tok = ["d_%d" % c for c in density_cat]
    o_tok = ["o_%d" % c for c in occ_cat]
    y_tok = ["y_%d" % c for c in poly_cat]
    ev = ev[:2] + [KEY_TO_TOKEN[key]] + d_tok + o_tok + y_tok + ev[2:]
    if tensiles is not None:
        first = [i for i, e in enumerate(ev) if e == track_names[0]]
        if len(first) != len(bar_pos):
            raise AssertionError("one tensile strain per bar")
        for k, p in enumerate(first):
            ev.insert(p + k, "s_%s" % tensiles[k])
    for name in ("bar_density", "bar_occupation", "bar_polyphony"):
        controls[name] = {t: [] for t in track_names}
    for t in track_names:
        controls[t] = {"instrument": 10, "density": 10, "polyphony": 10, "occupation": 10}
    for k, t in enumerate(track_names):
        b_occ, b_poly = _category(bar_occ[k]), _category(bar_poly[k])
        spots = [i + 1 for i, e in enumerate(ev) if e == t]
        added = 0
        for i, p in enumerate(spots):
            # (the reference's density bound is '>', its other two '>=')
            dv = 0 if i > len(bar_density[t]) else bar_density[t][i]
            ov = 0 if i >= len(b_occ) else b_occ[i]
            yv = 0 if i >= len(b_poly) else b_poly[i]
            ev[p + added:p + added] = ["d_%d" % dv, "o_%d" % ov, "y_%d" % yv]
            added += 3
            controls["bar_density"][t].append(dv)
            controls["bar_occupation"][t].append(ov)
            controls["bar_polyphony"][t].append(yv)
    controls["track_nums"] = n_tracks
    for k, prog in enumerate(header[2:]):
        t = track_names[k]
        controls[t]["instrument"] = midi.program_to_instrument_name(int(str(prog)[2:]))
        controls[t]["density"] = int(d_tok[k][-1])
        controls[t]["polyphony"] = int(y_tok[k][-1])
        controls[t]["occupation"] = int(o_tok[k][-1])
    controls["tensile"] = tensiles
    controls["bar_nums"] = len(tensiles)
    return ev, controls


def encode_midi(pm, controls=None, infill=True, track_names=()):
    """PrettyMIDI -> (SMER events with controls, controls dict) for the
    plugin's infill call (`encode.py:1376-1505`): the first 16 bars, tempo
    binned, key token, tensile strain per bar (from controls['tensile']),
    clip- and bar-level density / occupation / polyphony per track.
    controls = {'key': name in ALL_KEY_NAMES, 'tensile': [int per bar]}."""
    controls = controls or {}
    key = controls.get("key")
    if not (key and key != "Not Set" and infill):
        raise NotImplementedError("encode_midi: tension / key detection (tension_calculation.py, music21) "
                                  "is data preparation, out of scope; pass controls={'key', 'tensile'}")
    tensiles = controls["tensile"]
    res = midi_2event(pm, track_names=list(track_names))
    if res is None:
        return None
    events, pm, tempo = res
    pm = event_2midi(events, tempo)
    if pm is None:
        return None
    n_tracks = sum(1 for e in events if _PROGRAM.match(e))
    if n_tracks < 1:
        return None
    events = list(events)
    events[1] = "t_%d" % int(np.where((float(events[1]) - TEMPO_BINS) >= 0)[0][-1])
    header = events[:2 + n_tracks]
    bar_pos = [i for i, e in enumerate(events) if e == "bar"]
    n_bars = min(len(tensiles), len(bar_pos))
    if n_bars > 16:
        n_bars = 16
        events = events[:bar_pos[16]]
    if n_bars < 16:
        events = events[:bar_pos[n_bars + 1]]
    bar_pos = bar_pos[:n_bars]
    return _add_controls(events[bar_pos[0]:], header, key, list(tensiles[:n_bars]), pm)


# ----------------------------------------------------------------------------
# DAW note lists
# ----------------------------------------------------------------------------
def note_midi(data, start_bar, total_tracks=5):
    """DAW clip dict -> PrettyMIDI (`encode.py:83-133`): data = {'tempo',
    'numerator', 'denominator', 'track_k': [[pitch, start_beat, beats], ...],
    'track_k_program': GM program + 1 (0 = absent)}; track 4 is the drums;
    times are shifted so that start_bar begins at 0."""
    tempo = data["tempo"]
    num, den = data["numerator"], data["denominator"]
    bar_time = 4 * 60 / tempo * num / den
    shift = (start_bar - 1) * bar_time
    beat = 60 / tempo
    pm = midi.PrettyMIDI(initial_tempo=tempo)
    pm.time_signature_changes = [midi.TimeSignature(num, den, 0)]
    for k in range(total_tracks):
        name = "track_%d" % k
        if name in data and data[name + "_program"] > 0:
            inst = midi.Instrument(program=data[name + "_program"] - 1, is_drum=k == 4)
            pm.instruments.append(inst)
            for nt in data[name]:
                if len(nt) == 3:
                    inst.notes.append(midi.Note(100, nt[0], nt[1] * beat - shift,
                                                nt[1] * beat + nt[2] * beat - shift))
            inst.notes.sort(key=lambda n: (n.start, n.end, n.pitch))
    return pm if pm.instruments else None


def midi2notes(pm, tempo, track_names, controls):
    """PrettyMIDI -> {track: [{'pitch', 'start_time', 'duration'} in beats]}
    for the tracks the request regenerated (controls[track] == 0) between
    bars s_bar .. e_bar, shifted back to the clip's start_bar
    (`encode.py:1317-1344`); event_2midi's placeholder notes are skipped."""
    out = {name: [] for name in track_names}
    start_bar = controls["start_bar"]
    s_bar = controls["s_bar"] - start_bar
    e_bar = controls["e_bar"] - start_bar + 1
    ts = pm.time_signature_changes[0]
    bar_beats = ts.numerator * 4 / ts.denominator
    shift = bar_beats * (start_bar - 1)
    beat = 60 / tempo
    for k, inst in enumerate(pm.instruments):
        name = track_names[k]
        if controls[name] != 0:
            continue
        for n in inst.notes:
            sb = n.start / beat
            if sb / bar_beats + 0.01 > s_bar and sb / bar_beats < e_bar:
                if n.pitch == 1 and n.duration < 0.02:
                    continue
                out[name].append({"pitch": n.pitch, "start_time": n.start / beat + shift,
                                  "duration": n.duration / beat})
    return out


def merge_pm(total_pm, partial_pm, controls, numerator, denominator, tempo):
    """Splice the regenerated bars of partial_pm into total_pm in place
    (`encode.py:1347-1373`): the target bars' notes (and placeholder notes)
    are cut from each track and partial_pm's notes there, shifted to the
    clip's start_bar, are added."""
    beat = 60 / tempo
    fill0 = beat * numerator * (controls["s_bar"] - 1)
    fill1 = beat * numerator * controls["e_bar"]
    shift = (controls["start_bar"] - 1) * beat * numerator
    for k, inst in enumerate(total_pm.instruments):
        cut = [i for i, n in enumerate(inst.notes) if n.pitch == 1 or (fill0 - 0.01 < n.start < fill1)]
        if cut:
            inst.notes = inst.notes[:cut[0]] + inst.notes[cut[-1] + 1:]
        for n in partial_pm.instruments[k].notes:
            n.start += shift
            n.end += shift
            if n.pitch != 1 and fill0 <= n.start < fill1:
                inst.notes.append(n)
        inst.notes.sort(key=lambda n: n.start)
    return total_pm
