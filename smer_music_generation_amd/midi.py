"""Minimal MIDI object model for the SMER codec.

The reference codec (`encode.py`) works on `pretty_midi` objects; pretty_midi
is not installed here, so this module supplies the subset the
codec touches, restating pretty_midi's published algorithms:

  * `Note`, `Instrument`, `TimeSignature`, `Lyric`, `PrettyMIDI` with one
    tempo (the SMER header carries a single tempo and time signature:
    `encode.py:1157-1190` rejects files with more);
  * `PrettyMIDI.get_beats` / `get_downbeats` (beats one period apart from 0,
    the last one at or past the end time dropped; a downbeat every numerator
    beats, every numerator / 3 beats in compound meters such as 6/8, where a
    beat is a dotted quarter: pretty_midi's `qpm_to_bpm`);
  * `get_piano_roll(fs)`: velocities summed over columns
    int(start * fs) .. int(end * fs) per note, width int(fs * end_time), drum
    tracks all zero; `get_end_time`;
  * `program_to_instrument_name` (the General MIDI program names);
  * Standard MIDI File I/O (`PrettyMIDI.write`, `read_midi`): format 1, one
    tempo track plus one track per instrument, times quantised to
    `resolution` ticks per quarter note.

Parity note: pretty_midi itself cannot run here, so these semantics are
pinned by their own tests (tests/test_codec.py), not by reference outputs
("parity unpinned").
"""
from __future__ import annotations

import struct

import numpy as np

GM_PROGRAM_NAMES = (
    "Acoustic Grand Piano", "Bright Acoustic Piano", "Electric Grand Piano", "Honky-tonk Piano",
    "Electric Piano 1", "Electric Piano 2", "Harpsichord", "Clavinet", "Celesta", "Glockenspiel",
    "Music Box", "Vibraphone", "Marimba", "Xylophone", "Tubular Bells", "Dulcimer", "Drawbar Organ",
    "Percussive Organ", "Rock Organ", "Church Organ", "Reed Organ", "Accordion", "Harmonica",
    "Tango Accordion", "Acoustic Guitar (nylon)", "Acoustic Guitar (steel)", "Electric Guitar (jazz)",
    "Electric Guitar (clean)", "Electric Guitar (muted)", "Overdriven Guitar", "Distortion Guitar",
    "Guitar Harmonics", "Acoustic Bass", "Electric Bass (finger)", "Electric Bass (pick)", "Fretless Bass",
    "Slap Bass 1", "Slap Bass 2", "Synth Bass 1", "Synth Bass 2", "Violin", "Viola", "Cello", "Contrabass",
    "Tremolo Strings", "Pizzicato Strings", "Orchestral Harp", "Timpani", "String Ensemble 1",
    "String Ensemble 2", "Synth Strings 1", "Synth Strings 2", "Choir Aahs", "Voice Oohs", "Synth Choir",
    "Orchestra Hit", "Trumpet", "Trombone", "Tuba", "Muted Trumpet", "French Horn", "Brass Section",
    "Synth Brass 1", "Synth Brass 2", "Soprano Sax", "Alto Sax", "Tenor Sax", "Baritone Sax", "Oboe",
    "English Horn", "Bassoon", "Clarinet", "Piccolo", "Flute", "Recorder", "Pan Flute", "Blown bottle",
    "Shakuhachi", "Whistle", "Ocarina", "Lead 1 (square)", "Lead 2 (sawtooth)", "Lead 3 (calliope)",
    "Lead 4 chiff", "Lead 5 (charang)", "Lead 6 (voice)", "Lead 7 (fifths)", "Lead 8 (bass + lead)",
    "Pad 1 (new age)", "Pad 2 (warm)", "Pad 3 (polysynth)", "Pad 4 (choir)", "Pad 5 (bowed)",
    "Pad 6 (metallic)", "Pad 7 (halo)", "Pad 8 (sweep)", "FX 1 (rain)", "FX 2 (soundtrack)",
    "FX 3 (crystal)", "FX 4 (atmosphere)", "FX 5 (brightness)", "FX 6 (goblins)", "FX 7 (echoes)",
    "FX 8 (sci-fi)", "Sitar", "Banjo", "Shamisen", "Koto", "Kalimba", "Bag pipe", "Fiddle", "Shanai",
    "Tinkle Bell", "Agogo", "Steel Drums", "Woodblock", "Taiko Drum", "Melodic Tom", "Synth Drum",
    "Reverse Cymbal", "Guitar Fret Noise", "Breath Noise", "Seashore", "Bird Tweet", "Telephone Ring",
    "Helicopter", "Applause", "Gunshot")


def program_to_instrument_name(program):
    if not 0 <= int(program) < 128:
        raise ValueError("program %d out of range" % program)
    return GM_PROGRAM_NAMES[int(program)]


class Note:
    __slots__ = ("velocity", "pitch", "start", "end")

    def __init__(self, velocity, pitch, start, end):
        self.velocity, self.pitch, self.start, self.end = velocity, pitch, start, end

    @property
    def duration(self):
        return self.end - self.start

    def __repr__(self):
        return "Note(start=%.6f, end=%.6f, pitch=%d, velocity=%d)" % (self.start, self.end, self.pitch,
                                                                      self.velocity)


class TimeSignature:
    __slots__ = ("numerator", "denominator", "time")

    def __init__(self, numerator, denominator, time):
        self.numerator, self.denominator, self.time = numerator, denominator, time


class Lyric:
    __slots__ = ("text", "time")

    def __init__(self, text, time):
        self.text, self.time = text, time


class Instrument:
    def __init__(self, program, is_drum=False, name=""):
        self.program, self.is_drum, self.name = int(program), bool(is_drum), name
        self.notes = []

    def get_end_time(self):
        return max((n.end for n in self.notes), default=0.0)

    def get_piano_roll(self, fs=100):
        """[128, int(fs * end)] velocity sums; all zero for a drum track."""
        if not self.notes:
            return np.zeros((128, 0))
        roll = np.zeros((128, int(fs * self.get_end_time())))
        if self.is_drum:
            return roll
        for n in self.notes:
            roll[n.pitch, int(n.start * fs):int(n.end * fs)] += n.velocity
        return roll


def _beat_period(tempo, numerator, denominator):
    """Seconds per beat: pretty_midi's qpm_to_bpm (compound meters count
    dotted quarters, 3/x counts the denominator note)."""
    if denominator in (1, 2, 4, 8, 16, 32):
        if numerator == 3:
            bpm = tempo * denominator / 4.0
        elif numerator % 3 == 0:
            bpm = tempo / 3.0 * denominator / 4.0
        else:
            bpm = tempo * denominator / 4.0
    else:
        bpm = tempo
    return 60.0 / bpm


class PrettyMIDI:
    """One tempo, time signatures at time 0 (all the SMER header encodes)."""

    def __init__(self, initial_tempo=120.0, resolution=220):
        self.initial_tempo = float(initial_tempo)
        self.resolution = int(resolution)
        self.instruments = []
        self.time_signature_changes = []
        self.lyrics = []

    def get_tempo_changes(self):
        return np.array([0.0]), np.array([self.initial_tempo])

    def get_end_time(self):
        times = [i.get_end_time() for i in self.instruments]
        times += [ts.time for ts in self.time_signature_changes] + [ly.time for ly in self.lyrics]
        times += [0.0]
        return max(times)

    def _ts(self):
        ts = self.time_signature_changes
        return (ts[0].numerator, ts[0].denominator) if ts else (4, 4)

    def get_beats(self, start_time=0.0):
        """Beats one period apart from start_time by repeated addition while
        the last is before the end time; that last one is dropped."""
        period = _beat_period(self.initial_tempo, *self._ts())
        end = self.get_end_time()
        beats = [start_time]
        while beats[-1] < end:
            beats.append(beats[-1] + period)
        return np.array(beats[:-1])

    def get_downbeats(self, start_time=0.0):
        beats = self.get_beats(start_time)
        num, _ = self._ts()
        step = num // 3 if (num % 3 == 0 and num != 3) else num
        down = beats[::step]
        return down[down >= start_time]

    def get_piano_roll(self, fs=100):
        if not self.instruments:
            return np.zeros((128, 0))
        rolls = [i.get_piano_roll(fs=fs) for i in self.instruments]
        out = np.zeros((128, max(r.shape[1] for r in rolls)))
        for r in rolls:
            out[:, :r.shape[1]] += r
        return out

    # ---- Standard MIDI File I/O ------------------------------------------
    def time_to_tick(self, t):
        return int(round(t * self.initial_tempo / 60.0 * self.resolution))

    def tick_to_time(self, tick):
        return tick * 60.0 / (self.initial_tempo * self.resolution)

    def write(self, path):
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    def to_bytes(self):
        def vlq(v):
            out = [v & 0x7F]
            v >>= 7
            while v:
                out.append(0x80 | (v & 0x7F))
                v >>= 7
            return bytes(reversed(out))

        def track(events):
            events.sort(key=lambda e: (e[0], e[1]))
            body, last = b"", 0
            for tick, _, data in events:
                body += vlq(tick - last) + data
                last = tick
            body += vlq(0) + b"\xff\x2f\x00"
            return b"MTrk" + struct.pack(">I", len(body)) + body

        tempo_us = int(round(60e6 / self.initial_tempo))
        meta = [(0, 0, b"\xff\x51\x03" + tempo_us.to_bytes(3, "big"))]
        for ts in self.time_signature_changes:
            dd = int(ts.denominator).bit_length() - 1
            meta.append((self.time_to_tick(ts.time), 1, bytes([0xFF, 0x58, 4, ts.numerator, dd, 24, 8])))
        for ly in self.lyrics:
            txt = ly.text.encode()
            meta.append((self.time_to_tick(ly.time), 2, b"\xff\x05" + vlq(len(txt)) + txt))
        chunks = [track(meta)]
        for k, inst in enumerate(self.instruments):
            ch = 9 if inst.is_drum else [c for c in range(16) if c != 9][k % 15]
            ev = [(0, 0, bytes([0xC0 | ch, inst.program & 0x7F]))]
            for n in inst.notes:
                # note-offs sort before note-ons at the same tick (key 1 < 2)
                ev.append((self.time_to_tick(n.start), 2, bytes([0x90 | ch, n.pitch & 0x7F, n.velocity & 0x7F])))
                ev.append((self.time_to_tick(n.end), 1, bytes([0x80 | ch, n.pitch & 0x7F, 0])))
            chunks.append(track(ev))
        header = b"MThd" + struct.pack(">IHHH", 6, 1, len(chunks), self.resolution)
        return header + b"".join(chunks)


def read_midi(path_or_bytes):
    """Standard MIDI File -> PrettyMIDI (first tempo and time signature;
    note-on with velocity 0 is a note-off; overlapping same-pitch notes end
    first-in-first-out)."""
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    if data[:4] != b"MThd":
        raise ValueError("not a Standard MIDI File")
    _, fmt, ntrk, div = struct.unpack(">IHHH", data[4:14])
    if div & 0x8000:
        raise ValueError("SMPTE time division is not supported")
    pos = 14
    tracks = []
    tempo, ts = 120.0, None
    for _ in range(ntrk):
        if data[pos:pos + 4] != b"MTrk":
            raise ValueError("bad track chunk")
        ln = struct.unpack(">I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + ln]
        pos += 8 + ln
        i, tick, status, evs = 0, 0, 0, []
        while i < len(body):
            d = 0
            while True:
                b = body[i]
                i += 1
                d = (d << 7) | (b & 0x7F)
                if not b & 0x80:
                    break
            tick += d
            b = body[i]
            if b & 0x80:
                status = b
                i += 1
            if status == 0xFF:
                typ = body[i]
                i += 1
                ln2 = 0
                while True:
                    c = body[i]
                    i += 1
                    ln2 = (ln2 << 7) | (c & 0x7F)
                    if not c & 0x80:
                        break
                payload = body[i:i + ln2]
                i += ln2
                if typ == 0x51 and tempo == 120.0:
                    tempo = 60e6 / int.from_bytes(payload, "big")
                elif typ == 0x58 and ts is None:
                    ts = (payload[0], 2 ** payload[1], tick)
            elif status in (0xF0, 0xF7):
                ln2 = 0
                while True:
                    c = body[i]
                    i += 1
                    ln2 = (ln2 << 7) | (c & 0x7F)
                    if not c & 0x80:
                        break
                i += ln2
            else:
                kind = status & 0xF0
                n = 1 if kind in (0xC0, 0xD0) else 2
                evs.append((tick, status, bytes(body[i:i + n])))
                i += n
        tracks.append(evs)
    pm = PrettyMIDI(initial_tempo=tempo, resolution=div)
    if ts is not None:
        pm.time_signature_changes = [TimeSignature(ts[0], ts[1], pm.tick_to_time(ts[2]))]
    for evs in tracks:
        insts = {}
        active = {}
        for tick, status, d in evs:
            ch, kind = status & 0x0F, status & 0xF0
            if kind == 0xC0:
                insts.setdefault(ch, Instrument(d[0], is_drum=ch == 9)).program = d[0]
            elif kind == 0x90 and d[1] > 0:
                insts.setdefault(ch, Instrument(0, is_drum=ch == 9))
                active.setdefault((ch, d[0]), []).append((tick, d[1]))
            elif kind in (0x80, 0x90):
                q = active.get((ch, d[0]))
                if q:
                    t0, vel = q.pop(0)
                    insts[ch].notes.append(Note(vel, d[0], pm.tick_to_time(t0), pm.tick_to_time(tick)))
        for ch in sorted(insts):
            insts[ch].notes.sort(key=lambda n: (n.start, n.end, n.pitch))
            pm.instruments.append(insts[ch])
    return pm
