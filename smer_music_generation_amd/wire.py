"""Host-side SMER event surgery around the infill decode (plugin wire surface).

Restates, with the same inputs/outputs:
* `mask_bar_and_track` (`generation.py:248-341`)
* `restore_marked_input` (`generation.py:417-465`)
* `fill_empty_bars` (`generation.py:230-245`)
* `change_controls` (`generation.py:698-877`)
* the `mask_target` list of `generation_all` (`generation.py:485-492`)

Lists are scanned once (O(n)) instead of the reference's repeated
`np.where`/`np.insert` passes; outputs are identical (pinned by
tests/golden/mask_bar_and_track.json and infill_micro.json).
"""
from __future__ import annotations

import operator
import re

import numpy as np

from .durations import time2durations

_TRACK_RE = re.compile(r'track_\d')
N_TRACK_CONTROLS = 3  # density, occupation, polyphony (generation.py:249)


def track_names_of(events):
    # the regex runs over the distinct tokens (a few hundred), not the song
    return sorted(t for t in set(events) if t.startswith('track_') and _TRACK_RE.match(t))


def bar_track_spans(events):
    """Per bar, the (first, end) body span of every track: first = index after
    the track token, end = index of the next track/bar token (or len).
    Same grouping as `generation.py:258-292`."""
    names = set(track_names_of(events))
    n_tracks = len(names)
    # positions of every 'bar' / track token: one C-level list.index scan
    # per head kind (a few hundred hits) instead of a Python pass per token
    seq = events if isinstance(events, list) else list(events)
    marks = []
    for head in names | {'bar'}:
        i = -1
        try:
            while True:
                i = seq.index(head, i + 1)
                marks.append(i)
        except ValueError:
            pass
    marks.sort()
    marks.append(len(events))
    out = []
    cur = []
    for i, pos in enumerate(marks[1:]):
        k = i % (n_tracks + 1)
        if k == 0:
            cur = [pos]
        else:
            cur.append(pos)
            if k == n_tracks:
                out.append([(cur[j] + 1, cur[j + 1]) for j in range(len(cur) - 1)])
    return out


def mask_bar_and_track(event, vocab, mask_tracks, mask_bars):
    """Replace each masked track body (notes) and each of its end controls
    (plus the bar's end tensile on the last track) by one `m_0`.
    Returns (src ids np.ndarray, mask_track_names, mask_bar_names)."""
    spans = bar_track_spans(event)
    tensile = set(vocab.name_to_tokens['tensile'])
    pairs = []
    mask_bar_names, mask_track_names = [], []
    for bar in mask_bars:
        for tpos, (a, b) in enumerate(spans[bar]):
            if tpos not in mask_tracks:
                continue
            mask_bar_names.append(bar)
            mask_track_names.append(tpos)
            tail = 1 if event[b - 1] in tensile else 0
            body_end = b - N_TRACK_CONTROLS - tail
            pairs.append((a + N_TRACK_CONTROLS, body_end))
            pairs.extend((body_end + i, body_end + i + 1) for i in range(N_TRACK_CONTROLS + tail))
    toks = list(event)
    for a, b in reversed(pairs):
        del toks[a:a + max(0, b - a)]
        toks.insert(a, 'm_0')
    return _to_ids(vocab, toks), mask_track_names, mask_bar_names


def _to_ids(vocab, toks):
    """np.array([vocab.char2index(t) for t in toks]); one dict lookup per
    token (char2index's per-call overhead dominated the host preparation)
    unless some token is unknown (then char2index itself, for its report)."""
    table = vocab._char2idx
    try:
        return np.array(list(map(table.__getitem__, toks)), dtype=np.int64)
    except KeyError:
        return np.array([vocab.char2index(t) for t in toks])


def decoder_targets(event, vocab, mask_tracks, mask_bars):
    """The decoder target stream `mask_bar_and_track` builds (and discards):
    per span [m_0, tokens..., <eos>] (`generation.py:321-327`)."""
    spans = bar_track_spans(event)
    tensile = set(vocab.name_to_tokens['tensile'])
    out = []
    for bar in mask_bars:
        for tpos, (a, b) in enumerate(spans[bar]):
            if tpos not in mask_tracks:
                continue
            tail = 1 if event[b - 1] in tensile else 0
            body_end = b - N_TRACK_CONTROLS - tail
            for lo, hi in [(a + N_TRACK_CONTROLS, body_end)] + \
                    [(body_end + i, body_end + i + 1) for i in range(N_TRACK_CONTROLS + tail)]:
                out.append(vocab.mask_indices[0])
                out.extend(vocab.char2index(t) for t in event[lo:hi])
                out.append(vocab.eos_index)
    return out


_FIRST9 = operator.itemgetter(slice(0, 9))


def restore_marked_input(src_token, generated_output):
    """Splice each generated span (the text between successive 'm_0' in
    `generated_output`) into the successive 'm_0' of `src_token`.  Returns a
    '<U9' array like the reference (tokens longer than 9 chars truncate).
    Raises IndexError when the source runs out of 'm_0' (reference behaviour
    of `np.where(...)[0][0]`)."""
    # (the reference's np.array(src_token) as '<U9': str() and truncation)
    if set(map(type, src_token)) <= {str}:
        src = list(map(_FIRST9, src_token))
    else:
        src = [str(t)[:9] for t in src_token]
    gen = [t if type(t) is str else str(t) for t in generated_output]
    starts = [i for i, t in enumerate(gen) if t == 'm_0']
    segs = []
    for j, s in enumerate(starts):
        e = starts[j + 1] if j + 1 < len(starts) else len(gen)
        segs.append(gen[s + 1:e])
    # the first len(segs) 'm_0' of the source take the spans, in order
    holes, at = [], 0
    for _ in segs:
        try:
            at = src.index('m_0', at)
        except ValueError:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0") from None
        holes.append(at)
        at += 1
    out, prev = [], 0
    for i, seg in zip(holes, segs):
        out += src[prev:i]
        out += seg
        prev = i + 1
    out += src[prev:]
    return np.array(out, dtype='<U9')


def fill_empty_bars(events, generate_bar_number, bar_duration, duration_time_to_name,
                    duration_times):
    """Append empty bars (`generation.py:230-245`); emits the reference's
    'a_0' placeholder (not a vocab token)."""
    fill = time2durations(bar_duration, duration_time_to_name, duration_times)
    n_tracks = len(track_names_of(events))
    for _ in range(generate_bar_number):
        events += ['bar', 's_2', 'a_0']
        for t in range(n_tracks):
            events += ['track_%d' % t, 'rest_e'] + list(fill)
    return events


def mask_targets(events, tracks_to_generate, bars_to_generate):
    """`generation.py:481-492`: per masked (bar, track) the control kinds
    r,d,o,p (+t for the last track).  Returns (mask_target, track positions)."""
    names = track_names_of(events)
    tracks = [names.index('track_%d' % t) for t in tracks_to_generate]
    target = []
    for _ in bars_to_generate:
        for t in tracks:
            target += ['r', 'd', 'o', 'p']
            if t == len(names) - 1:
                target.append('t')
    return target, tracks


def change_controls(original_event, controls):
    """Apply plugin control edits and copy bar/track controls to the end of
    each bar/track (`generation.py:698-877`)."""
    ev = original_event
    names = track_names_of(ev)
    n_tracks = len(names)
    bars = [i for i, t in enumerate(ev) if t == 'bar']
    head = ev[:bars[0]]
    dens = [t for t in head if re.match(r'd_\d', t)]
    poly = [t for t in head if re.match(r'y_\d', t)]
    occ = [t for t in head if re.match(r'o_\d', t)]

    def find_after(tok, start):
        for i in range(start, len(ev)):
            if ev[i] == tok:
                return i
        raise IndexError(tok)

    last = [-1, -1, -1]
    for t in range(n_tracks):
        cname = 'track_%s_c' % names[t][-1]
        pos = [find_after(dens[t], last[0] + 1), find_after(occ[t], last[1] + 1),
               find_after(poly[t], last[2] + 1)]
        last = pos
        ev[pos[0]] = 'd_%s' % controls[cname]["density"]
        ev[pos[2]] = 'y_%s' % controls[cname]["polyphony"]
        ev[pos[1]] = 'o_%s' % controls[cname]["occupation"]

    spans = bar_track_spans(ev)
    if controls['bar_track'] == 0:
        for b in range(len(bars)):
            for tpos, (a, _) in enumerate(spans[b]):
                for off, key, pre in ((0, 'bar_density', 'd'), (1, 'bar_occupation', 'o'),
                                      (2, 'bar_polyphony', 'y')):
                    val = controls[key][names[tpos]][b]
                    ev[a + off] = 'unk' if val == 10 else '%s_%s' % (pre, val)
    else:
        for b in range(len(bars)):
            if controls['s_bar'] <= b <= controls['e_bar']:
                for tpos, (a, _) in enumerate(spans[b]):
                    if controls[names[tpos]] == 0:
                        ev[a] = ev[a + 1] = ev[a + 2] = 'unk'

    # copy each bar's tensile to the bar end and each track's 3 controls to
    # the track end: one forward pass that rebuilds the list (O(n)); the
    # reference's backward walk of list inserts (O(n^2)) is kept only for an
    # event list whose bars do not each hold exactly n_tracks track tokens
    nameset = set(names)
    marks = sorted([i for i, t in enumerate(ev) if t in nameset] + bars)
    marks.append(len(ev))
    barset = set(bars)
    bar_idx = [k for k, p in enumerate(marks[:-1]) if p in barset]
    regular = all(k + n_tracks + 1 < len(marks) and
                  not any(marks[k + t] in barset for t in range(1, n_tracks + 1)) and
                  (k + n_tracks + 1 == len(marks) - 1 or marks[k + n_tracks + 1] in barset)
                  for k in bar_idx)
    if regular:
        out = ev[:marks[0]]
        for k in bar_idx:
            bar_pos = marks[k]
            out += ev[bar_pos:marks[k + 1]]
            for t in range(n_tracks):
                a, b = marks[k + t + 1], marks[k + t + 2]
                out += ev[a:b]
                out += ev[a + 1:a + N_TRACK_CONTROLS + 1]
            out.append(ev[bar_pos + 1])
        ev[:] = out
        return ev
    for bp in range(len(marks) - 1, -1, -1):
        if marks[bp] not in barset:
            continue
        bar_pos = marks[bp]
        next_bar = marks[bp + n_tracks + 1]
        ev.insert(next_bar, ev[bar_pos + 1])
        for t in range(n_tracks):
            start = marks[bp + t + 1] + N_TRACK_CONTROLS * t
            ins = marks[bp + t + 2] + N_TRACK_CONTROLS * t
            ctl = ev[start + 1:start + N_TRACK_CONTROLS + 1]
            for c in reversed(ctl):
                ev.insert(ins, c)
    return ev
