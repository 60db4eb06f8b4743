"""Seeded synthetic SMER sequences (no MIDI corpus is available here).

Produces event lists in the plugin's bar-control-at-end layout (SURVEY.md
Appendix B; `encode.py:720-781` header/controls, `generation.py:842-875`
control copy to the track/bar end) and span-masked training batches shaped
like `dataset.py:702-730` (per span: decoder_in = [m_0, tok...],
decoder_target = [tok..., <eos>]) collated like `dataset.py:802-862`.
"""
from __future__ import annotations

import numpy as np

from .durations import get_note_duration_dict

_DUR_NAMES_44 = ["quarter", "eighth", "half", "sixteenth", "quarter_eighth", "half_quarter",
                 "eighth_sixteenth", "whole"]


def _bar_notes(rng, sixteenths, allow_whole):
    """One track's notes for one bar, following the note grammar of
    `encode.py:957-1141`: `rest <dur>`, `[continue p.. <dur> sep] p.. <dur>`."""
    out = []
    left = sixteenths
    sizes = {"whole": 16, "half": 8, "quarter": 4, "eighth": 2, "sixteenth": 1}
    first = True
    while left > 0:
        cands = [n for n in _DUR_NAMES_44 if sum(sizes[p] for p in n.split("_")) <= left
                 and (allow_whole or "whole" not in n)]
        name = cands[int(rng.integers(len(cands)))]
        dur = name.split("_")
        left -= sum(sizes[p] for p in dur)
        r = rng.random()
        if r < 0.2:
            out.append("rest")
        elif first and r < 0.3:
            out.append("continue")
            out.append("p_%d" % int(rng.integers(40, 90)))
            out.extend(dur)
            out.append("sep")
            for _ in range(int(rng.integers(1, 3))):
                out.append("p_%d" % int(rng.integers(40, 90)))
        else:
            for _ in range(int(rng.integers(1, 4))):
                out.append("p_%d" % int(rng.integers(21, 109)))
        out.extend(dur)
        first = False
    return out


def synth_events(seed, n_bars=4, n_tracks=2, time_signature="4/4", copy_controls=True):
    """A plugin-format SMER event list (strings).  copy_controls=False gives
    the encoder's layout before `change_controls` (generation.py:698-877)
    copies each track's controls to the track end and the bar's tensile to
    the bar end."""
    rng = np.random.default_rng(seed)
    num, den = int(time_signature[0]), int(time_signature[2])
    sixteenths = num * (4 if den == 4 else 2)
    allow_whole = den == 4 and num >= 4
    ev = [time_signature, "t_%d" % int(rng.integers(7)), "k_%d" % int(rng.integers(24))]
    ev += ["d_%d" % int(rng.integers(10)) for _ in range(n_tracks)]
    ev += ["o_%d" % int(rng.integers(10)) for _ in range(n_tracks)]
    ev += ["y_%d" % int(rng.integers(10)) for _ in range(n_tracks)]
    ev += ["i_%d" % int(rng.integers(128)) for _ in range(n_tracks)]
    for _ in range(n_bars):
        tens = "s_%d" % int(rng.integers(12))
        ev += ["bar", tens]
        for t in range(n_tracks):
            ctl = ["d_%d" % int(rng.integers(10)), "o_%d" % int(rng.integers(10)),
                   "y_%d" % int(rng.integers(10))]
            ev += ["track_%d" % t] + ctl + _bar_notes(rng, sixteenths, allow_whole)
            if copy_controls:
                ev += ctl
        if copy_controls:
            ev.append(tens)
    return ev


def _track_spans(events):
    """(start, end) of every bar x track body, exclusive of the track name."""
    spans = []
    n = len(events)
    i = 0
    while i < n:
        if events[i].startswith("track_"):
            j = i + 1
            while j < n and not (events[j].startswith("track_") or events[j] == "bar"):
                j += 1
            spans.append((i + 1, j))
            i = j
        else:
            i += 1
    return spans


def synth_training_example(rng, vocab, S, T, n_tracks=3):
    """One (src[S], tgt_in[T], tgt_out[T]) example: note spans of random
    bar x tracks plus their end controls become single m_0 tokens."""
    events = synth_events(int(rng.integers(1 << 30)), n_bars=max(4, S // 40 + 2), n_tracks=n_tracks)
    spans = _track_spans(events)
    order = rng.permutation(len(spans))
    masked = []
    dec_len = 0
    for k in order:
        a, b = spans[k]
        body = (a + 3, b - 3 - (1 if events[b - 1].startswith("s_") else 0))
        if body[0] >= body[1] or body[1] > S:
            continue
        pieces = [body] + [(body[1] + i, body[1] + i + 1) for i in range(3)]
        cost = sum(p[1] - p[0] + 1 for p in pieces)
        if dec_len + cost > T and masked:
            break
        masked.extend(pieces)
        dec_len += cost
    masked.sort()
    dec_in, dec_out = [], []
    for a, b in masked:
        dec_in.append(vocab.mask_indices[0])
        for tok in events[a:b]:
            dec_in.append(vocab.char2index(tok))
            dec_out.append(vocab.char2index(tok))
        dec_out.append(vocab.eos_index)
    src_ev = list(events)
    for a, b in masked[::-1]:
        del src_ev[a:b]
        src_ev.insert(a, "m_0")
    src = np.array([vocab.char2index(t) for t in src_ev], dtype=np.int64)

    def fit(x, L):
        x = np.asarray(x, dtype=np.int64)[:L]
        return np.pad(x, (0, L - len(x)))

    return fit(src, S), fit(dec_in, T), fit(dec_out, T)


def synth_training_batch(seed, vocab, B, S, T, n_tracks=3):
    """Collated batch like `collate_mlm_*` (`dataset.py:802-925`): int64 ids
    plus bool key-padding masks (`x == 0`)."""
    rng = np.random.default_rng(seed)
    ex = [synth_training_example(rng, vocab, S, T, n_tracks) for _ in range(B)]
    src = np.stack([e[0] for e in ex])
    tin = np.stack([e[1] for e in ex])
    tout = np.stack([e[2] for e in ex])
    return {"input": src, "target_in": tin, "target_out": tout,
            "input_pad_mask": src == 0, "target_pad_mask": tin == 0}
