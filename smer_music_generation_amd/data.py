"""SMER training-data pipeline: token-budget packing of
songs into groups and the dataset that masks them for pretraining / bar
infilling, with the reference's surface and random streams.

Reference: `stack_batches` (load_dataset.py:167-289),
`ParallelLanguageDataset` (dataset.py:12-164, `random_word` 166-311,
`mask_bars` 314-777) and `collate_mlm_pretraining` / `_finetuning`
(dataset.py:802-925).  Same constructor arguments, same item format (three
lists of int64 arrays: encoder tokens, decoder input, decoder target), same
in-place effects on the stored groups, and the same draws from Python's
`random` and numpy's global `np.random` in the same order, so a seeded run
reproduces the reference's batches exactly (pinned by
tests/golden/data_golden.npz, generated from the reference itself).

What is different is the cost: the reference spends ~O(vocab) per token
(list membership tests) and a Python loop iteration per token; here the
pretraining inner loop (control corruption + span masking, one or two
random() draws per token) runs natively in `libsmer_data.so`
(csrc/dataset.cpp) on token ids with a replica of CPython's MT19937 — the
generator state is handed over and back, so the Python-side draws before
and after continue the same stream — and the per-token bookkeeping of bar
masking is numpy.
"""
from __future__ import annotations

import ctypes
import os
import random
import re

import numpy as np
import torch

from .generation import gen_nopeek_mask  # noqa: F401  (dataset.py:786-799 re-export)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsmer_data.so")
_lib = None

_TRACK_RE = re.compile(r"track_\d")
_PROGRAM_RE = re.compile(r"i_\d")


def _native():
    """libsmer_data.so (host code, built by csrc/build.py); raises if absent:
    there is no pure-Python fallback on the product path."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError("libsmer_data.so not built (run smer_music_generation_amd/csrc/build.py)")
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        lib.smer_span_mask.restype = ctypes.c_int
        lib.smer_span_mask.argtypes = [P, ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_double, ctypes.c_double, P, P, P, P]
        lib.smer_mt_random.restype = None
        lib.smer_mt_random.argtypes = [P, ctypes.c_int, P]
        _lib = lib
    return _lib


def _ptr(a):
    return a.ctypes.data


def _mt_get():
    """CPython random's MT19937 state as 625 uint32 (624 words + index)."""
    st = random.getstate()
    return np.array(st[1], dtype=np.uint32), st


def _mt_set(arr, st):
    random.setstate((st[0], tuple(arr.tolist()), st[2]))


def mt_random(n):
    """n draws of random.random() through the native generator (advances the
    module's stream exactly as n calls of random.random() would)."""
    mt, st = _mt_get()
    out = np.empty(n, dtype=np.float64)
    _native().smer_mt_random(_ptr(mt), int(n), _ptr(out))
    _mt_set(mt, st)
    return out


# ---------------------------------------------------------------------------
# token-budget packing (load_dataset.py:167-289)
# ---------------------------------------------------------------------------
def stack_batches(files, max_token_length=2200, augment=False, add_control=False, rest_multi=True,
                  test_dataset=False, loader=None, logger=None):
    """Songs -> groups of songs whose summed length stays below
    max_token_length, plus {group size: [group indices]}.

    `files`: paths (each unpickled by `loader`, default pickle — only for
    files your own pipeline wrote) or already-loaded per-file event lists.
    Songs are sorted by length (stable), adjacent duplicates dropped, then
    packed greedily in that order; a song longer than the budget is skipped
    and, as in the reference, resets the running length without opening a
    new group (the next song joins the previous group)."""
    random.seed(99)  # load_dataset.py:175 (no draws follow; kept for the stream)
    per_file = []
    for f in files:
        if isinstance(f, (str, os.PathLike)):
            if loader is None:
                import pickle
                with open(f, "rb") as fh:
                    events = pickle.load(fh)
            else:
                events = loader(f)
        else:
            events = f
        per_file.append(events)
    if test_dataset:
        return per_file, None

    songs = [ev for events in per_file if events for ev in events]
    songs.sort(key=len)
    uniq = []
    for ev in songs:  # adjacent duplicates (np.array_equal on the sorted list)
        if uniq and len(uniq[-1]) == len(ev) and list(uniq[-1]) == list(ev):
            continue
        uniq.append(ev)

    groups = []
    running = 0
    for ev in uniq:
        n = len(ev)
        if running + n < max_token_length:
            if groups:
                groups[-1].append(ev)
            else:
                groups.append([ev])
            running += n
        elif n > max_token_length:
            if logger is not None:
                logger.info("the event size %d is greater than %d, skip this file, or increase the "
                            "max token length" % (n, max_token_length))
            running = 0
        else:
            groups.append([ev])
            running = n
    lengths = {}
    for i, g in enumerate(groups):
        lengths.setdefault(len(g), []).append(i)
    return groups, lengths


# ---------------------------------------------------------------------------
# dataset (dataset.py:12-777)
# ---------------------------------------------------------------------------
class ParallelLanguageDataset(torch.utils.data.Dataset):
    """Masked-span (pretraining) / masked-bar (finetuning) items over packed
    song groups; constructor as dataset.py:13-23."""

    def __init__(self, vocab, batches, batch_lengths, batch_size, total_mask_ratio, logger,
                 pretraining=True, verbose=False, bar_track_control=False, bar_control_at_end=False):
        random.seed(99)
        self.vocab = vocab
        self.batch_size = batch_size
        self.verbose = verbose
        self.logger = logger
        self.batches = batches
        self.batch_lengths = batch_lengths
        self.total_mask_ratio = total_mask_ratio
        self.previous_index = 0
        self.pretraining = pretraining
        self.bar_track_control = bar_track_control
        self.bar_control_at_end = bar_control_at_end
        kinds = set(vocab.token_class_ranges.values())
        self.total_track_control_types = sum(k in kinds for k in ("density", "occupation", "polyphony"))
        self.tension_control = "tensile" in kinds
        self.len = len(batches)

        self._keep = set(vocab.control_tokens) | set(vocab.basic_tokens)
        self._controls = set(vocab.control_tokens)
        self._c2i = dict(vocab._char2idx)
        V = vocab.vocab_size
        self._cls = np.zeros(V, dtype=np.uint8)
        for tok, i in self._c2i.items():
            if tok in self._controls:
                self._cls[i] |= 1
            if tok == "bar" or _TRACK_RE.match(tok):
                self._cls[i] |= 2
        self._is_tensile = np.zeros(V, dtype=bool)
        self._is_tensile[[self._c2i[t] for t in vocab.name_to_tokens.get("tensile", ())]] = True
        self._is_prog = np.array([bool(_PROGRAM_RE.match(vocab.index2char(i) or "")) for i in range(V)])
        self._bar_id = self._c2i["bar"]
        self._unk_id = self._c2i[vocab.corrupt_tokens[0]]
        # the mask token inserted in the encoder copy is vocab.mask[0] = 'm_0'
        # (dataset.py:728 uses the module's list), i.e. mask_indices[0]
        self._filtered = {}     # id(event) -> length after filtering (filtering is idempotent)
        self._ids = {}          # id(event) -> (length, int32 ids) once filtered / completed

    def __len__(self):
        return self.len

    # ---- item selection, filtering, control copy (dataset.py:59-161) ----
    def __getitem__(self, idx):
        if self.batch_lengths == 0:
            return_idx = idx
        else:
            if idx % self.batch_size == 0:
                this_idx = random.randint(0, len(self.batches) - 1)
                if this_idx + self.batch_size - 1 > len(self.batches) - 1:
                    this_idx = this_idx - self.batch_size + 1
                self.previous_index = this_idx
            else:
                self.previous_index += 1
                this_idx = self.previous_index
            if this_idx > len(self.batches) - 1:
                print(f'invalid this index {this_idx}')
                print(f'idx is {idx}')
                this_idx = len(self.batches) - 1
            return_idx = random.choice(self.batch_lengths[len(self.batches[this_idx])])
        group = self.batches[return_idx]

        keep = self._keep
        for ev in group:
            if self._filtered.get(id(ev)) != len(ev):
                if any(t not in keep for t in ev):
                    ev[:] = [t for t in ev if t in keep]
                self._filtered[id(ev)] = len(ev)

        if self.bar_track_control and self.bar_control_at_end:
            self._copy_controls_to_ends(group)

        if self.pretraining:
            return self.random_word(group, self.total_mask_ratio)
        return self.mask_bars(group)

    def _copy_controls_to_ends(self, group):
        """dataset.py:102-153: copy each track's controls to the track end and
        the bar's tensile to the bar end, in place, once per song (a song
        already ending in a control is left alone).  The program-count regex
        is swapped for the track regex after the first song of the group, as
        in the reference."""
        ctl = self._controls
        ntc = self.total_track_control_types
        for k, ev in enumerate(group):
            if ev[-1] in ctl:
                continue
            regex = _PROGRAM_RE if k == 0 else _TRACK_RE
            track_nums = len(set(filter(regex.match, ev)))
            names = sorted(set(filter(_TRACK_RE.match, ev)))
            bar_poses = [i for i, t in enumerate(ev) if t == "bar"]
            marks = sorted([i for i, t in enumerate(ev) if t in names] + bar_poses)
            marks.append(len(ev))
            bar_set = set(bar_poses)
            for back in range(len(marks) - 1, -1, -1):
                if marks[back] not in bar_set:
                    continue
                bar_pos = marks[back]
                if back + track_nums + 1 >= len(marks):
                    print(back + track_nums + 1)
                next_bar = marks[back + track_nums + 1]
                if self.tension_control:
                    ev.insert(next_bar, ev[bar_pos + 1])
                if ntc > 0:
                    for tn in range(track_nums):
                        start = marks[back + tn + 1] + ntc * tn
                        at = marks[back + tn + 2] + ntc * tn
                        for c in ev[start + 1:start + ntc + 1][::-1]:
                            ev.insert(at, c)
            self._filtered[id(ev)] = len(ev)

    def _encode(self, ev, seq):
        """int32 ids of a stored song, cached per song object (its tokens only
        change through the filtering / control copy above, which both change
        its length)."""
        hit = self._ids.get(id(ev))
        if hit is not None and hit[0] == len(seq) and hit[2] is ev:
            return hit[1]
        c2i = self._c2i
        arr = np.fromiter((c2i[t] for t in seq), dtype=np.int32, count=len(seq))
        self._ids[id(ev)] = (len(seq), arr, ev)
        return arr

    # ---- pretraining: span masking (dataset.py:166-311) ----
    def random_word(self, events, total_ratio):
        span_lengths = [3, 1, 2]
        span_ratio = [.5, .25, .25]
        thr15 = float(total_ratio / np.dot(span_ratio, span_lengths)) * 1.5
        random.shuffle(events)
        seqs = [ev if isinstance(ev, list) else ev.tolist() for ev in events]
        enc = [self._encode(ev, s) for ev, s in zip(events, seqs)]
        n = [len(e) for e in enc]
        off = np.zeros(len(seqs) + 1, dtype=np.int64)
        np.cumsum(n, out=off[1:])
        total = int(off[-1])
        ids = np.concatenate(enc) if enc else np.zeros(0, dtype=np.int32)
        c2i = self._c2i
        tokens = np.empty(max(total, 1), dtype=np.int32)
        dec_in = np.empty(max(2 * total, 1), dtype=np.int32)
        dec_tgt = np.empty(max(2 * total, 1), dtype=np.int32)
        lens = np.zeros(3 * max(len(seqs), 1), dtype=np.int64)
        mode = 1 if (self.bar_track_control and self.bar_control_at_end) else 0
        mt, st = _mt_get()
        rc = _native().smer_span_mask(
            _ptr(mt), len(seqs), _ptr(ids), _ptr(off), _ptr(self._cls), len(self._cls), mode,
            c2i[self.vocab.corrupt_tokens[0]], self.vocab.mask_indices[0], self.vocab.eos_index,
            float(total_ratio), thr15, _ptr(tokens), _ptr(dec_in), _ptr(dec_tgt), _ptr(lens))
        if rc != 0:
            raise ValueError("smer_span_mask: token id outside the vocabulary")
        _mt_set(mt, st)
        out_t, out_i, out_o = [], [], []
        a = b = c = 0
        for e in range(len(seqs)):
            kt, ki, ko = (int(v) for v in lens[3 * e:3 * e + 3])
            if ki > 0:
                out_t.append(tokens[a:a + kt].astype(np.int64))
                out_i.append(dec_in[b:b + ki].astype(np.int64))
                out_o.append(dec_tgt[c:c + ko].astype(np.int64))
            a, b, c = a + kt, b + ki, c + ko
        return out_t, out_i, out_o

    def _bar_tracks(self, ids):
        """Per bar, the (start, end) of every track body (after the track
        name, up to the next track / bar token), dataset.py:363-400; on ids:
        the marks are the track-name and bar positions."""
        cls = self._cls[ids]
        bar_poses = np.flatnonzero(ids == self._bar_id)
        track_nums = int(np.count_nonzero(self._is_prog[ids]))
        marks = np.flatnonzero(cls & 2).tolist()
        marks.append(len(ids))
        bars = []
        cur = pairs = None
        for i, pos in enumerate(marks[1:]):
            if i % (track_nums + 1) == 0:
                cur, pairs = [pos], []
            else:
                cur.append(pos)
                if i % (track_nums + 1) == track_nums:
                    for j in range(len(cur) - 1):
                        pairs.append((cur[j] + 1, cur[j + 1]))
                    bars.append(pairs)
        return bar_poses, track_nums, bars

    def _span(self, ids, track_start, track_end):
        """The masked body of one track and, with controls at the end, the
        single-token pairs of the trailing controls (dataset.py:433-455)."""
        out = []
        tensile_end = 0
        if self.bar_track_control:
            token_start = track_start + self.total_track_control_types
            if self.bar_control_at_end:
                if self.tension_control and self._is_tensile[ids[track_end - 1]]:
                    tensile_end = 1
                token_end = track_end - self.total_track_control_types - tensile_end
            else:
                token_end = track_end
        else:
            token_start, token_end = track_start, track_end
        out.append((token_start, token_end))
        if self.bar_control_at_end:
            for i in range(self.total_track_control_types + tensile_end):
                out.append((token_end + i, token_end + 1 + i))
        return out

    def _corrupt_track_controls(self, ids, track_start):
        """10 / 10 / 10 % one / two / three track controls -> unk (3 control
        types), 10 % the single one (1 type): dataset.py:459-493."""
        unk = self._unk_id
        if self.total_track_control_types == 3:
            p = random.random()
            idxs = ()
            if 0.2 < p < 0.3:
                idxs = np.sort(np.random.choice(range(3), 1, replace=False))
            if 0.1 < p < 0.2:
                idxs = np.sort(np.random.choice(range(3), 2, replace=False))
            if p < 0.1:
                idxs = range(3)
            for k in idxs:
                ids[track_start + k] = unk
        elif self.total_track_control_types == 1:
            p = random.random()
            if 0.2 < p < 0.3:
                ids[track_start] = unk

    # ---- finetuning: bar / track masking (dataset.py:314-777) ----
    def mask_bars(self, events):
        random.shuffle(events)
        p = random.random()
        mask_mode = 0 if p > 0.6 else (1 if .3 < p <= 0.6 else 2)
        mask_id = self.vocab.mask_indices[0]
        eos = self.vocab.eos_index
        unk = self._unk_id
        out_t, out_i, out_o = [], [], []
        weight = None  # (the reference's `weight` survives from song to song)
        for event in events:
            seq = event if isinstance(event, list) else event.tolist()
            ids = self._encode(event, seq).astype(np.int64)  # the song copy (corrupted in place)
            bar_poses, track_nums, bars = self._bar_tracks(ids)
            pairs = []
            if mask_mode == 0:
                w_bars = np.logspace(1, 2, num=len(bar_poses))[::-1]
                n_bars = random.choices(range(len(bar_poses)), weights=w_bars)[0] + 1
                chosen = np.sort(np.random.choice(len(bar_poses), size=n_bars, replace=False))
                for b in chosen:
                    bar_pairs = []
                    weight = {1: [1], 2: [10, 1], 3: [10, 5, 1], 4: [10, 5, 3, 1],
                              5: [10, 5, 3, 2, 1]}.get(track_nums, weight)
                    if weight is None:
                        raise NameError("weight: no track-count weights for %d tracks" % track_nums)
                    if len(range(track_nums)) != len(weight):
                        print('what')
                        print(range(track_nums))
                        print(weight)
                    n_tr = random.choices(range(track_nums), weights=weight)[0] + 1
                    tracks = np.sort(np.random.choice(track_nums, size=n_tr, replace=False))
                    for t in tracks:
                        s, e = bars[b][t]
                        bar_pairs.extend(self._span(ids, s, e))
                        if self.bar_track_control:
                            self._corrupt_track_controls(ids, s)
                    pairs.extend(bar_pairs)
            elif mask_mode == 1:
                weight = {1: [1], 2: [10, 1], 3: [10, 2, 1]}.get(track_nums, weight)
                if weight is None:
                    raise NameError("weight: no track-count weights for %d tracks" % track_nums)
                n_tr = random.choices(range(track_nums), weights=weight)[0] + 1
                tracks = np.sort(np.random.choice(track_nums, size=n_tr, replace=False))
                tset = set(int(t) for t in tracks)
                for bar in bars:
                    for t, (s, e) in enumerate(bar):
                        if t in tset:
                            pairs.extend(self._span(ids, s, e))
                if self.bar_track_control:
                    if random.random() > 0.5:
                        n_bars = len(bar_poses)
                    else:
                        n_bars = np.random.randint(len(bar_poses))
                    chosen = np.sort(np.random.choice(len(bar_poses), size=n_bars, replace=False))
                    if self.total_track_control_types == 3:
                        q = random.random()
                        if q > 0.6:
                            idxs = np.sort(np.random.choice(range(3), 1, replace=False))
                        elif .35 < q <= 0.6:
                            idxs = np.sort(np.random.choice(range(3), 2, replace=False))
                        elif .25 < q <= .35:
                            idxs = range(3)
                        else:
                            idxs = []
                    else:
                        idxs = [0] if random.random() > 0.5 else []
                    cset = set(int(b) for b in chosen)
                    for bn, bar in enumerate(bars):
                        if bn in cset:
                            for t, (s, e) in enumerate(bar):
                                if t in tset:
                                    for k in idxs:
                                        ids[s + k] = unk
            else:
                w_bars = np.logspace(1, 2, num=len(bar_poses))[::-1]
                n_bars = random.choices(range(len(bar_poses)), weights=w_bars)[0] + 1
                if random.random() > .5:
                    first = np.random.randint(0, len(bar_poses) - (n_bars - 1))
                    chosen = range(first, first + n_bars)
                else:
                    chosen = np.sort(np.random.choice(len(bar_poses), size=n_bars, replace=False))
                for b in chosen:
                    bar = bars[b]
                    for s, e in bar:
                        pairs.extend(self._span(ids, s, e))
                        if self.bar_track_control:
                            self._corrupt_track_controls(ids, s)
                    if self.tension_control and random.random() < .1:
                        ids[bar[0][0] - 2] = unk

            if not pairs:
                continue
            # decoder sequences in pair order: [mask, span...] / [span..., eos]
            # (dataset.py:706-719); the encoder copy with every pair replaced by
            # one mask token, applied from the last pair by position (720-731)
            d_in, d_out = [], []
            for s, e in pairs:
                seg = ids[s:e] if e > s else ids[:0]
                d_in += [[mask_id], seg]
                d_out += [seg, [eos]]
            tok = ids.tolist()
            for s, e in sorted(pairs, key=lambda tup: tup[0])[::-1]:
                del tok[s:s + max(0, e - s)]
                tok.insert(s, mask_id)
            out_t.append(np.array(tok, dtype=np.int64))
            out_i.append(np.concatenate(d_in).astype(np.int64))
            out_o.append(np.concatenate(d_out).astype(np.int64))
        if not out_t:
            print('why')
            return None
        return out_t, out_i, out_o


# ---------------------------------------------------------------------------
# collate (dataset.py:783-925)
# ---------------------------------------------------------------------------
def pad1d(x, max_len):
    return np.pad(x, (0, max_len - len(x)), mode='constant')


def _collate(batch):
    batch = [b for b in batch if b]
    if not batch:
        return None
    S = max(max(x.shape[0] for x in item[0]) for item in batch)
    T = max(max(x.shape[0] for x in item[1]) for item in batch)
    rows = [x for item in batch for x in item[0]]
    rows_i = [x for item in batch for x in item[1]]
    rows_o = [x for item in batch for x in item[2]]
    src = np.zeros((len(rows), S), dtype=np.int64)
    tin = np.zeros((len(rows_i), T), dtype=np.int64)
    tout = np.zeros((len(rows_o), T), dtype=np.int64)
    for r, x in enumerate(rows):
        src[r, :len(x)] = x
    for r, x in enumerate(rows_i):
        tin[r, :len(x)] = x
    for r, x in enumerate(rows_o):
        tout[r, :len(x)] = x
    src_t = torch.from_numpy(src)
    tin_t = torch.from_numpy(tin)
    return {"input": src_t, "target_in": tin_t, "target_out": torch.from_numpy(tout),
            "input_pad_mask": src_t == 0, "target_pad_mask": tin_t == 0}


def collate_mlm_pretraining(batch):
    """Pad every song of every item to the batch maxima (dataset.py:802-862)."""
    return _collate(batch)


def collate_mlm_finetuning(batch):
    """Identical to the pretraining collate (dataset.py:865-925)."""
    return _collate(batch)


# ---------------------------------------------------------------------------
# host throughput (bench.py "data_pipeline"; tools/data_rate.py)
# ---------------------------------------------------------------------------
def synth_corpus(n_songs=240, seed0=0):
    """Seeded synthetic corpus: 8-24 bars, 1-3 tracks, controls at track /
    bar ends (the bar_control_at_end layout), in files of 20 songs."""
    from .synth import synth_events
    songs = [synth_events(seed0 + k, 8 + k % 17, 1 + k % 3) for k in range(n_songs)]
    return [songs[i:i + 20] for i in range(0, n_songs, 20)]


def measure_rate(seconds=5.0, control_mode=2, pretraining=True, batch_size=2, dataset_cls=None,
                 collate=None, vocab=None):
    """Items (pretraining masking of one 2200-token group each) + collate in
    one process for ~`seconds`: returns collated tokens/s in the trainer's
    unit B*(S+T) (padded encoder + decoder positions) and raw ids/s."""
    import time
    from .vocab import WordVocab
    vocab = vocab or WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    dataset_cls = dataset_cls or ParallelLanguageDataset
    collate = collate or collate_mlm_pretraining
    groups, lengths = stack_batches(synth_corpus(), max_token_length=2200)
    btc, bcae = {0: (False, False), 1: (True, False), 2: (True, True)}[control_mode]
    np.random.seed(0)
    ds = dataset_cls(vocab, groups, lengths, batch_size, total_mask_ratio=.15, logger=None,
                     pretraining=pretraining, bar_track_control=btc, bar_control_at_end=bcae)
    for i in range(batch_size):  # first touch filters / copies controls in place
        ds[i]
    n = padded = raw = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        items = [ds[n * batch_size + j] for j in range(batch_size)]
        out = collate(items)
        n += 1
        if out is None:
            continue
        B = out["input"].shape[0]
        padded += B * (out["input"].shape[1] + out["target_in"].shape[1])
        raw += int((~out["input_pad_mask"]).sum() + (~out["target_pad_mask"]).sum())
    dt = time.perf_counter() - t0
    return {"batches": n, "seconds": round(dt, 3), "tokens_per_s": padded / dt,
            "ids_per_s": raw / dt, "unit": "collated B*(S+T) tokens/s, one process",
            "groups": len(groups), "mode": control_mode, "pretraining": bool(pretraining)}
