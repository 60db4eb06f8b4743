"""Inputs shared by the data-pipeline fixture generator (make_golden_data.py,
run against the reference) and its tests (test_data_pipeline.py, run
against smer_music_generation_amd.data): seeded synthetic songs and the
dataset configurations (train.py:470-536 control modes)."""
from smer_music_generation_amd.synth import synth_events

ALL5 = ['key', 'tensile', 'density', 'polyphony', 'occupation']
KD = ['key', 'density']


def _song(seed):
    """Song spec from a seed: bars, tracks, meter, control layout."""
    n_bars = 2 + seed % 6
    n_tracks = 1 + (seed // 6) % 3
    ts = ("4/4", "3/4", "2/4")[(seed // 18) % 3]
    copy_controls = (seed % 4) != 1
    return (seed, n_bars, n_tracks, ts, copy_controls)


def _files(first, n_files, per_file):
    return [[_song(first + f * per_file + k) for k in range(per_file)] for f in range(n_files)]


def build_files(spec):
    """[[song spec...] per file] -> [[event list...] per file] (fresh lists)."""
    out = []
    for songs in spec:
        out.append([synth_events(s, nb, nt, ts, copy_controls=cc) for (s, nb, nt, ts, cc) in songs])
    return out


# stack_batches: duplicates (same seed twice), one song over the budget
_stack_files = _files(100, 4, 9)
_stack_files[1].append(_song(103))          # duplicate of a song of file 0
_stack_files[2].append((777, 60, 3, "4/4", True))  # longer than the budget: skipped
STACK_CASE = {"files": _stack_files, "max_token_length": 700}


def _case(name, pretraining, mode, controls, first):
    btc, bcae = {0: (False, False), 1: (True, False), 2: (True, True)}[mode]
    return {"name": name, "pretraining": pretraining, "bar_track_control": btc,
            "bar_control_at_end": bcae, "controls": controls, "files": _files(first, 3, 8),
            "max_token_length": 900, "batch_size": 2, "items": 12, "np_seed": first}


CASES = [
    _case("pre_mode0_all5", True, 0, ALL5, 200),
    _case("pre_mode1_all5", True, 1, ALL5, 300),
    _case("pre_mode2_all5", True, 2, ALL5, 400),
    _case("pre_mode2_kd", True, 2, KD, 500),
    _case("fine_mode0_all5", False, 0, ALL5, 600),
    _case("fine_mode1_all5", False, 1, ALL5, 700),
    _case("fine_mode2_all5", False, 2, ALL5, 800),
    _case("fine_mode1_kd", False, 1, KD, 900),
    _case("fine_mode2_kd", False, 2, KD, 1000),
]


def flatten_item(item, vals, struct):
    """(tokens, dec_in, dec_tgt) lists of arrays -> flat values + structure
    ([-1] for a None item, else [n_songs, (len_t, len_i, len_o) x n])."""
    if item is None:
        struct.append(-1)
        return
    t, i, o = item
    struct.append(len(t))
    for a, b, c in zip(t, i, o):
        struct += [len(a), len(b), len(c)]
        vals += [int(x) for x in a] + [int(x) for x in b] + [int(x) for x in c]
