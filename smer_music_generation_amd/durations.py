"""Note-duration tables used by the infill wire surface.

Restates `encode.get_note_duration_dict` (`encode.py:213-277`) and
`encode.time2durations` (`encode.py:947-954`) without the MIDI libraries the
reference module pulls in at import (`encode.py:1-8`).
"""
from __future__ import annotations

import itertools

import numpy as np

_BASIC = ("half", "quarter", "eighth", "sixteenth")


def get_note_duration_dict(beat_duration, curr_time_signature):
    """Return (name->time, time->name, sorted times, bar duration).

    Durations are sums of 1-4 distinct basic notes joined with '_' in
    combination order (`encode.py:247-266`), plus 'zero' and, for n/4 with
    n >= 4, 'whole' (`encode.py:268-273`).
    """
    num, den = curr_time_signature
    if den == 4:
        quarter = beat_duration
        bar_duration = num * quarter
    else:  # compound (6/8)
        quarter = beat_duration / 3 * 2
        bar_duration = num * (quarter / 2)
    base = {"half": quarter * 2, "quarter": quarter, "eighth": quarter / 2,
            "sixteenth": quarter / 4}
    table = dict(base)
    for r in (2, 3, 4):
        for combo in itertools.combinations(_BASIC, r):
            total = 0
            for name in combo:
                total = total + base[name]
            table["_".join(combo)] = total
    table["zero"] = 0
    if den == 4 and num >= 4:
        table["whole"] = 4 * quarter
    time_to_name = {v: k for k, v in table.items()}
    times = np.sort(np.array(list(time_to_name.keys())))
    return table, time_to_name, times, bar_duration


def time2durations(note_duration, duration_time_to_name, duration_times):
    """Nearest representable duration, split into its component tokens."""
    name = duration_time_to_name[duration_times[int(np.argmin(np.abs(note_duration - duration_times)))]]
    if name == "zero":
        return []
    return name.split("_")


def durations_for_events(events):
    """The (beat, time signature) choice of `generation.py:470-475`."""
    num, den = int(events[0][0]), int(events[0][2])
    beat = 1.5 if den == 8 else 1
    return get_note_duration_dict(beat, (num, den))
