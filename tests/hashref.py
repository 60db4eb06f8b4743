"""numpy restatement of the engine's counter-based dropout
(csrc/common.h smer_rowkey / smer_pair_bits / smer_keep16) so tests can
rebuild the exact keep-mask of any dropout site."""
import numpy as np


def mix32(h):
    with np.errstate(over="ignore"):
        h = np.asarray(h, dtype=np.uint32)
        h = h ^ (h >> np.uint32(16))
        h = (h * np.uint32(0x7FEB352D)).astype(np.uint32)
        h = h ^ (h >> np.uint32(15))
        h = (h * np.uint32(0x846CA68B)).astype(np.uint32)
        h = h ^ (h >> np.uint32(16))
    return h


def attn_threshold(p):
    if p <= 0:
        return 0
    return int(min(65535, max(1, int(p * 65536.0 + 0.5))))


def attn_scale(p):
    t = attn_threshold(p)
    return 65536.0 / (65536.0 - t) if t else 1.0


def keep_mask(seed, p, rows, cols, row_ids=None):
    """bool [rows, cols] keep-mask; rows are the site's row ids (activation
    row / token, or (b*H + h)*Lq + query for attention), cols its columns."""
    with np.errstate(over="ignore"):
        r = np.arange(rows, dtype=np.uint32) if row_ids is None else np.asarray(row_ids, np.uint32)
        rk = mix32(mix32(r ^ np.uint32(0x85EBCA6B)) ^ np.uint32(seed))
        c = np.arange(cols, dtype=np.uint32)
        h = mix32((rk[:, None] + (c[None, :] >> np.uint32(1)) * np.uint32(0x9E3779B9)).astype(np.uint32))
    bits = np.where((c[None, :] & 1) == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return bits >= np.uint32(attn_threshold(p))


attn_keep_mask = keep_mask
drop_scale = attn_scale
