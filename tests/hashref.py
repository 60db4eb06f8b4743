"""numpy restatement of the engine's counter-based dropout hash
(csrc/common.h smer_hash3) so tests can rebuild the exact keep-mask."""
import numpy as np


def _rotl(x, r):
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def hash3(seed, a, b):
    with np.errstate(over="ignore"):
        a = np.asarray(a, dtype=np.uint32)
        b = np.asarray(b, dtype=np.uint32)
        h = np.uint32(seed) ^ np.uint32(0x9E3779B9)
        h = (h ^ (a * np.uint32(0xCC9E2D51))).astype(np.uint32)
        h = _rotl(h, 15)
        h = (h * np.uint32(0x1B873593)).astype(np.uint32)
        h = (h ^ (b * np.uint32(0x85EBCA6B))).astype(np.uint32)
        h = _rotl(h, 13)
        h = (h * np.uint32(5) + np.uint32(0xE6546B64)).astype(np.uint32)
        h ^= h >> np.uint32(16)
        h = (h * np.uint32(0x85EBCA6B)).astype(np.uint32)
        h ^= h >> np.uint32(13)
        h = (h * np.uint32(0xC2B2AE35)).astype(np.uint32)
        h ^= h >> np.uint32(16)
    return h


def threshold(p):
    if p <= 0:
        return 0
    t = p * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def keep_mask(seed, p, rows, cols, row_ids=None):
    """bool [rows, cols]: keep(seed, row, col) for row in row_ids (default range)."""
    r = np.arange(rows, dtype=np.uint32) if row_ids is None else np.asarray(row_ids, np.uint32)
    c = np.arange(cols, dtype=np.uint32)
    h = hash3(seed, r[:, None], c[None, :])
    return h >= np.uint32(threshold(p))
