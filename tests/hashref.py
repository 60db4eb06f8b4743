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


# --- attention-probability dropout (csrc/common.h smer_attn_keep) ----------
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


def attn_keep_mask(seed, p, rows, cols):
    """bool [rows, cols]: row = (b*H + h)*Lq + query, col = key."""
    with np.errstate(over="ignore"):
        r = np.arange(rows, dtype=np.uint32)
        rk = mix32(mix32(r ^ np.uint32(0x85EBCA6B)) ^ np.uint32(seed))
        c = np.arange(cols, dtype=np.uint32)
        h = mix32((rk[:, None] + (c[None, :] >> np.uint32(1)) * np.uint32(0x9E3779B9)).astype(np.uint32))
    bits = np.where((c[None, :] & 1) == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return bits >= np.uint32(attn_threshold(p))
