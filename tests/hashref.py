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


def drop_threshold(p):
    """16-bit keep threshold of the activation / gradient dropout sites."""
    if p <= 0:
        return 0
    return int(min(65535, max(1, int(p * 65536.0 + 0.5))))


def drop_scale(p):
    t = drop_threshold(p)
    return 65536.0 / (65536.0 - t) if t else 1.0


def _rowkeys(seed, rows, row_ids):
    r = np.arange(rows, dtype=np.uint32) if row_ids is None else np.asarray(row_ids, np.uint32)
    return mix32(mix32(r ^ np.uint32(0x85EBCA6B)) ^ np.uint32(seed))


def keep_mask(seed, p, rows, cols, row_ids=None):
    """bool [rows, cols] keep-mask of the 16-bit sites (csrc/common.h
    smer_keep16); rows are the site's row ids (activation row / token)."""
    with np.errstate(over="ignore"):
        rk = _rowkeys(seed, rows, row_ids)
        c = np.arange(cols, dtype=np.uint32)
        h = mix32((rk[:, None] + (c[None, :] >> np.uint32(1)) * np.uint32(0x9E3779B9)).astype(np.uint32))
    bits = np.where((c[None, :] & 1) == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return bits >= np.uint32(drop_threshold(p))


# ---- attention probabilities: 7-bit thresholds, one hash per 4 keys ----
def mix24(h):
    """csrc/common.h smer_attn_bits' mixer: 24-bit multiplies (v_mul_u32_u24)."""
    with np.errstate(over="ignore"):
        h = np.asarray(h, dtype=np.uint32)
        h = h ^ (h >> np.uint32(16))
        h = ((h & np.uint32(0xFFFFFF)).astype(np.uint64) * 0xEB352D & 0xFFFFFFFF).astype(np.uint32)
        h = h ^ (h >> np.uint32(15))
        h = ((h & np.uint32(0xFFFFFF)).astype(np.uint64) * 0x6CA68B & 0xFFFFFFFF).astype(np.uint32)
        h = h ^ (h >> np.uint32(16))
    return h


def attn_threshold(p):
    if p <= 0:
        return 0
    return int(min(127, max(1, int(p * 128.0 + 0.5))))


def attn_scale(p):
    t = attn_threshold(p)
    return 128.0 / (128.0 - t) if t else 1.0


def attn_keep_mask(seed, p, rows, cols, row_ids=None):
    """bool [rows, cols] keep-mask of attention dropout (smer_attn_keep):
    rows = (b*H + h)*Lq + query, cols = keys; the low 7 bits of byte (key & 3)
    of the hash of (row key, key >> 2) are compared with round(p * 128)."""
    with np.errstate(over="ignore"):
        rk = _rowkeys(seed, rows, row_ids)
        c = np.arange(cols, dtype=np.uint32)
        h = mix24((rk[:, None] + (c[None, :] >> np.uint32(2)) * np.uint32(0x9E3779B9)).astype(np.uint32))
    byte = (h >> (np.uint32(8) * (c[None, :] & np.uint32(3)))) & np.uint32(0x7F)
    return byte >= np.uint32(attn_threshold(p))
