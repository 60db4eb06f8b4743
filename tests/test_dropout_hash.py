"""CPU checks of the attention-dropout hash restated in tests/hashref.py
(csrc/common.h smer_attn_bits / smer_attn_ge / attn_fold_keep): the SWAR
byte compare equals a per-byte compare for every threshold, the keep-word
fold puts key (mt, r) at bit 4r + mt, and the realised keep rate / pairwise
independence are those of a fair 8-bit draw."""
import numpy as np

from tests.hashref import attn_keep_mask, attn_scale, attn_threshold, mix24


def swar_ge(h, thr):
    """numpy restatement of smer_attn_ge (bit 8r+7 set iff byte r >= thr)."""
    lo4 = np.uint32((thr & 127) * 0x01010101)
    sel = np.uint32(0xFFFFFFFF if thr < 128 else 0)
    with np.errstate(over="ignore"):
        d = (h | np.uint32(0x80808080)) - lo4
    return ((h & d) | (sel & (h ^ d))) & np.uint32(0x80808080)


def test_swar_compare_all_thresholds():
    rng = np.random.default_rng(0)
    h = rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32)
    h[:256] = np.arange(256, dtype=np.uint32) * np.uint32(0x01010101)  # every byte value
    for thr in range(1, 256):
        ge = swar_ge(h, thr)
        for r in range(4):
            byte = (h >> np.uint32(8 * r)) & np.uint32(0xFF)
            assert np.array_equal(((ge >> np.uint32(8 * r + 7)) & 1).astype(bool), byte >= thr), (thr, r)


def test_keep_word_fold_layout():
    """OR_mt ge_mt >> (7 - mt), then the nibble fold: bit 4r + mt."""
    rng = np.random.default_rng(1)
    for _ in range(200):
        keep = rng.integers(0, 2, (4, 4)).astype(bool)  # [mt, r]
        acc = 0
        for mt in range(4):
            ge = sum(int(keep[mt, r]) << (8 * r + 7) for r in range(4))
            acc |= ge >> (7 - mt)
        y = acc | (acc >> 4)
        word = ((y & 0xFF) | ((y >> 8) & 0xFF00)) & 0xFFFF
        for mt in range(4):
            for r in range(4):
                assert ((word >> (4 * r + mt)) & 1) == keep[mt, r]


def test_attention_keep_statistics():
    p = 0.1
    assert attn_threshold(p) == 26 and abs(attn_scale(p) - 256 / 230) < 1e-12
    keep = attn_keep_mask(1234, p, 2048, 1024)
    rate = 1.0 - keep.mean()
    assert abs(rate - 26 / 256) < 2e-3
    k = keep.astype(np.float64) - keep.mean()
    var = (k * k).mean()
    for a, b in ((k[:, :-1], k[:, 1:]), (k[:, :-4], k[:, 4:]), (k[:-1], k[1:])):
        assert abs((a * b).mean() / var) < 5e-3
    # different seeds draw different masks
    assert (attn_keep_mask(1235, p, 64, 256) != attn_keep_mask(1234, p, 64, 256)).mean() > 0.1


def test_mix24_avalanche():
    rng = np.random.default_rng(2)
    x = rng.integers(0, 2 ** 32, 50000, dtype=np.uint64).astype(np.uint32)
    hx = mix24(x)
    for b in range(32):
        d = hx ^ mix24(x ^ np.uint32(1 << b))
        frac = np.unpackbits(d.view(np.uint8)).mean()
        assert 0.47 < frac < 0.53, (b, frac)
