"""CPU checks of the attention-dropout hash restated in tests/hashref.py
(csrc/common.h smer_attn_bits / smer_attn_ge, attention.hip half_masks /
attn_fold_keep): the SWAR byte compare equals a per-byte 7-bit compare for
every threshold, the bf16 half masks select exactly the kept keys, the
keep-word fold puts key (mt, r) at bit 4r + mt, and the realised keep rate /
pairwise independence are those of a fair 7-bit draw."""
import numpy as np

from tests.hashref import attn_keep_mask, attn_scale, attn_threshold, mix24


def swar_ge(h, thr):
    """numpy restatement of smer_attn_ge (bit 8r+7 set iff (byte r & 127) >= thr)."""
    with np.errstate(over="ignore"):
        return (h | np.uint32(0x80808080)) - np.uint32(thr * 0x01010101)


def test_swar_compare_all_thresholds():
    rng = np.random.default_rng(0)
    h = rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32)
    h[:256] = np.arange(256, dtype=np.uint32) * np.uint32(0x01010101)  # every byte value
    for thr in range(1, 128):
        ge = swar_ge(h, thr)
        for r in range(4):
            byte = (h >> np.uint32(8 * r)) & np.uint32(0x7F)
            assert np.array_equal(((ge >> np.uint32(8 * r + 7)) & 1).astype(bool), byte >= thr), (thr, r)


def test_half_masks_from_ge():
    """v_perm bytes [r0 r0 r1 r1] then the 16-bit arithmetic shift by 15:
    0xFFFF for a kept key's bf16 half, 0 for a dropped one."""
    rng = np.random.default_rng(3)
    h = rng.integers(0, 2 ** 32, 2048, dtype=np.uint64).astype(np.uint32)
    ge = swar_ge(h, 13)
    for sel in ((0, 1), (2, 3)):
        b0 = (ge >> np.uint32(8 * sel[0])) & np.uint32(0xFF)
        b1 = (ge >> np.uint32(8 * sel[1])) & np.uint32(0xFF)
        perm = b0 | (b0 << np.uint32(8)) | (b1 << np.uint32(16)) | (b1 << np.uint32(24))
        halves = perm.view(np.int16).reshape(-1, 2) >> 15
        for k, r in enumerate(sel):
            keep = ((h >> np.uint32(8 * r)) & np.uint32(0x7F)) >= 13
            assert np.array_equal(halves[:, k] == -1, keep)


def test_keep_word_fold_layout():
    """OR_mt ge_mt >> (7 - mt), then the nibble fold: bit 4r + mt."""
    rng = np.random.default_rng(1)
    for _ in range(200):
        keep = rng.integers(0, 2, (4, 4)).astype(bool)  # [mt, r]
        acc = 0
        for mt in range(4):
            # don't-care low bits set: the fold must mask them out
            ge = sum(int(keep[mt, r]) << (8 * r + 7) for r in range(4)) | 0x7F7F7F7F
            acc |= (ge >> (7 - mt)) & (0x01010101 << mt)
        y = acc | (acc >> 4)
        word = ((y & 0xFF) | ((y >> 8) & 0xFF00)) & 0xFFFF
        for mt in range(4):
            for r in range(4):
                assert ((word >> (4 * r + mt)) & 1) == keep[mt, r]


def test_attention_keep_statistics():
    p = 0.1
    assert attn_threshold(p) == 13 and abs(attn_scale(p) - 128 / 115) < 1e-12
    keep = attn_keep_mask(1234, p, 2048, 1024)
    rate = 1.0 - keep.mean()
    assert abs(rate - 13 / 128) < 2e-3
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
