"""the warm batch-1 (plugin) session rounds its cache
capacities up to powers of two, but never across the 512-row boundary where
smer_attn_decode switches to its 8-wave variant (csrc/attention.hip
`big = cap_rows >= 512`), so a warm and a cold session of the same request
run the same decode-attention kernels and give the same logits."""
import pytest

from smer_music_generation_amd.generation import _plugin_capacity


@pytest.mark.parametrize("S0", [1, 100, 128, 129, 255, 257, 300, 480, 511, 512, 513, 1024, 1500, 2049])
@pytest.mark.parametrize("T0", [8, 127, 128, 308, 400, 509, 510, 511, 600, 1100])
def test_capacity_rounding_stays_in_the_variant_class(S0, T0):
    S, T = _plugin_capacity(S0, T0)
    assert S >= S0 and T >= T0
    assert (S >= 512) == (S0 >= 512)           # cross memory rows
    assert (T + 1 >= 512) == (T0 + 1 >= 512)   # self cache rows (+ trash slot)
    # still rounded up (reuse across similar calls): powers of two, or the cap
    assert S in (511,) or S & (S - 1) == 0
    assert T in (510,) or (T + 1) & T == 0


def test_capacity_rounding_is_monotone():
    prev = (0, 0)
    for n in range(1, 3000, 7):
        cur = _plugin_capacity(n, n)
        assert cur[0] >= prev[0] and cur[1] >= prev[1]
        prev = cur
