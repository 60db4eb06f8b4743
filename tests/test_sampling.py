"""The host sampler's fast path draws the same ids from the same NumPy stream
as `np.random.choice` (the reference's `weighted_sampling`,
`/root/reference/generation.py:33-38`), and leaves the generator in the same
state; inputs NumPy's checks reject still raise NumPy's errors."""
import numpy as np
import pytest

from smer_music_generation_amd import generation as G


def _ref_weighted(probs):
    probs = probs / sum(probs)
    sorted_index = np.argsort(probs)[::-1]
    return np.random.choice(sorted_index, size=1, p=probs[sorted_index])[0]


@pytest.mark.parametrize("seed", range(6))
def test_choice1_matches_numpy_choice(seed):
    rng = np.random.default_rng(seed)
    for trial in range(300):
        n = int(rng.integers(1, 400))
        kind = trial % 4
        if kind == 0:
            p = rng.random(n)
        elif kind == 1:  # peaked softmax
            p = np.exp(rng.normal(0, 6, n))
        elif kind == 2:  # zeros and ties
            p = rng.integers(0, 3, n).astype(np.float64)
            p[0] += 1.0
        else:  # one-hot
            p = np.zeros(n)
            p[int(rng.integers(0, n))] = 1.0
        p = p / p.sum()
        a = np.arange(n)[::-1].copy()
        np.random.seed(1000 * seed + trial)
        want = np.random.choice(a, size=1, p=p)[0]
        st_want = np.random.get_state()[1].copy()
        np.random.seed(1000 * seed + trial)
        got = G._choice1(a, p)
        assert got == want
        assert np.array_equal(np.random.get_state()[1], st_want)


def test_sampling_stream_matches_reference_weighted_sampling():
    """sampling() over masked logits, token after token on one stream."""
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    rng = np.random.default_rng(7)
    logits = [rng.normal(0, 4, v.vocab_size).astype(np.float32) for _ in range(400)]
    np.random.seed(3)
    got = [G.sampling(lg, v, no_pitch=bool(i % 3 == 0), no_eos=bool(i % 2)) for i, lg in enumerate(logits)]
    np.random.seed(3)
    want = []
    for i, lg in enumerate(logits):
        keep = G.allowed_ids(v, no_pitch=bool(i % 3 == 0), no_eos=bool(i % 2))
        x = np.where(keep, lg.astype(np.float64), -100.0)
        e = np.exp(x)
        want.append(_ref_weighted(e / np.sum(e)))
    assert got == want


def test_choice1_rejects_like_numpy():
    a = np.arange(3)
    for p in (np.array([0.5, np.nan, 0.5]), np.array([0.7, -0.2, 0.5])):
        with pytest.raises(ValueError):
            np.random.choice(a, size=1, p=p)
        with pytest.raises(ValueError):
            G._choice1(a, p)


def test_reject_table_matches_grammar_checks():
    """The device sampler's redraw table (generation.reject_table) holds the
    reference's redraw checks (generation.py:556-615, grammar_spec) state by
    state: 1 exactly where the check asks for another draw."""
    from smer_music_generation_amd.generation import N_GRAMMAR_STATES, grammar_spec, reject_table
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    rej = reject_table(v)
    assert rej.shape == (N_GRAMMAR_STATES, v.vocab_size)
    for code in range(N_GRAMMAR_STATES):
        chk = grammar_spec(v, code)[1]
        want = [bool(chk(i)) if chk is not None else False for i in range(v.vocab_size)]
        assert [bool(x) for x in rej[code]] == want
    assert rej[0].sum() > 0 and rej[6:10].sum() == 0 and rej[11:].sum() == 0
