"""The reference's own test properties (SamplerTest.scala), asserted on the CPU oracle.

The reference holds no golden outputs; what its tests pin is behaviour: sample == sampleAll
across collection shapes under one seed, boundary cases, duplicate handling and 5-sigma
fairness.  The oracle must satisfy all of them before it may judge the GPU engine.
"""
import math

import numpy as np
import pytest


def _sample_elements(oracle, k, xs, seed=0):
    s = oracle.AlgoL(k, seed)
    for x in xs:
        s.sample(x)
    return s.result().tolist()


def test_sample_equals_sample_all_every_shape(oracle):
    """SamplerTest.scala:117-142: per-element, IndexedSeq and chunked sampleAll agree."""
    base = _sample_elements(oracle, 20, range(1, 3001))
    chunkings = [[(1, 1000), (1001, 2000), (2001, 3000)], [(1, 3000)], [(1, 7), (8, 19), (20, 21), (22, 3000)]]
    for chunks in chunkings:
        s = oracle.AlgoL(20, 0)
        for a, b in chunks:
            s.sample_all(np.arange(a, b + 1, dtype=np.int64))
        assert s.result().tolist() == base
    # mixed per-element and batch calls
    s = oracle.AlgoL(20, 0)
    for x in range(1, 500):
        s.sample(x)
    s.sample_all(np.arange(500, 3001, dtype=np.int64))
    assert s.result().tolist() == base


@pytest.mark.parametrize("k", [1, 5, 64, 100, 1023, 1024])
def test_sample_equals_sample_all_random_sizes(oracle, k):
    rng = np.random.default_rng(k)
    n = 20000
    xs = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)
    base = _sample_elements(oracle, k, xs.tolist(), seed=k)
    s = oracle.AlgoL(k, k)
    cuts = np.sort(rng.choice(np.arange(1, n), size=9, replace=False))
    for a, b in zip(np.r_[0, cuts], np.r_[cuts, n]):
        s.sample_all(xs[a:b])
    assert s.result().tolist() == base


def test_boundaries(oracle):
    # SamplerTest.scala:81-91
    assert sorted(_sample_elements(oracle, 5, range(1, 6))) == [1, 2, 3, 4, 5]
    assert sorted(_sample_elements(oracle, 6, range(1, 6))) == [1, 2, 3, 4, 5]
    assert _sample_elements(oracle, 1, []) == []
    # SamplerTest.scala:319-339: duplicates kept / collapsed
    assert _sample_elements(oracle, 10, [1] * 10) == [1] * 10
    d = oracle.Distinct(10, 0, oracle.HASH_JAVA_INT)
    for _ in range(10):
        d.sample(1)
    assert d.result()[0].tolist() == [1]


def test_fairness_five_sigma(oracle):
    """SamplerTest.scala:156-176 (1e6 trials there; 2e4 here with the same 5-sigma rule)."""
    trials = 20000
    elements = list(range(1, 11))
    counts = {e: 0 for e in elements}
    for t in range(trials):
        for e in _sample_elements(oracle, 5, elements, seed=t + 1):
            counts[e] += 1
    sd = math.sqrt(trials / 4.0)
    for c in counts.values():
        assert abs(c - trials / 2) < math.ceil(5 * sd)


def test_distinct_order_independent_with_injective_hash(oracle):
    rng = np.random.default_rng(3)
    vals = rng.integers(-2**63, 2**63 - 1, size=3000, dtype=np.int64)
    vals = np.concatenate([vals, vals[:1000]])
    sets = []
    for perm_seed in range(5):
        p = np.random.default_rng(perm_seed).permutation(vals)
        d = oracle.Distinct(100, 11, oracle.HASH_IDENTITY)
        d.sample_all(p)
        sets.append(d.result()[0].tolist())
    assert all(s == sets[0] for s in sets)
    # and it is exactly the bottom-100 of the scrambled hash over the distinct values
    d = oracle.Distinct(100, 11, oracle.HASH_IDENTITY)
    h = sorted((oracle.scramble(d.r0, d.r1, int(v)), int(v)) for v in set(vals.tolist()))
    assert sorted(v for _, v in h[:100]) == sorted(sets[0])


def test_distinct_colliding_hash_keeps_everything_below_max(oracle):
    """the final set = every distinct element with h < M, plus some at M."""
    rng = np.random.default_rng(9)
    vals = rng.integers(0, 2**40, size=5000, dtype=np.int64)
    vals = np.concatenate([vals, vals ^ (vals << 32)])  # Long.hashCode collisions
    d = oracle.Distinct(64, 5, oracle.HASH_JAVA_LONG)
    d.sample_all(vals)
    keys, hs = d.result()
    M = hs.max()
    below = {int(v) for v in set(vals.tolist())
             if oracle.scramble(d.r0, d.r1, oracle.lib().or_java_long_hashcode(int(v))) < M}
    assert below <= set(keys.tolist())


def test_algo_r_draw_uniformity(oracle):
    """Draw format R2: j_i uniform on [0, i] (chi-square over 32 bins at i = 31)."""
    # index 31 in many independent streams
    j = np.array([oracle.draw_j(1234, s, 31) for s in range(64000)])
    assert j.min() >= 0 and j.max() <= 31
    obs = np.bincount(j, minlength=32)
    exp = 64000 / 32
    chi2 = ((obs - exp) ** 2 / exp).sum()
    assert chi2 < 80  # dof 31: p(chi2 > 80) ~ 2e-6


def test_algo_r_replay_matches(oracle):
    keys = oracle.splitmix_keys(77, 5000)
    j = oracle.export_draws(5, 6, 0, 5000)
    want, _ = oracle.algo_r(5, 6, 50, keys)
    assert oracle.algo_r_replay(50, j, keys).tolist() == want.tolist()
