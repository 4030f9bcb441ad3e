"""Sampler.distinct (RandomValues, Sampler.scala:383-412) on the GPU (K3 + merge).

Parity contract P3: with an injective hash the GPU set equals the oracle's RandomValues set
bit-exactly (compared as sets; the reference's order is HashSet order).  With a colliding hash
(the default Long.hashCode) every element whose scrambled hash is below the final maximum is
kept by both; only the tie bucket at the maximum is order-dependent (parity unpinned there).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


@pytest.mark.parametrize("case", GOLDEN["distinct"], ids=lambda c: f"k{c['k']}_h{c['hash_kind']}")
def test_golden_distinct(cuda, oracle, case):
    from reservoir_amd import Sampler

    kinds = {oracle.HASH_IDENTITY: "identity", oracle.HASH_JAVA_LONG: "java_long", oracle.HASH_JAVA_INT: "java_int"}
    key_type = "int" if case["hash_kind"] == oracle.HASH_JAVA_INT else "long"
    d = Sampler.distinct(case["k"], seed=case["seed"], key_type=key_type)(hash=kinds[case["hash_kind"]])
    d.sample_all(np.array(case["values"], dtype=np.int64))
    got = d.result().tolist()
    want = case["result_sorted_by_hash"]
    if case["hash_kind"] == oracle.HASH_JAVA_LONG:
        # only the part strictly below the max is order-free
        hs = dict(zip(case["result_sorted_by_hash"], case["hashes"]))
        M = max(case["hashes"])
        assert {v for v in want if hs[v] < M} <= set(got) and len(got) == len(want)
    else:
        assert got == want  # GPU order: ascending scrambled hash, as the oracle sorts


@pytest.mark.parametrize("k", [1, 10, 1000, 65_536])
@pytest.mark.parametrize("n", [5_000, 2_000_000])
def test_identity_hash_parity(cuda, oracle, k, n):
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(k + n)
    base = rng.integers(-2**63, 2**63 - 1, size=int(n * 0.7), dtype=np.int64)
    vals = np.concatenate([base, base[rng.integers(0, base.size, size=n - base.size)]])
    rng.shuffle(vals)
    ref = oracle.Distinct(k, 17, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    want = ref.result()[0]
    d = Sampler.distinct(k, seed=17)(hash="identity")
    vd = torch.from_numpy(vals).to(cuda)
    cut = n // 3
    d.sample_all(vd[:cut])
    d.sample_all(vd[cut:])
    got = d.result()
    assert np.array_equal(got, want)


def test_int_default_hash_and_per_element(cuda, oracle):
    from reservoir_amd import Sampler

    xs = [int(x) for x in np.random.default_rng(5).integers(-2**31, 2**31 - 1, size=3000)] * 2
    ref = oracle.Distinct(50, 8, oracle.HASH_JAVA_INT)
    ref.sample_all(xs)
    d = Sampler.distinct(50, seed=8, key_type="int")()
    for x in xs:
        d.sample(x)
    assert d.result().tolist() == ref.result()[0].tolist()


def test_default_long_hash_below_max(cuda, oracle):
    from reservoir_amd import Sampler

    rng = np.random.default_rng(1)
    v = rng.integers(0, 2**40, size=200_000, dtype=np.int64)
    vals = np.concatenate([v, v ^ (v << 32)])  # Long.hashCode collisions
    ref = oracle.Distinct(500, 4, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    wk, wh = ref.result()
    d = Sampler.distinct(500, seed=4)()  # default hash = Long.hashCode (Sampler.scala:75)
    d.sample_all(vals)
    got = set(d.result().tolist())
    M = wh.max()
    assert len(got) == 500
    assert {int(x) for x, h in zip(wk, wh) if h < M} <= got


def test_precomputed_hash(cuda, oracle):
    from reservoir_amd import Sampler

    xs = list(range(10_000))
    d = Sampler.distinct(30, seed=2)(hash=lambda x: x * 31 + 7)
    d.sample_all(xs)
    ref = oracle.Distinct(30, 2, oracle.HASH_IDENTITY)
    ref.sample_all([x * 31 + 7 for x in xs])  # identity over the hashed values: same h per element
    want = sorted((x - 7) // 31 for x in ref.result()[0].tolist())
    assert sorted(d.result().tolist()) == want


def test_distinct_lifecycle_and_duplicates(cuda):
    from reservoir_amd import IllegalStateException, Sampler

    d = Sampler.distinct(10, key_type="int")()
    for _ in range(10):
        d.sample(1)
    assert d.result().tolist() == [1]  # SamplerTest.scala:330-338
    with pytest.raises(IllegalStateException):
        d.sample(2)
    r = Sampler.distinct(64, reusable=True, key_type="int")()
    r.result()
    r.sample(1)
    assert r.result().tolist() == [1] and r.is_open


def test_distinct_fairness_five_sigma(cuda):
    """SamplerTest.scala:156-176 for the distinct sampler (4e3 trials, same 5-sigma rule)."""
    import math

    from reservoir_amd import Sampler

    trials = 4_000
    counts = np.zeros(11, dtype=np.int64)
    for t in range(trials):
        d = Sampler.distinct(5, seed=t * 7919 + 1, key_type="int")()
        d.sample_all(np.arange(1, 11, dtype=np.int32))
        for e in d.result():
            counts[e] += 1
    sd = math.sqrt(trials / 4.0)
    assert np.all(np.abs(counts[1:] - trials / 2) < math.ceil(5 * sd)), counts


def test_distinct_merge(cuda, oracle):
    """Multi-GPU contract on one device: bottom-k of per-shard sets == bottom-k of the union."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(4)
    vals = rng.integers(-2**63, 2**63 - 1, size=600_000, dtype=np.int64)
    vals = np.concatenate([vals, vals[:200_000]])
    ref = oracle.Distinct(4096, 6, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    parts = 3
    ks, hs, ns = [], [], []
    for p, chunk in enumerate(np.array_split(vals, parts)):
        d = Sampler.distinct(4096, seed=6)(hash="identity")
        d.sample_all(torch.from_numpy(chunk).to(cuda))
        _, kk, hh, n = d.export_state(cuda)
        ks.append(kk)
        hs.append(hh)
        ns.append(n)
    m = Sampler.distinct(4096, seed=6)(hash="identity")
    m.merge_state(torch.zeros((parts, 4096), dtype=torch.int64, device=cuda), torch.stack(ks), torch.stack(hs),
                  ns, vals.size)
    assert np.array_equal(m.result(), ref.result()[0])


def test_maximum_sample_size(cuda, oracle):
    """k = Int.MaxValue - 2: the distinct state grows with what it holds, not with k."""
    from reservoir_amd import Sampler

    k = 2**31 - 1 - 2
    vals = np.concatenate([oracle.splitmix_keys(2, 300_000)] * 2)
    d = Sampler.distinct(k, seed=3)(hash="identity")
    d.sample_all(vals)
    ref = oracle.Distinct(1 << 20, 3, oracle.HASH_IDENTITY)  # k above the distinct count: all kept
    ref.sample_all(vals)
    assert np.array_equal(d.result(), ref.result()[0])
