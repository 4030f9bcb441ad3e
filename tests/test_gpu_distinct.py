"""Sampler.distinct (RandomValues, Sampler.scala:383-412) on the GPU (K3 + merge).

Parity contract P3: with an injective hash the GPU set equals the oracle's RandomValues set
bit-exactly (compared as sets; the reference's order is HashSet order).  With a colliding hash
(the default Long.hashCode) the default order "auto" -> RSV_DISTINCT_ORDERED replays the reference's
heap, so the set is bit-exact too, tie bucket at the maximum included (against the oracle's
scala-PriorityQueue restatement; the library source itself is not in the image).  order="set"
keeps the order-independent bottom-k by (hash, key): everything below the maximum agrees.
"""
import json
import os
import sys

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
    assert got == want  # GPU order: ascending (scrambled hash, key), as the oracle sorts


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
    """order="set": the bottom-k by (hash, key) keeps everything below the reference's maximum."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(1)
    v = rng.integers(0, 2**40, size=200_000, dtype=np.int64)
    vals = np.concatenate([v, v ^ (v << 32)])  # Long.hashCode collisions
    ref = oracle.Distinct(500, 4, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    wk, wh = ref.result()
    d = Sampler.distinct(500, seed=4, order="set")()  # default hash = Long.hashCode (Sampler.scala:75)
    d.sample_all(vals)
    got = set(d.result().tolist())
    M = wh.max()
    assert len(got) == 500
    assert {int(x) for x, h in zip(wk, wh) if h < M} <= got


def _colliding(rng, n, buckets):
    """Long keys whose Long.hashCode (hi ^ lo) takes only `buckets` values: every hash bucket holds
    many distinct elements, so the reference's boundary bucket is always tied."""
    hi = rng.integers(0, 2**31, size=n, dtype=np.int64)
    lo = (hi ^ rng.integers(0, buckets, size=n, dtype=np.int64)) & 0xFFFFFFFF
    return (hi << 32) | lo


@pytest.mark.parametrize("k,n,buckets", [(1, 10_000, 50), (20, 50_000, 200), (500, 400_000, 3000),
                                         (4096, 2_000_000, 20_000), (3000, 30_000, 100_000)])
def test_default_long_hash_ordered_exact(cuda, oracle, k, n, buckets):
    """Default hash (Long.hashCode, colliding): bit-exact set vs the sequential reference, ties included."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(k + buckets)
    vals = _colliding(rng, n, buckets)
    vals = np.concatenate([vals, vals[: n // 3]])  # repeats of earlier elements
    ref = oracle.Distinct(k, 8, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    wk, wh = ref.result()
    assert (wh == wh.max()).sum() >= 1
    d = Sampler.distinct(k, seed=8)()  # order "auto" -> ordered for Long.hashCode
    d.sample_all(torch.from_numpy(vals).to(cuda))
    assert d.result().tolist() == wk.tolist()
    s = Sampler.distinct(k, seed=8, order="set")()
    s.sample_all(torch.from_numpy(vals).to(cuda))
    got = s.result()
    assert got.size == wk.size


def test_ordered_heavy_repeats(cuda, oracle):
    """Streams of repeats of set members: most survive the maxHash filter (they are below it), so
    the chunks shrink to the candidate buffer; the replica still matches the reference."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(31)
    base = _colliding(rng, 600, 40)
    vals = np.concatenate([base] + [rng.permutation(base) for _ in range(300)])
    ref = oracle.Distinct(50, 13, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    d = Sampler.distinct(50, seed=13)()
    d.sample_all(vals)
    assert d.result().tolist() == ref.result()[0].tolist()


def test_ordered_batching_invariance(cuda, oracle):
    """sample == sampleAll == any chunking, host or device memory, in the ordered mode."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(12)
    vals = np.concatenate([_colliding(rng, 300_000, 2000)] * 2)
    ref = oracle.Distinct(300, 21, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    want = ref.result()[0].tolist()
    cuts = np.r_[0, np.sort(rng.choice(np.arange(1, vals.size), 15, replace=False)), vals.size]
    dd = Sampler.distinct(300, seed=21)()
    dh = Sampler.distinct(300, seed=21)()
    de = Sampler.distinct(300, seed=21)()
    kd = torch.from_numpy(vals).to(cuda)
    for a, b in zip(cuts[:-1], cuts[1:]):
        dd.sample_all(kd[a:b])
        dh.sample_all(vals[a:b])
    for x in vals[:5000]:
        de.sample(int(x))
    de.sample_all(vals[5000:])
    assert dd.result().tolist() == want
    assert dh.result().tolist() == want
    assert de.result().tolist() == want


def test_ordered_forced_on_injective_and_int(cuda, oracle):
    """order="ordered" with injective hashes equals the bottom-k (and the oracle)."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(3)
    vals = rng.integers(-2**63, 2**63 - 1, size=500_000, dtype=np.int64)
    vals = np.concatenate([vals, vals[:100_000]])
    ref = oracle.Distinct(1000, 5, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    d = Sampler.distinct(1000, seed=5, order="ordered")(hash="identity")
    d.sample_all(vals)
    assert d.result().tolist() == ref.result()[0].tolist()
    xs = rng.integers(-2**31, 2**31 - 1, size=100_000).astype(np.int32)
    ref = oracle.Distinct(77, 6, oracle.HASH_JAVA_INT)
    ref.sample_all(xs.astype(np.int64))
    d = Sampler.distinct(77, seed=6, key_type="int", order="ordered")()
    d.sample_all(xs)
    assert d.result().astype(np.int64).tolist() == ref.result()[0].tolist()


def test_ordered_reusable_and_merge(cuda, oracle):
    """Reusable ordered sampler: result() between batches is non-destructive; the multi-GPU merge
    of ordered shards is the bottom-k by (hash, key) of the union, like order="set"."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(9)
    vals = _colliding(rng, 200_000, 5000)
    ref = oracle.Distinct(256, 2, oracle.HASH_JAVA_LONG)
    d = Sampler.distinct(256, seed=2, reusable=True)()
    for part in np.array_split(vals, 4):
        d.sample_all(part)
        ref.sample_all(part)
        assert d.result().tolist() == ref.result()[0].tolist()
    parts = []
    for chunk in np.array_split(vals, 3):
        e = Sampler.distinct(256, seed=2)()
        e.sample_all(torch.from_numpy(chunk).to(cuda))
        parts.append(e.export_state(cuda))
    outs = []
    for order in ("ordered", "set"):
        m = Sampler.distinct(256, seed=2, order=order)()
        m.merge_state(torch.zeros((3, 256), dtype=torch.int64, device=cuda), torch.stack([p[1] for p in parts]),
                      torch.stack([p[2] for p in parts]), [p[3] for p in parts], vals.size)
        outs.append(m.result().tolist())
    assert outs[0] == outs[1] and len(outs[0]) == 256


@pytest.mark.parametrize("buckets", [200_000, 1_000_000])
def test_ordered_sparse_collisions_many_seeds(cuda, oracle, buckets):
    """Long.hashCode with few collisions (~0.1-0.5 elements per hash value): across seeds the
    boundary bucket is sometimes oversubscribed (the set depends on the heap's tie choice: host
    replay of the logged candidates) and mostly not (the device bottom-k is the reference's set
    as is).  Both must match the reference, in one batch and in several with result() between."""
    import torch

    from reservoir_amd import Sampler

    for seed in range(12):
        rng = np.random.default_rng(1000 + seed)
        vals = _colliding(rng, 60_000, buckets)
        vals = np.concatenate([vals, vals[rng.integers(0, vals.size, 20_000)]])
        ref = oracle.Distinct(64, seed, oracle.HASH_JAVA_LONG)
        ref.sample_all(vals)
        d = Sampler.distinct(64, seed=seed)()
        d.sample_all(torch.from_numpy(vals).to(cuda))
        assert d.result().tolist() == ref.result()[0].tolist(), seed
        ref = oracle.Distinct(64, seed, oracle.HASH_JAVA_LONG)
        r = Sampler.distinct(64, seed=seed, reusable=True)()
        for part in np.array_split(vals, 5):
            r.sample_all(part)
            ref.sample_all(part)
            assert r.result().tolist() == ref.result()[0].tolist(), seed


def test_ordered_eager_log_replay(cuda, oracle, monkeypatch):
    """A candidate log at its limit is replayed into the host replica before the next chunk
    (RSV_ORDERED_LOG_LIMIT: test hook, read at creation); the result is unchanged."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", "1")
    rng = np.random.default_rng(5)
    vals = _colliding(rng, 400_000, 4000)
    ref = oracle.Distinct(300, 17, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    want = ref.result()[0].tolist()
    for parts in (1, 6):
        d = Sampler.distinct(300, seed=17)()
        for part in np.array_split(vals, parts):
            d.sample_all(torch.from_numpy(part).to(cuda))
        assert d.result().tolist() == want


@pytest.mark.parametrize("first_min,overlap", [("1", "1"), ("1", "0"), ("1000000000", "1")])
def test_ordered_first_occurrence_replay(cuda, oracle, monkeypatch, first_min, overlap):
    """The host replay of a logged segment either probes the member set per candidate or runs the
    heap alone over the device's first-occurrence flags (a key that repeats an earlier candidate of
    the segment or a member at its start can never be admitted).  RSV_FIRST_MIN (test hook, read at
    creation) picks the form for every segment; eager replays (RSV_ORDERED_LOG_LIMIT) and a reusable
    sampler give many segments whose candidates repeat members and each other: the same set.
    RSV_REPLAY_OVERLAP (test hook, read at creation): each next segment's flags and copies staged on
    the device while the host replays the current one (flags against the members at the current
    segment's start plus its keys) or not."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_FIRST_MIN", first_min)
    monkeypatch.setenv("RSV_REPLAY_OVERLAP", overlap)
    rng = np.random.default_rng(21)
    base = _colliding(rng, 300_000, 2000)
    vals = np.concatenate([base, base[rng.integers(0, base.size, size=200_000)]])
    rng.shuffle(vals)
    for limit in (None, "1"):
        if limit:
            monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", limit)
        ref = oracle.Distinct(500, 9, oracle.HASH_JAVA_LONG)
        r = Sampler.distinct(500, seed=9, reusable=True)()
        for part in np.array_split(vals, 4):
            r.sample_all(torch.from_numpy(part).to(cuda))
            ref.sample_all(part)
            assert r.result().tolist() == ref.result()[0].tolist(), (first_min, limit)


def test_ordered_first_occurrence_replay_int_keys(cuda, monkeypatch):
    """The flags form with 4-byte keys (a colliding precomputed hash, so the replay runs): the same
    set as the set-based form, and as the same stream sampled as Long keys (the scrambled hash
    depends on the hash value only)."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(4)
    xs = rng.integers(-2**31, 2**31 - 1, size=6_000).astype(np.int64)
    xs = np.concatenate([xs, xs[rng.integers(0, xs.size, size=3_000)]]).tolist()
    got = []
    for first_min, key_type in (("1", "int"), ("1000000000", "int"), ("1", "long")):
        monkeypatch.setenv("RSV_FIRST_MIN", first_min)
        monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", "1")
        d = Sampler.distinct(40, seed=12, key_type=key_type)(hash=lambda x: x % 211)
        d.sample_all(xs)
        info = d.distinct_info()
        got.append(sorted(int(v) for v in d.result().tolist()))
        assert info["ordered"] and info["tied"]  # the boundary bucket is oversubscribed: replayed
    assert got[0] == got[1] == got[2]
    assert len(got[0]) == 40


def test_precomputed_hash(cuda, oracle):
    from reservoir_amd import Sampler

    xs = list(range(10_000))
    d = Sampler.distinct(30, seed=2)(hash=lambda x: x * 31 + 7)
    d.sample_all(xs)
    ref = oracle.Distinct(30, 2, oracle.HASH_IDENTITY)
    ref.sample_all([x * 31 + 7 for x in xs])  # identity over the hashed values: same h per element
    want = sorted((x - 7) // 31 for x in ref.result()[0].tolist())
    assert sorted(d.result().tolist()) == want


@pytest.mark.parametrize("key_type", ["long", "int"])
@pytest.mark.parametrize("n_hashes", [1, 3, 40, 5000])
def test_set_mode_few_hash_values(cuda, oracle, key_type, n_hashes):
    """A precomputed hash with few values: thousands of distinct elements share each scrambled
    hash, so no threshold separates k candidates (the batch is then taken in slices that keep every
    element) and the device merge's buckets overflow (> 256 entries; merged on the radix-sort path
    instead); with 5000 values the buckets hold.  Either way the set is the bottom-k by
    (scrambled hash, key) over the distinct elements, in several batches."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(n_hashes)
    hi = 2**31 - 1 if key_type == "int" else 2**62
    xs = rng.integers(-hi, hi, size=60_000, dtype=np.int64)
    xs = np.concatenate([xs, xs[:20_000]])
    k = 700
    d = Sampler.distinct(k, seed=11, key_type=key_type, order="set")(hash=lambda x: (x * 0x9E3779B1) % n_hashes)
    for part in np.array_split(xs, 3):
        d.sample_all(part)
    got = d.result().tolist()
    r = oracle.Distinct(k, 11, oracle.HASH_IDENTITY)
    r0, r1 = r.r0, r.r1
    ent = sorted({(oracle.scramble(r0, r1, (int(x) * 0x9E3779B1) % n_hashes), int(x)) for x in xs.tolist()})
    assert got == [x for _, x in ent[:k]]


def test_ordered_constant_hash(cuda):
    """hash = constant: the reference's heap fills with the first k distinct elements and then
    rejects everything (h < maxHash never holds, Sampler.scala:403), in every batching."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(9)
    xs = rng.integers(-2**40, 2**40, size=30_000, dtype=np.int64)
    xs = np.concatenate([xs[:50], xs])  # repeats inside the fill phase
    k = 1000
    want = sorted(list(dict.fromkeys(xs.tolist()))[:k])
    for parts in (1, 7):
        d = Sampler.distinct(k, seed=3)(hash=lambda x: 12345)  # precomputed -> ordered by default
        for part in np.array_split(xs, parts):
            d.sample_all(part)
        assert sorted(d.result().tolist()) == want


def test_ordered_extreme_keys(cuda, oracle):
    """Keys at the bottom of the Long range (the host replica's element set marks free slots with
    Long.MinValue + 1 and tracks that key by a flag): kept once, repeats rejected, like any key.
    The precomputed hash gives Long.MinValue + 1 the smallest scrambled hash of 1000 values (the
    lowest few of the stream), so it stays in the set; Long.MinValue gets a hash of its own."""
    from reservoir_amd import Sampler

    s_key, m_key = -2**63 + 1, -2**63
    r = oracle.Distinct(5, 4, oracle.HASH_IDENTITY)
    v0 = min(range(1000), key=lambda v: oracle.scramble(r.r0, r.r1, v))
    rng = np.random.default_rng(77)
    xs = rng.integers(10**6, 10**12, size=6000, dtype=np.int64).tolist()
    for p in (0, 7, 500, 2999, 5999):
        xs.insert(p, s_key)
    for p in (3, 1200, 4000):
        xs.insert(p, m_key)
    hf = {s_key: v0, m_key: 1000}
    for k in (1, 5, 64):
        d = Sampler.distinct(k, seed=4)(hash=lambda x: hf.get(x, x))
        d.sample_all(xs)
        ref = oracle.Distinct(k, 4, oracle.HASH_IDENTITY)
        ref.sample_all([hf.get(x, x) for x in xs])
        inv = {v: x for x, v in hf.items()}
        want = sorted(inv.get(v, v) for v in ref.result()[0].tolist())
        got = d.result().tolist()
        assert sorted(got) == want and got.count(s_key) == want.count(s_key) <= 1
        assert k < 64 or (s_key in want and m_key in xs)


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


@pytest.mark.parametrize("key_type", ["long", "int"])
def test_set_mode_speculative_publication(cuda, oracle, monkeypatch, key_type):
    """Set-mode batches of at least RSV_SPEC_MIN_BATCH keys (test hook, read at creation; the
    product default is 2^27) publish the merged set right behind the ctl read, and result() only
    waits for it.  Forced on every batch here: several batches, a reusable sampler read between
    batches, threshold retries (heavy duplication), the few-hash-values slice fallback, and host
    batches -- every result equals the oracle's."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_SPEC_MIN_BATCH", "1")
    dt = np.int64 if key_type == "long" else np.int32
    hi = 2**31 - 1 if key_type == "int" else 2**62
    rng = np.random.default_rng(21)
    for k, n, uniq in [(1000, 2_000_000, 0.7), (65_536, 1_500_000, 0.05), (10, 5_000, 1.0)]:
        base = rng.integers(-hi, hi, size=max(1, int(n * uniq)), dtype=np.int64)
        vals = np.concatenate([base, base[rng.integers(0, base.size, size=n - base.size)]])
        rng.shuffle(vals)
        vals = vals.astype(dt)
        d = Sampler.distinct(k, seed=23, key_type=key_type, reusable=True)(hash="identity")
        ref = oracle.Distinct(k, 23, oracle.HASH_IDENTITY)
        vd = torch.from_numpy(vals).to(cuda)
        for part_i, (a, b) in enumerate([(0, n // 4), (n // 4, n // 2), (n // 2, n)]):
            if part_i == 1:
                d.sample_all(vals[a:b])  # host batch
            else:
                d.sample_all(vd[a:b])
            ref.sample_all(vals[a:b].astype(np.int64))
            assert np.array_equal(d.result(), ref.result()[0].astype(dt)), (k, n, part_i)
    # few hash values: the slice fallback (sub-batches below the hook's threshold still publish)
    xs = rng.integers(-hi, hi, size=30_000, dtype=np.int64).astype(dt)
    d = Sampler.distinct(300, seed=11, key_type=key_type, order="set")(hash=lambda x: (x * 0x9E3779B1) % 3)
    d.sample_all(xs)
    r = oracle.Distinct(300, 11, oracle.HASH_IDENTITY)
    ent = sorted({(oracle.scramble(r.r0, r.r1, (int(x) * 0x9E3779B1) % 3), int(x)) for x in xs.tolist()})
    assert d.result().tolist() == [x for _, x in ent[:300]]


def _c4_like(cuda, n, seed):
    sys_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
    if sys_path not in sys.path:
        sys.path.insert(0, sys_path)
    import workloads

    return workloads.c4_data(n, cuda, seed=seed)


@pytest.mark.parametrize("k,n,seed,batches", [(2048, 4_000_000, 3, 1), (1000, 3_000_000, 5, 3), (64, 2_000_000, 9, 2)])
def test_ordered_scheduled_pass(cuda, oracle, monkeypatch, k, n, seed, batches):
    """The scheduled pass (one filter with per-range bounds fixed ahead, verified in the merge,
    rsv_distinct.hip sched_sample) gives the reference's set; so does the chunk loop alone
    (RSV_ORDERED_SCHED=0, read at creation), and a schedule too tight to verify
    (RSV_SCHED_BETA=0.2) that falls back to the chunk loop with the set restored."""
    import torch

    from reservoir_amd import Sampler

    vals = _c4_like(cuda, n, seed)
    host = vals.cpu().numpy()
    ref = oracle.Distinct(k, 17, oracle.HASH_JAVA_LONG)
    ref.sample_all(host)
    want = ref.result()[0].tolist()
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    for env in ({}, {"RSV_ORDERED_SCHED": "0"}, {"RSV_SCHED_BETA": "0.2"}):
        for key, v in env.items():
            monkeypatch.setenv(key, v)
        d = Sampler.distinct(k, seed=17)()
        for a, b in zip(cuts[:-1], cuts[1:]):
            d.sample_all(vals[a:b])
        info = d.distinct_info()  # which path ran (the fallbacks are silent otherwise)
        if not env:
            assert info["sched_passes"] >= 1 and info["sched_fallbacks"] == 0, info
        elif "RSV_ORDERED_SCHED" in env:
            assert info["sched_passes"] == 0 and info["sched_fallbacks"] == 0, info
        else:
            assert info["sched_fallbacks"] >= 1, info
        assert d.result().tolist() == want, env
        for key in env:
            monkeypatch.delenv(key)
    del vals
    torch.cuda.empty_cache()


def test_ordered_fused_plan_without_full_heap(cuda, oracle):
    """A fresh sampler's first chunk that does NOT fill the heap (its keys repeat a small set): the
    device plan behind it is void (ctl_plan), the chunk loop goes on, and the host plans the
    scheduled pass once the heap is full -- same set as the reference."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(77)
    k = 2048
    head = rng.integers(-2**63, 2**63 - 1, size=1500, dtype=np.int64)[rng.integers(0, 1500, 200_000)]
    tail = rng.integers(-2**63, 2**63 - 1, size=3_000_000, dtype=np.int64)
    vals = np.concatenate([head, tail, tail[:500_000]])
    ref = oracle.Distinct(k, 31, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    d = Sampler.distinct(k, seed=31)()
    d.sample_all(torch.from_numpy(vals).to(cuda))
    info = d.distinct_info()
    assert info["sched_passes"] >= 1, info
    assert d.result().tolist() == ref.result()[0].tolist()


def test_ordered_scheduled_pass_ties(cuda, oracle):
    """Colliding Long.hashCode values (tied boundary buckets) through the scheduled pass: the pass's
    candidates form one logged segment, and the host replay over it reproduces the reference."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(44)
    vals = _colliding(rng, 3_000_000, 400_000)
    vals = np.concatenate([vals, vals[:1_000_000]])
    ref = oracle.Distinct(1500, 23, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    d = Sampler.distinct(1500, seed=23)()
    d.sample_all(torch.from_numpy(vals).to(cuda))
    assert d.result().tolist() == ref.result()[0].tolist()


@pytest.mark.gpu
def test_ordered_speculative_publication(cuda, oracle, monkeypatch):
    """Ordered mode (default Long.hashCode): a batch that takes the scheduled pass publishes the
    merged set right behind the pass's verdict (RSV_SPEC_MIN_BATCH=1 forces it on every such batch),
    and result() takes that publication only when the pass verified and left no tie for the host
    replica.  Several batches of a reusable sampler with results read in between, host and device
    batches, colliding hashes (tied boundary buckets: the replay path must not use the stale
    publication), and a fresh single-use sampler: every result equals the oracle's sequential
    RandomValues."""
    import torch

    from reservoir_amd import Sampler

    monkeypatch.setenv("RSV_SPEC_MIN_BATCH", "1")
    rng = np.random.default_rng(31)
    for k, n, buckets in [(300, 600_000, None), (300, 600_000, 400), (2000, 900_000, None)]:
        if buckets is None:
            base = rng.integers(-2**62, 2**62, size=int(n * 0.7), dtype=np.int64)
            vals = np.concatenate([base, base[rng.integers(0, base.size, size=n - base.size)]])
            rng.shuffle(vals)
        else:
            vals = _colliding(rng, n, buckets)
        d = Sampler.distinct(k, seed=17, reusable=True)()  # default hash -> ordered
        ref = oracle.Distinct(k, 17, oracle.HASH_JAVA_LONG)
        vd = torch.from_numpy(vals).to(cuda)
        for part_i, (a, b) in enumerate([(0, n // 3), (n // 3, 2 * n // 3), (2 * n // 3, n)]):
            if part_i == 1:
                d.sample_all(vals[a:b])  # host batch
            else:
                d.sample_all(vd[a:b])
            ref.sample_all(vals[a:b])
            assert np.array_equal(np.sort(d.result()), np.sort(ref.result()[0])), (k, n, buckets, part_i)
    d = Sampler.distinct(500, seed=3)()
    d.sample_all(torch.from_numpy(vals).to(cuda))
    ref = oracle.Distinct(500, 3, oracle.HASH_JAVA_LONG)
    ref.sample_all(vals)
    assert np.array_equal(np.sort(d.result()), np.sort(ref.result()[0]))


@pytest.mark.parametrize("shards,k,n,buckets,int_keys", [(2, 64, 60_000, 200_000, False),
                                                         (2, 64, 60_000, 2000, False),
                                                         (3, 300, 400_000, 4000, False),
                                                         (8, 1000, 1_500_000, 30_000, False),
                                                         (4, 200, 200_000, 3000, True)])
def test_ordered_exact_shard_merge(cuda, oracle, shards, k, n, buckets, int_keys):
    """Default hash, stream split into contiguous pieces (piece r = rank r): distributed.merge_local
    (the rows, merge and exact replay of distributed.combine, without a process group) equals the
    reference's sequential RandomValues over the whole stream, tie bucket included -- into a fresh
    sampler and into shard 0 itself."""
    import torch

    from reservoir_amd import Sampler
    from reservoir_amd import distributed as D

    replays = 0
    for seed in range(4):
        rng = np.random.default_rng(700 + 10 * shards + seed)
        if int_keys:
            vals = rng.integers(-2**31, 2**31 - 1, size=n).astype(np.int64)
            vals = np.concatenate([vals, vals[rng.integers(0, n, n // 4)]])
            ref = oracle.Distinct(k, seed, oracle.HASH_JAVA_INT)
        else:
            vals = _colliding(rng, n, buckets)
            vals = np.concatenate([vals, vals[rng.integers(0, n, n // 4)]])
            ref = oracle.Distinct(k, seed, oracle.HASH_JAVA_LONG)
        ref.sample_all(vals)
        want = ref.result()[0].tolist()
        kt = "int" if int_keys else "long"
        dt = torch.int32 if int_keys else torch.int64
        for into_shard in (False, True):
            ss = []
            for piece in np.array_split(vals, shards):
                s = Sampler.distinct(k, seed=seed, key_type=kt, order="ordered", retain_log=True)()
                s.sample_all(torch.from_numpy(piece).to(dt).to(cuda))
                ss.append(s)
            target = ss[0] if into_shard else Sampler.distinct(k, seed=seed, key_type=kt, order="ordered")()
            replays += D.merge_local(target, ss)
            assert target.count == vals.size
            assert target.result().astype(np.int64).tolist() == want, (seed, into_shard)
    if not int_keys and buckets <= 30_000:
        assert replays > 0  # dense collisions oversubscribe the boundary bucket: the exact replay ran


def test_ordered_exact_merge_archived_log(cuda, oracle, monkeypatch):
    """Shards whose logs were replayed eagerly (RSV_ORDERED_LOG_LIMIT) or finalized by result-like
    calls keep every candidate in the host archive: the exact merge is unchanged.  Sampling after a
    merge drops the pre-merge log (rsv_export_log then reports it as not retained)."""
    import torch

    from reservoir_amd import Sampler, _native as N
    from reservoir_amd import distributed as D

    monkeypatch.setenv("RSV_ORDERED_LOG_LIMIT", "1")
    rng = np.random.default_rng(77)
    vals = _colliding(rng, 300_000, 2500)
    want = {}
    for seed in range(3):
        ref = oracle.Distinct(250, seed, oracle.HASH_JAVA_LONG)
        ref.sample_all(vals)
        want[seed] = ref.result()[0].tolist()
        ss = []
        for piece in np.array_split(vals, 3):
            s = Sampler.distinct(250, seed=seed, retain_log=True)()
            for sub in np.array_split(piece, 4):
                s.sample_all(torch.from_numpy(sub).to(cuda))
            ss.append(s)
        info = ss[1].distinct_info()
        assert info["ordered"] == 1 and info["log_retained"] == 1
        t = Sampler.distinct(250, seed=seed)()
        replayed = D.merge_local(t, ss)
        if replayed:  # rsv_merge_log: the replica is the history now
            assert t.distinct_info()["log_retained"] == 0
        assert t.result().tolist() == want[seed], seed
    # rsv_merge_state keeps the merged sampler's own log readable until it samples again
    s = ss[1]
    before = s.export_log()
    parts = [p.export_state(cuda) for p in ss]
    s.merge_state(torch.zeros((3, 250), dtype=torch.int64, device=cuda), torch.stack([p[1] for p in parts]),
                  torch.stack([p[2] for p in parts]), [p[3] for p in parts], vals.size)
    after = s.export_log()
    assert np.array_equal(before[0], after[0]) and np.array_equal(before[1], after[1])
    s.sample_all(torch.from_numpy(vals[:1000]).to(cuda))
    assert s.distinct_info()["log_retained"] == 0
    with pytest.raises(N.ReservoirError):
        s.export_log()
