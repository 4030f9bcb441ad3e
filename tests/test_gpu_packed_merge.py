"""The device combine of distinct samplers (rsv_export_packed / rsv_merge_packed on DISTINCT):
packed rows of every shard's set, merged on the device into the bottom-k by (scrambled hash, key)
of the union -- the multi-GPU merge of SURVEY.md 8(e) K3 (RandomValues, Sampler.scala:383-412).

Against the oracle's RandomValues over the whole stream (set mode: identity / Int hashes, where the
union's bottom-k is the reference's set), on the handle's own stream (the call settles) and on a
caller stream (the merge settles at the next call), into a fresh sampler, into a shard, into a
sampler that already holds a set; the radix fallbacks (a bucket overflow from a degenerate hash,
settled after the fact from the caller's rows; more than 64 rows); and the row layout itself."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _shards(cuda, vals, parts, k, seed, key_type="long", hash="identity"):
    import torch

    from reservoir_amd import Sampler

    dt = torch.int64 if key_type == "long" else torch.int32
    out = []
    for piece in np.array_split(vals, parts):
        s = Sampler.distinct(k, seed=seed, key_type=key_type)(hash=hash)
        s.sample_all(torch.from_numpy(piece).to(dt).to(cuda))
        out.append(s)
    return out


def _rows(cuda, shards):
    import torch

    rows = torch.empty((len(shards), shards[0].packed_width), dtype=torch.int64, device=cuda)
    for r, s in enumerate(shards):
        s.export_packed(rows[r])
    return rows


@pytest.mark.parametrize("parts,k,n,key_type", [(1, 100, 50_000, "long"), (2, 1, 1000, "long"),
                                                 (3, 4096, 600_000, "long"), (8, 65536, 2_000_000, "long"),
                                                 (5, 3000, 400_000, "int"), (4, 5000, 9000, "long")])
@pytest.mark.parametrize("caller_stream", [False, True])
def test_packed_merge_matches_oracle(cuda, oracle, parts, k, n, key_type, caller_stream):
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(parts * 1000 + k)
    if key_type == "long":
        vals = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
        hk = oracle.HASH_IDENTITY
        h = "identity"
    else:
        vals = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64)
        hk = oracle.HASH_JAVA_INT
        h = "java_int"
    vals = np.concatenate([vals, vals[rng.integers(0, n, n // 3)]])
    ref = oracle.Distinct(k, 21, hk)
    ref.sample_all(vals)
    want = np.sort(ref.result()[0])
    shards = _shards(cuda, vals, parts, k, 21, key_type, h)
    rows = _rows(cuda, shards)
    for into in ("fresh", "shard"):
        t = Sampler.distinct(k, seed=21, key_type=key_type)(hash=h) if into == "fresh" else shards[0]
        if caller_stream:
            t.set_stream(torch.cuda.current_stream(cuda).cuda_stream)
        t.merge_packed(rows, vals.size)
        assert t.count == vals.size
        info = t.distinct_info()  # settles a pending merge
        assert info["size"] == want.size and info["tied"] == 0
        assert np.array_equal(np.sort(t.result().astype(np.int64)), want), into


def test_packed_merge_into_a_held_set(cuda, oracle):
    """The target keeps its own set (run 0 of the merge) and its element count."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(3)
    vals = rng.integers(-2**63, 2**63 - 1, size=800_000, dtype=np.int64)
    vals = np.concatenate([vals, vals[:300_000]])
    a, b = vals[:500_000], vals[500_000:]
    ref = oracle.Distinct(2048, 4, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    t = Sampler.distinct(2048, seed=4, reusable=True)(hash="identity")
    t.sample_all(a)
    rows = _rows(cuda, _shards(cuda, b, 3, 2048, 4))
    t.merge_packed(rows, vals.size)
    assert np.array_equal(np.sort(t.result()), np.sort(ref.result()[0]))
    # sampling continues after the merge (the pending merge settles first)
    more = rng.integers(-2**63, 2**63 - 1, size=100_000, dtype=np.int64)
    t.sample_all(more)
    ref.sample_all(more)
    assert np.array_equal(np.sort(t.result()), np.sort(ref.result()[0]))


@pytest.mark.parametrize("n_hashes", [1, 3])
def test_packed_merge_overflow_fallback(cuda, oracle, n_hashes):
    """A precomputed hash with 1-3 values: every entry lands in one of a few buckets (> 256: the
    device merge overflows) and the merge is redone on the radix path -- on a caller stream that
    happens when the merge settles, from the caller's rows."""
    import torch

    from reservoir_amd import Sampler

    rng = np.random.default_rng(n_hashes)
    xs = rng.integers(-2**62, 2**62, size=20_000, dtype=np.int64)
    xs = np.concatenate([xs, xs[:5000]])
    k = 700
    hf = lambda x: (x * 0x9E3779B1) % n_hashes  # noqa: E731
    shards = []
    for piece in np.array_split(xs, 4):
        s = Sampler.distinct(k, seed=11, order="set")(hash=hf)
        s.sample_all(piece)
        shards.append(s)
    rows = _rows(cuda, shards)
    t = Sampler.distinct(k, seed=11, order="set")(hash=hf)
    t.set_stream(torch.cuda.current_stream(cuda).cuda_stream)
    t.merge_packed(rows, xs.size)
    r = oracle.Distinct(k, 11, oracle.HASH_IDENTITY)
    ent = sorted({(oracle.scramble(r.r0, r.r1, hf(int(x))), int(x)) for x in xs.tolist()})
    assert sorted(t.result().tolist()) == sorted(x for _, x in ent[:k])


def test_packed_merge_many_rows(cuda, oracle):
    """70 rows (> 64 runs: the radix form, host waits) equal the oracle too."""
    from reservoir_amd import Sampler

    rng = np.random.default_rng(70)
    vals = rng.integers(-2**63, 2**63 - 1, size=140_000, dtype=np.int64)
    ref = oracle.Distinct(512, 8, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    rows = _rows(cuda, _shards(cuda, vals, 70, 512, 8))
    t = Sampler.distinct(512, seed=8)(hash="identity")
    t.merge_packed(rows, vals.size)
    assert np.array_equal(np.sort(t.result()), np.sort(ref.result()[0]))


def test_packed_row_layout(cuda, oracle):
    """[keys (k) | hashes (k) | n, count, tied, max_hash, log_retained, ordered], ascending (h, key)."""
    from reservoir_amd import Sampler

    vals = oracle.splitmix_keys(5, 10_000)
    s = Sampler.distinct(64, seed=2)(hash="identity")
    s.sample_all(vals)
    rows = _rows(cuda, [s]).cpu().numpy()[0]
    ref = oracle.Distinct(64, 2, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    keys, hs = ref.result()
    o = np.lexsort((keys, hs))
    assert np.array_equal(rows[:64], keys[o]) and np.array_equal(rows[64:128], hs[o])
    assert rows[128:].tolist() == [64, 10_000, 0, int(hs[o][-1]), 0, 0]
    few = Sampler.distinct(64, seed=2, retain_log=True)()  # default Long hash: ordered
    few.sample_all(vals[:10])
    r = _rows(cuda, [few]).cpu().numpy()[0]
    assert r[128:].tolist()[0] == 10 and r[128 + 4] == 1 and r[128 + 5] == 1
    assert (r[64 + 10:128] == 2**63 - 1).all()


def test_log_retention_is_opt_in(cuda):
    """An ordered sampler keeps no host archive unless asked (rsv_retain_log): a low-cardinality
    stream (every element a candidate while the heap fills) leaves the host memory flat, and
    export_log reports the log as not retained."""
    import resource

    import torch

    from reservoir_amd import Sampler, _native as N

    vals = torch.arange(200_000, dtype=torch.int64, device=cuda) % 5000
    s = Sampler.distinct(100_000, seed=1)()  # more slots than distinct values: never full
    s.sample_all(vals)
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    # 2e7 candidates: the device log (~1.3e7 entries at this k) is replayed into the host replica
    # on the way -- with retention that alone would archive ~200 MB
    for _ in range(100):
        s.sample_all(vals)
    assert len(s.result()) == 5000
    s = Sampler.distinct(64, seed=1)()
    for _ in range(20):
        s.sample_all(vals)
    info = s.distinct_info()
    assert info["ordered"] == 1 and info["log_retained"] == 0
    with pytest.raises(N.ReservoirError):
        s.export_log()
    assert resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - rss0 < 100 * 1024  # KiB
    r = Sampler.distinct(64, seed=1, retain_log=True)()
    r.sample_all(vals)
    assert r.distinct_info()["log_retained"] == 1


def test_merge_local_needs_retained_logs_when_tied(cuda, oracle):
    """Ordered shards without a retained log whose merged boundary bucket ties: merge_local cannot
    form the reference's arrival-order set -- IllegalStateException by default, a
    RuntimeWarning and the (hash, key) bottom-k with strict=False; with retain_log the exact set."""
    import torch

    from reservoir_amd import IllegalStateException, Sampler
    from reservoir_amd import distributed as D

    rng = np.random.default_rng(8)
    hi = rng.integers(0, 2**31, size=60_000, dtype=np.int64)
    v = (hi << 32) | ((hi ^ rng.integers(0, 700, size=hi.size)) & 0xFFFFFFFF)  # 700 Long.hashCode values
    parts = np.array_split(v, 3)

    def shards(retain):
        out = []
        for p in parts:
            s = Sampler.distinct(300, seed=4, retain_log=retain)()
            s.sample_all(torch.from_numpy(p).to(cuda))
            out.append(s)
        return out

    with pytest.raises(IllegalStateException):
        D.merge_local(Sampler.distinct(300, seed=4)(), shards(False))
    t = Sampler.distinct(300, seed=4)()
    with pytest.warns(RuntimeWarning):
        assert not D.merge_local(t, shards(False), strict=False)
    assert t.result().size == 300
    t = Sampler.distinct(300, seed=4)()
    assert D.merge_local(t, shards(True))
    ref = oracle.Distinct(300, 4, oracle.HASH_JAVA_LONG)
    ref.sample_all(v)
    assert sorted(t.result().tolist()) == sorted(ref.result()[0].tolist())
