"""Element sampler (Sampler.apply) on the GPU: parity with the oracle, boundaries, lifecycle.

Parity contract P2: the "philox_r" engine equals the sequential Algorithm R
restatement fed the same draw sequence (format R2), bit-exactly, for every batching and split.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def _dev_keys(torch, cuda, keys):
    return torch.from_numpy(np.ascontiguousarray(keys)).to(cuda)


@pytest.mark.parametrize("case", GOLDEN["algo_r"], ids=lambda c: f"k{c['k']}_n{c['n']}")
def test_golden_algo_r(cuda, oracle, case):
    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(case["key_base"], case["n"])
    s = Sampler(case["k"], seed=case["seed"], stream_id=case["stream"])()
    s.sample_all(keys)
    assert s.result().tolist() == case["result"]


@pytest.mark.parametrize("k", [1, 2, 5, 63, 64, 100, 1000, 1024, 4099])
@pytest.mark.parametrize("n", [0, 1, 7, 1000, 65_537, 300_000])
def test_parity_vs_oracle(cuda, oracle, k, n):
    import torch

    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(k * 1000 + n, n)
    want, _ = oracle.algo_r(0xABCDEF + k, n, k, keys)
    s = Sampler(k, seed=0xABCDEF + k, stream_id=n)()
    s.sample_all(_dev_keys(torch, cuda, keys))
    got = s.result()
    assert got.size == min(n, k)
    assert np.array_equal(got, want[: got.size])


def test_batching_and_memory_invariance(cuda, oracle):
    """sample == sampleAll == any chunking, host or device memory (SamplerTest.scala:117-142)."""
    import torch

    from reservoir_amd import Sampler

    n, k = 500_000, 1024
    keys = oracle.splitmix_keys(5, n)
    want, _ = oracle.algo_r(99, 1, k, keys)
    rng = np.random.default_rng(0)
    cuts = np.r_[0, np.sort(rng.choice(np.arange(1, n), 20, replace=False)), n]
    s_dev = Sampler(k, seed=99, stream_id=1)()
    s_host = Sampler(k, seed=99, stream_id=1)()
    kd = _dev_keys(torch, cuda, keys)
    for a, b in zip(cuts[:-1], cuts[1:]):
        s_dev.sample_all(kd[a:b])
        s_host.sample_all(keys[a:b])
    assert np.array_equal(s_dev.result(), want)
    assert np.array_equal(s_host.result(), want)
    s_el = Sampler(k, seed=99, stream_id=1)()
    for x in keys[:3000]:
        s_el.sample(int(x))
    s_el.sample_all(keys[3000:])
    assert np.array_equal(s_el.result(), want)


def test_int_keys_and_map(cuda, oracle):
    from reservoir_amd import Sampler

    xs = list(range(1, 20001))
    s = Sampler(10, key_type="int", seed=3)(lambda x: x * 2)
    s.sample_all(xs)
    want, _ = oracle.algo_r(3, 0, 10, np.array(xs, dtype=np.int64) * 2)
    assert s.result().tolist() == want.tolist()


def test_draw_export_matches_oracle(cuda, oracle):
    from reservoir_amd import batch

    for case in GOLDEN["draws"]:
        j = batch.export_draws(case["seed"], case["stream"], case["i0"], case["n"]).cpu().numpy()
        assert [int(x) for x in j.astype(np.uint64)] == case["j"]
    j = batch.export_draws(17, 3, 10_000, 100_000).cpu().numpy().astype(np.uint64)
    assert np.array_equal(j, oracle.export_draws(17, 3, 10_000, 100_000))


def test_draw_replay_contract(cuda, oracle):
    """north star: equal to a sequential sampler fed the exported per-element draw sequence."""
    import torch

    from reservoir_amd import Sampler, batch

    n, k = 200_000, 256
    keys = oracle.splitmix_keys(8, n)
    j = batch.export_draws(42, 9, 0, n).cpu().numpy().astype(np.uint64)
    want = oracle.algo_r_replay(k, j, keys)
    s = Sampler(k, seed=42, stream_id=9)()
    s.sample_all(torch.from_numpy(keys).to(cuda))
    assert np.array_equal(s.result(), want)


def test_boundaries_and_duplicates(cuda):
    from reservoir_amd import Sampler

    def run(k, xs):
        s = Sampler(k, key_type="int")()
        for x in xs:
            s.sample(x)
        return s.result().tolist()

    assert sorted(run(5, range(1, 6))) == [1, 2, 3, 4, 5]  # SamplerTest.scala:81-83
    assert sorted(run(6, range(1, 6))) == [1, 2, 3, 4, 5]  # :85-87
    assert run(1, []) == []  # :89-91
    assert run(10, [1] * 10) == [1] * 10  # :320-327


def test_single_use_lifecycle(cuda):
    from reservoir_amd import IllegalStateException, Sampler

    s = Sampler(10)()
    assert s.is_open
    s.result()
    assert not s.is_open  # SamplerTest.scala:263-267
    with pytest.raises(IllegalStateException):
        s.sample(1)  # :246-250
    with pytest.raises(IllegalStateException):
        s.result()  # :252-256
    # the device fast path checks open first (Sampler.scala:186): a closed sampler raises
    # IllegalStateException even for a tensor it would reject on dtype
    import torch

    with pytest.raises(IllegalStateException):
        s.sample_all(torch.zeros(8, dtype=torch.int32, device=cuda))
    with pytest.raises(IllegalStateException):
        s.sample_all(torch.zeros(8, dtype=torch.int64, device=cuda))


def test_reusable_does_not_clobber(cuda):
    """SamplerTest.scala:292-316."""
    from reservoir_amd import Sampler

    s = Sampler(64, reusable=True, key_type="int")()

    def results():
        res = s.result()
        lst = res.tolist()
        return res, s.result(), lst

    outs = [results()]
    for a, b in [(1, 32), (33, 64), (65, 128)]:
        for x in range(a, b + 1):
            s.sample(x)
        outs.append(results())
    for ra, rb, lst in outs:
        assert np.array_equal(ra, rb) and ra.tolist() == lst
    assert s.is_open
    assert sorted(outs[2][0].tolist()) == list(range(1, 65))


def test_statistics_sometimes_and_not_always(cuda):
    """SamplerTest.scala:93-115 via independent samplers (fresh seeds)."""
    from reservoir_amd import Sampler

    res = [Sampler(5, key_type="int")() for _ in range(100)]
    for s in res:
        s.sample_all(range(1, 7))
    got = [s.result().tolist() for s in res]
    assert any(6 in g for g in got) and any(6 not in g for g in got)


def test_index_range_split_merge(cuda, oracle):
    """Multi-GPU contract on one device: shards sampled after seek(offset), merged per slot."""
    import torch

    from reservoir_amd import Sampler

    n, k, parts = 1_000_003, 1024, 5
    keys = oracle.splitmix_keys(31, n)
    want, _ = oracle.algo_r(7, 2, k, keys)
    kd = torch.from_numpy(keys).to(cuda)
    bounds = np.linspace(0, n, parts + 1).astype(np.int64)
    idx_parts, key_parts = [], []
    for p in range(parts):
        s = Sampler(k, seed=7, stream_id=2)()
        s.seek(int(bounds[p]))
        s.sample_all(kd[bounds[p]:bounds[p + 1]])
        idx, kk, _, _ = s.export_state(cuda)
        idx_parts.append(idx)
        key_parts.append(kk)
    merged = Sampler(k, seed=7, stream_id=2)()
    merged.merge_state(torch.stack(idx_parts), torch.stack(key_parts),
                       torch.zeros((parts, k), dtype=torch.int64, device=cuda), [k] * parts, n)
    assert merged.count == n
    assert np.array_equal(merged.result(), want)


@pytest.mark.parametrize("key_type", ["long", "int"])
def test_index_range_split_packed(cuda, oracle, key_type):
    """The packed rows of distributed.combine: export_packed -> stacked rows -> merge_packed,
    with a stride wider than 2k (the count column) and one part merged into a non-empty sampler."""
    import torch

    from reservoir_amd import Sampler

    n, k, parts = 700_001, 777, 4
    keys = oracle.splitmix_keys(77, n)
    if key_type == "int":
        keys = keys.astype(np.int32)  # wraps: negative Int keys exercise the sign-extended rows
    want, _ = oracle.algo_r(5, 9, k, keys.astype(np.int64))
    kd = torch.from_numpy(keys).to(cuda)
    bounds = np.linspace(0, n, parts + 1).astype(np.int64)
    rows = torch.full((parts - 1, 2 * k + 1), -7, dtype=torch.int64, device=cuda)
    for p in range(parts - 1):
        s = Sampler(k, seed=5, stream_id=9, key_type=key_type)()
        s.seek(int(bounds[p]))
        s.sample_all(kd[bounds[p]:bounds[p + 1]])
        s.export_packed(rows[p])
        s.close()
    last = Sampler(k, seed=5, stream_id=9, key_type=key_type)()
    last.seek(int(bounds[-2]))
    last.sample_all(kd[bounds[-2]:])
    last.merge_packed(rows, n)
    assert last.count == n
    got = last.result()
    assert got.dtype == keys.dtype
    assert np.array_equal(got.astype(np.int64), want)


@pytest.mark.slow
def test_full_size_split_invariance(cuda):
    """C2 size (1e9 keys, k = 1024): one pass == 7 ragged batches == 4-way index split."""
    import torch

    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    keys = torch.arange(n, dtype=torch.int64, device=cuda)  # key == index: result exposes indices
    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
    s.set_stream(torch.cuda.current_stream().cuda_stream)
    s.sample_all(keys)
    one = s.result()
    assert one.size == k and len(set(one.tolist())) == k  # distinct indices
    assert one.min() >= 0 and one.max() < n
    cuts = [0, 1, 1023, 1024, 7_777_777, 400_000_000, 999_999_999, n]
    s2 = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
    for a, b in zip(cuts[:-1], cuts[1:]):
        s2.sample_all(keys[a:b])
    assert np.array_equal(s2.result(), one)
    # slot j holds its last writer: every winner index i >= k must draw j
    from reservoir_amd import batch

    for j in range(0, k, 97):
        i = int(one[j])
        if i >= k:
            assert int(batch.export_draws(0xC0FFEE, 0x5A5A, i, 1)[0]) == j


@pytest.mark.parametrize("i0,k,n", [(2**32 - 100, 1024, 1_000_000), (5 * 10**9, 65_536, 2_000_000),
                                    (2**40 + 3, 1 << 20, 8_000_000), (2**36 - 3_000_001, 1 << 20, 6_000_000)])
def test_high_index_offsets(cuda, oracle, i0, k, n):
    """Ranks beyond the first 2^32 indices (8-GPU C2 reaches 8e9): 64-bit draw arithmetic.  The
    last case crosses index 2^36 = level-0 block 2^32, where K1 splits its launch (the Philox
    counter's high word is a per-launch scalar)."""
    import ctypes as C

    import torch

    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(i0 & 0xFFFF, n)
    res = np.zeros(k, dtype=np.int64)
    idx = np.full(k, -1, dtype=np.int64)
    oracle.lib().or_algo_r(3, 4, k, i0, keys, n, res, idx.ctypes.data_as(C.c_void_p))
    s = Sampler(k, seed=3, stream_id=4)()
    s.seek(i0)
    s.sample_all(torch.from_numpy(keys).to(cuda))
    gidx, gkeys, _, _ = s.export_state(cuda)
    assert np.array_equal(gidx.cpu().numpy(), idx)
    hit = idx >= 0
    assert hit.sum() > 0
    assert np.array_equal(gkeys.cpu().numpy()[hit], res[hit])


def test_maximum_sample_size(cuda, oracle):
    """k = Int.MaxValue - 2 is legal (Sampler.scala:71, :80); 24 B x k of HBM state (51 GB)."""
    from reservoir_amd import Sampler

    k = 2**31 - 1 - 2
    keys = oracle.splitmix_keys(1, 5000)
    s = Sampler(k, seed=1)()
    s.sample_all(keys)
    assert np.array_equal(s.result(), keys)  # n < k: every element, in order (resultImpl :318-331)


@pytest.mark.parametrize("kt", ["long", "int"])
def test_recycled_handle_resources(cuda, oracle, kt):
    """Samplers created after others were closed reuse their pooled slot blocks (rsv_pool.hip and
    the clean-slot cache): no state may leak from the previous owner -- partial fills, empty
    slots in export_state, and full parity all hold for every generation."""
    import torch

    from reservoir_amd import Sampler

    k = 300
    dt = np.int64 if kt == "long" else np.int32
    for gen in range(6):
        n = [100_000, 50, 0, 299, 300, 7_777][gen]
        keys = oracle.splitmix_keys(40_000 + gen, n).astype(dt)
        want, _ = oracle.algo_r(1234 + gen, gen, k, keys.astype(np.int64))
        s = Sampler(k, seed=1234 + gen, stream_id=gen, key_type=kt)()
        if n:
            s.sample_all(_dev_keys(torch, cuda, keys))
        idx, kk, _, cnt = s.export_state(cuda)
        m = min(n, k)
        idx = idx.cpu().numpy()
        assert (idx[m:] == -1).all() and (idx[:m] >= 0).all()
        got = s.result()
        assert got.size == m
        assert np.array_equal(got, want[:m].astype(dt))
        s.close()


@pytest.mark.parametrize("kt", ["long", "int"])
def test_fused_k1_resolve_publish(cuda, oracle, kt):
    """Batches that K1 covers in one launch with k <= 2048 run as one dispatch whose last
    workgroup resolves and publishes (rsv_elements.hip k1_resolve_publish); k = 2049 takes the
    two-kernel form.  The completion ticket is re-armed by every launch: back-to-back samplers
    of different grid sizes, batches inside and across the fill phase, all equal the oracle."""
    import torch

    from reservoir_amd import Sampler

    dt = np.int64 if kt == "long" else np.int32
    rng = np.random.default_rng(7)
    for it in range(24):
        k = [1, 64, 1000, 2047, 2048, 2049][it % 6]
        n = int(rng.integers(0, 3 * 10**6)) if it % 4 else int(rng.integers(0, 3 * k))
        keys = oracle.splitmix_keys(70_000 + it, n).astype(dt)
        want, _ = oracle.algo_r(555 + it, it, k, keys.astype(np.int64))
        s = Sampler(k, seed=555 + it, stream_id=it, key_type=kt)()
        kd = _dev_keys(torch, cuda, keys)
        cuts = np.r_[0, np.sort(rng.choice(np.arange(0, n + 1), 3)), n]
        for a, b in zip(cuts[:-1], cuts[1:]):
            if b > a:
                s.sample_all(kd[a:b])
        got = s.result()
        assert got.size == min(n, k)
        assert np.array_equal(got, want[: got.size].astype(dt)), (it, k, n)


def test_seek_past_k_after_partial_fill(cuda, oracle):
    """A batch that fills part of the reservoir, then a seek past k (the slots of other ranks'
    indices), then result(): min(count, k) keys -- the filled ones, then the empty slots as
    zeros -- never a stale publication of the partial fill (rsv_seek / pub_valid)."""
    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(61, 40)
    for kt, dt in (("long", np.int64), ("int", np.int32)):
        s = Sampler(100, seed=1, key_type=kt)()
        s.sample_all(keys.astype(dt))
        s.seek(5000)
        got = s.result()
        assert got.size == 100
        assert np.array_equal(got[:40], keys.astype(dt)) and (got[40:] == 0).all()


def test_caller_stream_pipelined_samplers(cuda, oracle):
    """On a caller stream every call is stream-ordered and returns without a host wait: a second
    sampler queued behind the first (bench.py's two steps in flight), the next batch on the
    handle, export_packed and result_device must all see the finished slots, and results read one
    step late are each step's own.  keys = arange: each slot's key is its last writer's index."""
    import torch

    from reservoir_amd import Sampler

    n1, n2, k, seed, sid = 200_000_000, 100_000_000, 1024, 77, 3
    keys = torch.arange(n1 + n2, dtype=torch.int64, device=cuda)
    stream = torch.cuda.current_stream().cuda_stream
    want = oracle.algo_r_last_writers(seed, sid, k, 0, n1 + n2)
    want1 = oracle.algo_r_last_writers(seed, sid, k, 0, n1)
    a = Sampler(k, seed=seed, stream_id=sid, reusable=True)()  # result_device, then result()
    a.set_stream(stream)
    a.sample_all(keys[:n1])
    b = Sampler(k, seed=seed, stream_id=sid)()  # queued behind a's work
    b.set_stream(stream)
    b.sample_all(keys[:n1])
    a.sample_all(keys[n1:])
    row = torch.empty(2 * k, dtype=torch.int64, device=cuda)
    a.export_packed(row)
    dev_out = torch.empty(k, dtype=torch.int64, device=cuda)
    assert a.result_device(dev_out) == k
    torch.cuda.synchronize()
    assert np.array_equal(row[:k].cpu().numpy(), want)
    assert np.array_equal(row[k:].cpu().numpy(), want)
    assert np.array_equal(dev_out.cpu().numpy(), want)
    assert np.array_equal(b.result(), want1)
    assert np.array_equal(a.result(), want)
    b.close()
    a.close()
    # pipelined single-use steps, results read one step late
    pending = None
    for step in range(6):
        s = Sampler(k, seed=seed, stream_id=sid)()
        s.set_stream(stream)
        s.sample_all(keys[:n1])
        if pending is not None:
            assert np.array_equal(pending.result(), want1), step
            pending.close()
        pending = s
    assert np.array_equal(pending.result(), want1)
    pending.close()
    del keys
    torch.cuda.empty_cache()


def test_set_stream_hands_over_pending_work(cuda, oracle):
    """rsv_set_stream with work still queued: the new stream is ordered after it by an event wait
    (no host synchronize).  A sampler samples on one torch stream and, with its K1 pass in flight,
    moves to a second stream where its combine kernels (export_packed, merge_packed), a further
    batch and result_device run; then back to the first for result().  keys = arange: each slot's
    key is its last writer's index; the merged rows are two copies of the same state."""
    import torch

    from reservoir_amd import Sampler

    n1, n2, k, seed, sid = 150_000_000, 50_000_000, 1024, 91, 5
    keys = torch.arange(n1 + n2, dtype=torch.int64, device=cuda)
    a_stream, b_stream = torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)
    a_stream.wait_stream(torch.cuda.current_stream())
    b_stream.wait_stream(torch.cuda.current_stream())
    want1 = oracle.algo_r_last_writers(seed, sid, k, 0, n1)
    want = oracle.algo_r_last_writers(seed, sid, k, 0, n1 + n2)
    s = Sampler(k, seed=seed, stream_id=sid, reusable=True)()
    s.set_stream(a_stream.cuda_stream)
    s.sample_all(keys[:n1])  # K1 + resolve queued on a
    s.set_stream(b_stream.cuda_stream)  # pending: b waits for a's record
    with torch.cuda.stream(b_stream):
        rows = torch.empty((2, 2 * k), dtype=torch.int64, device=cuda)
        s.export_packed(rows[0])
        s.export_packed(rows[1])
        s.merge_packed(rows, n1)
        mid = torch.empty(k, dtype=torch.int64, device=cuda)
        assert s.result_device(mid) == k
        s.sample_all(keys[n1:])
    s.set_stream(a_stream.cuda_stream)  # and back, with b's work pending
    got = s.result()
    torch.cuda.synchronize()
    assert np.array_equal(rows[0, :k].cpu().numpy(), want1)
    assert np.array_equal(mid.cpu().numpy(), want1)
    assert np.array_equal(got, want)
    s.close()
    del keys
    torch.cuda.empty_cache()

