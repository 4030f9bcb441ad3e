"""Every BASELINE.json config at its own workload, checked against the oracle (parity at full size).

  C1  10 M Longs, k = 100: philox_r vs sequential Algorithm R; java_l vs the reference's
      Algorithm L (Sampler.scala:248-273); distinct (default Long.hashCode -> ordered, and
      identity -> set) vs RandomValues (Sampler.scala:394-409)
  C2  1e9 Long keys, k = 1024: every slot's last writer (export_state indices) equals the oracle's
      (or_algo_r_last_writers: the exact R2 shortcut of or_algo_r, threaded) -- a dropped late hit
      would leave an earlier index -- and result() holds the keys at those indices
  C3  2^20 streams x 4096 Longs, k = 64, one launch (4.3e9 keys, past 2^32): every 4096th stream
      vs or_algo_r_segmented, every count == 64
  C4  one GPU's share of C4 (5e8 keys, 30 % duplicates, k = 65536) under the default
      Long.hashCode (ordered mode): the set equals the oracle's sequential RandomValues; and a
      hash-twin variant whose boundary hash bucket is oversubscribed, so the host replay runs;
      the share in set mode (hash = identity); and the FULL C4 (4e9 keys) as 8 one-GPU shards
      merged like the 8-GPU run, plus one sampler over >= 2^31-key batches, both hashes
  C5  akka path at k = 1 Mi: zero-copy pinned batches (rsv_stage_acquire/commit) over 3e7 keys and
      the Sample operator (SampleImpl.scala:27-31) vs the oracle; the per-element rsv_sample path
      at k = 1 Mi runs in tests/cpp/test_ffm_sequence.cpp (test_gpu_ffm.py)
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _w():
    import workloads

    return workloads


# ---------------------------------------------------------------------------------------- C1
def test_c1_elements_both_engines(cuda, oracle):
    import torch

    from reservoir_amd import Sampler

    n, k = 10_000_000, 100
    keys = oracle.splitmix_keys(0x5EED0000, n)  # the first 1e7 of the C2 stream
    kd = torch.from_numpy(keys).to(cuda)
    want, _ = oracle.algo_r(0xC0FFEE, 0x5A5A, k, keys)
    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
    s.sample_all(kd)
    assert np.array_equal(s.result(), want)
    ref = oracle.AlgoL(k, 0)
    ref.sample_all(keys)
    s = Sampler(k, engine="java_l", seed=0)()
    s.sample_all(kd)
    assert np.array_equal(s.result(), ref.result())


@pytest.mark.parametrize("hash_kind", ["default", "identity"])
def test_c1_distinct(cuda, oracle, hash_kind):
    import torch

    from reservoir_amd import Sampler

    n, k = 10_000_000, 100
    keys = oracle.splitmix_keys(0x5EED0000, n)
    keys[n // 2:] = keys[: n - n // 2][::-1]  # every element twice
    ref = oracle.Distinct(k, 3, oracle.HASH_JAVA_LONG if hash_kind == "default" else oracle.HASH_IDENTITY)
    ref.sample_all(keys)
    mk = Sampler.distinct(k, seed=3)
    d = mk() if hash_kind == "default" else mk(hash="identity")
    d.sample_all(torch.from_numpy(keys).to(cuda))
    assert sorted(d.result().tolist()) == sorted(ref.result()[0].tolist())


# ---------------------------------------------------------------------------------------- C2
def test_c2_full_size_last_writers(cuda, oracle):
    import torch

    from reservoir_amd import Sampler

    n, k, seed, stream = 1_000_000_000, 1024, 0xC0FFEE, 0x5A5A
    keys = torch.empty(n, dtype=torch.int64, device=cuda)
    _w().splitmix_fill(keys, 0x5EED0000)
    s = Sampler(k, seed=seed, stream_id=stream)()
    s.sample_all(keys)
    idx, _, _, _ = s.export_state(cuda)
    got_idx = idx.cpu().numpy()
    want_idx = oracle.algo_r_last_writers(seed, stream, k, 0, n)
    assert np.array_equal(got_idx, want_idx)
    res = s.result()
    f = oracle.lib().or_splitmix64
    assert [int(v) for v in res] == [(f(0x5EED0000 + int(i)) + 2**63) % 2**64 - 2**63 for i in want_idx]


@pytest.mark.parametrize("lo", [7_000_000_005, 8_000_000_003])
def test_c2_shard_two_group_schedule(cuda, oracle, lo):
    """A C2-sized shard as rank 7 / 8 of the 8-GPU run sees it (index range [lo, lo + 1.1e9)): K1
    takes its two-group schedule of half windows (>= ~1e9 draws, rsv_elements.hip k1_plan) with a
    block-unaligned first and last block; the second range crosses index 2^33, where the resolve
    leaves its FAST form.  Every slot's last writer equals the oracle's."""
    import torch

    from reservoir_amd import Sampler

    n, k, seed, stream = 1_100_000_000, 1024, 0xC0FFEE, 0x5A5A
    keys = torch.empty(n, dtype=torch.int64, device=cuda)
    _w().splitmix_fill(keys, 0x77)
    s = Sampler(k, seed=seed, stream_id=stream)()
    s.seek(lo)
    s.sample_all(keys)
    idx, _, _, _ = s.export_state(cuda)
    want_idx = oracle.algo_r_last_writers(seed, stream, k, lo, n)
    assert np.array_equal(idx.cpu().numpy(), want_idx)
    assert (want_idx >= lo).sum() > 50  # ~n / (lo + n) of the slots get a writer in the range


# ---------------------------------------------------------------------------------------- C3
def test_c3_full_launch(cuda, oracle):
    import torch

    from reservoir_amd import batch

    S, L, k, seed = 1 << 20, 4096, 64, 1
    n = S * L
    keys = torch.empty(n, dtype=torch.int64, device=cuda)
    _w().splitmix_fill(keys, 0)
    offs = torch.arange(0, n + 1, L, dtype=torch.int64, device=cuda)
    out, cnt = batch.sample_segmented(keys, offs, k, seed=seed)
    assert int(cnt.min()) == k and int(cnt.max()) == k
    check = np.arange(0, S, 4096, dtype=np.int64)
    check = np.r_[check, S - 1]
    got = out[torch.from_numpy(check).to(cuda)].cpu().numpy()
    for r, s in enumerate(check):
        host = keys[s * L:(s + 1) * L].cpu().numpy()
        want, wc = oracle.algo_r_segmented(seed, int(s), k, host, np.array([0, L], dtype=np.int64))
        assert wc[0] == k
        assert np.array_equal(got[r], want[0]), s
    del keys
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------------------- C4
def _scrambled(torch, keys, r0, r1):
    """RandomValues' hash (Sampler.scala:396) of Long.hashCode, on the device."""
    C1 = 0x9E3779B97F4A7C15 - (1 << 64)

    def bswap(v):
        return v.contiguous().view(torch.uint8).view(-1, 8).flip(1).contiguous().view(torch.int64).view(-1)

    def byteswap64(v):
        return bswap(v * C1) * C1

    hc = (((keys ^ ((keys >> 32) & 0xFFFFFFFF)) & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000  # (int) cast
    return byteswap64(r1 ^ byteswap64(r0 ^ hc))


@pytest.mark.parametrize("variant,seed", [("c4", 7), ("twins", 11)])
def test_c4_share_ordered(cuda, oracle, variant, seed):
    import torch

    from reservoir_amd import Sampler

    n, k = 500_000_000, 65536
    W = _w()
    vals = W.c4_data(n, cuda)
    if variant == "twins":
        vals = W.hash_twins(vals, 26)  # ~5 distinct keys per Long.hashCode value
    torch.cuda.synchronize()
    d = Sampler.distinct(k, seed=seed)()  # default hash (Long.hashCode) -> ordered mode
    d.sample_all(vals)
    got = d.result()
    host = vals.cpu().numpy()
    ref = oracle.Distinct(k, seed, oracle.HASH_JAVA_LONG)
    ref.sample_all(host)
    want, wh = ref.result()
    assert got.size == k
    assert np.array_equal(np.sort(got), np.sort(want))
    if variant == "twins":
        # the boundary bucket is oversubscribed: more distinct keys share the final maximum hash
        # than the set keeps, so the set depends on arrival order + heap ties (the host replay)
        top = int(wh.max())
        h = _scrambled(torch, vals, ref.r0, ref.r1)
        tied = torch.unique(vals[h == top]).numel()
        assert tied > int((wh == top).sum()), (tied, int((wh == top).sum()))
    del vals
    torch.cuda.empty_cache()


def test_c4_share_set_mode_identity(cuda, oracle):
    """C4's per-GPU share (5e8 keys, k = 65536) with hash = identity (set mode: analytic threshold,
    bucketed merge, speculative publication): the set equals the oracle's RandomValues."""
    from reservoir_amd import Sampler

    n, k = 500_000_000, 65536
    vals = _w().c4_data(n, cuda)
    d = Sampler.distinct(k, seed=7)(hash="identity")
    d.sample_all(vals)
    got = d.result()
    ref = oracle.Distinct(k, 7, oracle.HASH_IDENTITY)
    ref.sample_all(vals.cpu().numpy())
    assert got.size == k
    assert np.array_equal(np.sort(got), np.sort(ref.result()[0]))


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_c4_full_workload_8way(cuda, oracle):
    """C4 at its own workload (BASELINE.json configs[3]): 4e9 Long keys, 30 % duplicates,
    k = 65536, split 8 ways -- 8 distinct samplers on one GPU, each fed one contiguous 5e8 piece
    (= one rank of the 8-GPU run), merged with distributed.merge_local (export_packed -> the device
    merge_packed, plus the exact ordered replay for the default hash).  Also one sampler fed the whole stream in
    two batches of >= 2^31 keys (the chunk loop).  Both hashes vs the oracle's sequential
    RandomValues over all 4e9 keys (Sampler.scala:383-412)."""
    import threading

    import torch

    from reservoir_amd import Sampler
    from reservoir_amd import distributed as D

    n, k, parts, seed = 4_000_000_000, 65536, 8, 7
    keys = torch.empty(n, dtype=torch.int64, device=cuda)
    _w().c4_slice(n, 0, n, cuda, out=keys)
    torch.cuda.synchronize()
    refs = {"identity": oracle.Distinct(k, seed, oracle.HASH_IDENTITY),
            "default": oracle.Distinct(k, seed, oracle.HASH_JAVA_LONG)}
    step = 250_000_000
    for a in range(0, n, step):  # the oracle over the whole sequence, both hashes side by side
        host = keys[a:a + step].cpu().numpy()
        ts = [threading.Thread(target=r.sample_all, args=(host,)) for r in refs.values()]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    piece = n // parts
    cut = (1 << 31) + 12_345
    for name, ref in refs.items():
        want = np.sort(ref.result()[0])
        mk = Sampler.distinct(k, seed=seed, retain_log=name == "default")
        make = (lambda: mk(hash="identity")) if name == "identity" else (lambda: mk())
        shards = []
        for r in range(parts):
            s = make()
            s.sample_all(keys[r * piece:(r + 1) * piece])
            shards.append(s)
        target = make()
        D.merge_local(target, shards)
        assert target.count == n
        assert np.array_equal(np.sort(target.result()), want), name
        single = make()
        single.sample_all(keys[:cut])
        single.sample_all(keys[cut:])
        assert np.array_equal(np.sort(single.result()), want), name
        del shards, target, single
    del keys
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------------------- C5
def test_c5_staged_batches_k1mi(cuda, oracle):
    """rsv_stage_acquire/commit (the FFM zero-copy path of INTEGRATION.md) at C5's k = 1 Mi."""
    from reservoir_amd import Sampler, _native as N

    n, k, seed, stream = 30_000_000, 1 << 20, 5, 6
    keys = oracle.splitmix_keys(0x5EED0000, n)
    L = N.load()
    s = Sampler(k, seed=seed, stream_id=stream)()
    i = 0
    while i < n:
        buf, cap = C.c_void_p(), C.c_int64()
        N.check(L.rsv_stage_acquire(s.handle, C.byref(buf), None, C.byref(cap)))
        c = min(cap.value, n - i, 777_777)  # commits that straddle the 1 Mi staging buffers
        C.memmove(buf.value, keys[i:i + c].ctypes.data, c * 8)
        N.check(L.rsv_stage_commit(s.handle, c))
        i += c
    got = s.result()
    win = oracle.algo_r_last_writers(seed, stream, k, 0, n)
    assert (win >= 0).all()
    assert np.array_equal(got, keys[win])


def test_c5_sample_operator_k1mi(cuda, oracle):
    """The Sample operator (SampleImpl: grab -> sampler.sample -> push, per element) at k = 1 Mi."""
    from reservoir_amd import Sample

    n, k = 2_500_000, 1 << 20
    keys = oracle.splitmix_keys(0xA11A, n)
    flow = Sample(k, seed=21, stream_id=3)()
    out, fut = flow.run(keys.tolist())
    passed = sum(1 for _ in out)
    assert passed == n
    win = oracle.algo_r_last_writers(21, 3, k, 0, n)
    assert np.array_equal(fut.result(), keys[win])
    want_l = oracle.AlgoL(k, 4)
    want_l.sample_all(keys)
    flow = Sample(k, engine="java_l", seed=4)()
    out, fut = flow.run(keys.tolist())
    for _ in out:
        pass
    assert np.array_equal(fut.result(), want_l.result())
