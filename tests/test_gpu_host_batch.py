"""Host-keyed element batches move only their winners (round 6): rsv_sample_batch(RSV_MEM_HOST) on an
ELEMENTS sampler samples the batch by index (K1 / the Algorithm-L events), the host copies the <= k
winning keys out of the caller's buffer, and one kernel reads them across PCIe; a staged batch
(rsv_sample / rsv_stage_commit) whose expected winners are few is resolved in place from the
pinned staging buffer.  Every form must give the oracle's reservoir (Sampler.scala:243-273; draw
format R2 / java.util.Random Algorithm L), whatever the batching, and with a resolve stream set."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host_batch(L, N, h, keys):
    a = np.ascontiguousarray(keys)
    n = a.shape[0]
    N.check(L.rsv_sample_batch(h, a.ctypes.data_as(C.c_void_p), n, N.MEM_HOST, None))


def _stage_all(L, N, h, keys, step=None):
    """keys written straight into the handle's pinned staging buffer (rsv_stage_acquire/commit)"""
    i, n = 0, keys.size
    while i < n:
        buf, cap = C.c_void_p(), C.c_int64()
        N.check(L.rsv_stage_acquire(h, C.byref(buf), None, C.byref(cap)))
        c = min(cap.value, n - i, step or n)
        C.memmove(buf.value, keys[i:i + c].ctypes.data, c * 8)
        N.check(L.rsv_stage_commit(h, c))
        i += c


def _want(oracle, engine, k, keys, seed=12, stream=34):
    if engine == "philox_r":
        return oracle.algo_r(seed, stream, k, keys)[0]
    ref = oracle.AlgoL(k, seed)
    ref.sample_all(keys)
    return ref.result()


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
@pytest.mark.parametrize("k,cuts", [(1, [0, 5, 1000, 300_000]), (100, [0, 50, 99, 100, 250_000]),
                                    (1024, [0, 3000, 1_000_000]), (8192, [0, 8191, 500_000]),
                                    (10_000, [0, 4000, 600_000])])
def test_host_batches_winners_only(cuda, oracle, engine, k, cuts):
    from reservoir_amd import Sampler, _native as N

    L = N.load()
    n = cuts[-1]
    keys = oracle.splitmix_keys(77 + k, n)
    s = Sampler(k, seed=12, stream_id=34, engine=engine)()
    for a, b in zip(cuts[:-1], cuts[1:]):
        _host_batch(L, N, s.handle, keys[a:b])
    assert np.array_equal(s.result(), _want(oracle, engine, k, keys))


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
def test_host_batch_mixed_with_every_other_form(cuda, oracle, engine):
    """host batches between device batches, per-element calls, staged commits and index-only
    batches: one global index order, one reservoir"""
    import torch

    from reservoir_amd import Sampler, _native as N

    L = N.load()
    k, n = 4096, 3_000_000
    keys = oracle.splitmix_keys(5, n)
    s = Sampler(k, seed=12, stream_id=34, engine=engine)()
    _host_batch(L, N, s.handle, keys[:1000])                   # fill phase, host
    s.sample_all(torch.from_numpy(keys[1000:500_000]).to(cuda))  # device
    _host_batch(L, N, s.handle, keys[500_000:1_200_000])       # host
    for x in keys[1_200_000:1_200_300]:                         # per element (staged)
        s.sample(int(x))
    s.sample_all(keys[1_200_300:2_000_000])                     # IndexedSeq (index-only + fill)
    _host_batch(L, N, s.handle, keys[2_000_000:])              # host again
    assert np.array_equal(s.result(), _want(oracle, engine, k, keys))


def test_host_and_staged_batches_with_resolve_stream(cuda, oracle):
    """with a resolve stream set, a forked resolve must not read keys a later batch has
    already overwritten -- host batches at k = 4096 (no fused K1 + resolve), staged batches both in
    place and through the device chunk (k = 100000: the first flushes copy), device batches after"""
    import torch

    from reservoir_amd import Sampler, _native as N

    L = N.load()
    side = torch.cuda.Stream(device=cuda).cuda_stream
    for k, n in ((4096, 2_500_000), (100_000, 4_500_000)):
        keys = oracle.splitmix_keys(9 + k, n)
        s = Sampler(k, seed=12, stream_id=34)()
        s.set_resolve_stream(side)
        third = n // 3
        # staged (rsv_sample per element fills 1 Mi-key pinned batches, flushed asynchronously)
        _stage_all(L, N, s.handle, keys[:third])
        _host_batch(L, N, s.handle, keys[third:2 * third])
        t = torch.from_numpy(keys[2 * third:]).to(cuda)
        s.sample_all(t)
        del t  # the forked resolve still reads it: record_stream keeps the block
        torch.cuda.empty_cache()
        junk = torch.full((n,), -1, dtype=torch.int64, device=cuda)  # would reuse a freed block
        assert np.array_equal(s.result(), oracle.algo_r(12, 34, k, keys)[0])
        del junk


def test_wide_element_host_batches(cuda, oracle):
    """16- and 24-byte element keys from host memory: the winners' rows only"""
    from reservoir_amd import Sampler

    for width in (16, 24):
        k, n = 1000, 400_000
        rng = np.random.default_rng(width)
        rows = rng.integers(0, 256, size=(n, width), dtype=np.uint8)
        s = Sampler(k, seed=3, stream_id=4, key_type=f"bytes{width}")()
        s.sample_all(rows[:777])
        s.sample_all(rows[777:])
        win = oracle.algo_r_last_writers(3, 4, k, 0, n)
        assert np.array_equal(s.result(), rows[win])


def test_staged_in_place_large_reservoir(cuda, oracle):
    """k = 1 Mi (C5's reservoir): early flushes copy the batch (many winners), later ones resolve in
    place; both engines"""
    from reservoir_amd import Sampler, _native as N

    L = N.load()
    k, n = 1 << 20, 40 << 20
    keys = oracle.splitmix_keys(1, n)
    for engine in ("philox_r", "java_l"):
        s = Sampler(k, seed=12, stream_id=34, engine=engine)()
        _stage_all(L, N, s.handle, keys, step=1 << 20)
        assert np.array_equal(s.result(), _want(oracle, engine, k, keys))
