"""Zero-copy pinned batches (rsv_stage_acquire / rsv_stage_commit): keys written straight into the
handle's pinned staging buffer give the same reservoir as per-element rsv_sample and as sampleAll."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _stage_all(L, N, h, keys, hashes=None, step=None):
    i, n = 0, keys.size
    width = keys.dtype.itemsize
    while i < n:
        buf, hb, cap = C.c_void_p(), C.c_void_p(), C.c_int64()
        N.check(L.rsv_stage_acquire(h, C.byref(buf), C.byref(hb), C.byref(cap)))
        assert cap.value > 0
        c = min(cap.value, n - i, step or n)
        C.memmove(buf.value, keys[i:i + c].ctypes.data, c * width)
        if hashes is not None:
            assert hb.value
            C.memmove(hb.value, hashes[i:i + c].ctypes.data, c * 8)
        else:
            assert not hb.value
        N.check(L.rsv_stage_commit(h, c))
        i += c


@pytest.mark.parametrize("k,n,step", [(1024, 3_000_000, None), (7, 50_000, 333), (100_000, 2_500_000, 1 << 20)])
def test_stage_commit_parity(cuda, oracle, k, n, step):
    from reservoir_amd import Sampler, _native as N

    L = N.load()
    keys = oracle.splitmix_keys(k + n, n)
    want, _ = oracle.algo_r(12, 34, k, keys)
    s = Sampler(k, seed=12, stream_id=34)()
    _stage_all(L, N, s.handle, keys[: n // 2], step=step)
    s.sample_all(keys[n // 2: n // 2 + 1000])            # interleaved with a bulk batch
    for x in keys[n // 2 + 1000: n // 2 + 1100]:         # and per-element calls
        s.sample(int(x))
    _stage_all(L, N, s.handle, keys[n // 2 + 1100:], step=step)
    assert np.array_equal(s.result(), want)


def test_stage_commit_distinct_precomputed_and_errors(cuda, oracle):
    from reservoir_amd import IllegalArgumentException, Sampler, _native as N

    L = N.load()
    xs = np.arange(20_000, dtype=np.int64)
    d = Sampler.distinct(30, seed=2)(hash=lambda x: x * 31 + 7)
    _stage_all(L, N, d.handle, xs, hashes=xs * 31 + 7, step=4096)
    ref = oracle.Distinct(30, 2, oracle.HASH_IDENTITY)
    ref.sample_all(xs * 31 + 7)
    assert sorted(d.result().tolist()) == sorted(((x - 7) // 31) for x in ref.result()[0].tolist())
    s = Sampler(10)()
    buf, cap = C.c_void_p(), C.c_int64()
    N.check(L.rsv_stage_acquire(s.handle, C.byref(buf), None, C.byref(cap)))
    with pytest.raises(IllegalArgumentException):
        N.check(L.rsv_stage_commit(s.handle, cap.value + 1))
    with pytest.raises(IllegalArgumentException):
        N.check(L.rsv_stage_commit(s.handle, -1))
