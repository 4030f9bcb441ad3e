"""result() without the host copy (rsv_result_take / rsv_host_release): a single-use sampler hands
its pinned result buffer to the returned array.  The keys equal rsv_result's (the copy path, same
seed), the array outlives the sampler and every later buffer reuse, views keep the buffer alive, and
anything else (reusable samplers, results over 1 MB) reports RSV_E_UNSUPPORTED and copies."""
import ctypes as C
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _copy_result(s):
    from reservoir_amd import _native as N

    out = np.empty(s.max_sample_size, dtype=np.int64)
    n = C.c_int64()
    N.check(N.load().rsv_result(s.handle, out.ctypes.data_as(C.c_void_p), s.max_sample_size, C.byref(n)))
    return out[: n.value]


@pytest.mark.parametrize("kind", ["elements", "distinct_set", "distinct_ordered"])
def test_take_equals_copy_and_outlives_the_sampler(cuda, oracle, kind):
    import torch

    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(41, 300_000)
    kd = torch.from_numpy(keys).to(cuda)

    def make():
        if kind == "elements":
            return Sampler(1000, seed=9)()
        if kind == "distinct_set":
            return Sampler.distinct(4096, seed=9)(hash="identity")
        return Sampler.distinct(4096, seed=9)()

    a, b = make(), make()
    a.sample_all(kd)
    b.sample_all(kd)
    got = a.result()  # handed over
    want = _copy_result(b)
    assert np.array_equal(got, want)
    view = got[7:]
    a.close()
    del got
    gc.collect()
    # the pool hands buffers out again: the taken one must not be among them while `view` lives
    for i in range(6):
        c = make()
        c.sample_all(kd[i * 1000:])
        c.result()
        c.close()
    assert np.array_equal(view, want[7:])
    del view
    gc.collect()


def test_take_unsupported_falls_back(cuda, oracle):
    from reservoir_amd import Sampler, _native as N

    L = N.load()
    keys = oracle.splitmix_keys(5, 50_000)
    r = Sampler(64, seed=1, reusable=True)()
    r.sample_all(keys)
    buf, n = C.c_void_p(), C.c_int64()
    assert L.rsv_result_take(r.handle, C.byref(buf), C.byref(n)) == N.E_UNSUPPORTED
    assert np.array_equal(r.result(), r.result())  # reusable: still open, copies
    big = Sampler(1 << 18, seed=1)()  # 2 MB of keys: over the published-result limit
    big.sample_all(keys)
    assert L.rsv_result_take(big.handle, C.byref(buf), C.byref(n)) == N.E_UNSUPPORTED
    assert big.is_open  # untouched
    res = big.result()
    assert res.size == keys.size and np.array_equal(np.sort(res), np.sort(keys))
    assert not big.is_open


def test_take_closes_and_empty(cuda):
    from reservoir_amd import IllegalStateException, Sampler

    s = Sampler(16, seed=2)()
    r = s.result()  # nothing sampled
    assert r.size == 0 and not s.is_open
    with pytest.raises(IllegalStateException):
        s.sample(1)
    d = Sampler.distinct(16, seed=2)()
    d.sample_all(np.arange(5, dtype=np.int64))
    assert sorted(d.result().tolist()) == [0, 1, 2, 3, 4]
    with pytest.raises(IllegalStateException):
        d.result()
