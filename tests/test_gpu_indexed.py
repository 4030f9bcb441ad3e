"""sampleAll over an IndexedSeq without its keys (rsv_sample_indexed / rsv_fill_slots): the
reference's sampleIndexed (Sampler.scala:261-273) reads only the elements it evicts with, and the
engine's index-only batch likewise asks the caller for the reservoir's new holders alone.

Checked against the oracle (the same reservoir as every other path, Sampler.scala:117-142's
"sample == sampleAll for every collection shape"), with `map` counted, and the ABI's
IllegalStateException while keys are owed."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
@pytest.mark.parametrize("k,n", [(1, 10), (20, 3000), (1024, 500), (1024, 1024), (1000, 2_000_003)])
def test_indexed_equals_every_other_shape(cuda, oracle, engine, k, n):
    """list / range / numpy array (indexed) == device tensor == per element, same seed; map runs at
    most min(n, k) times per indexed batch."""
    import torch

    from reservoir_amd import Sampler

    keys = oracle.splitmix_keys(k + 17, n)
    got = {}
    calls = [0]

    def counted(x):
        calls[0] += 1
        return x

    s = Sampler(k, seed=5, stream_id=3, engine=engine)(counted)
    s.sample_all(keys.tolist())  # a Python list: IndexedSeq
    assert calls[0] <= min(n, k)
    got["list"] = s.result()
    s = Sampler(k, seed=5, stream_id=3, engine=engine)()
    s.sample_all(keys)  # host numpy array: IndexedSeq
    got["ndarray"] = s.result()
    s = Sampler(k, seed=5, stream_id=3, engine=engine)()
    s.sample_all(torch.from_numpy(keys).to(cuda))
    got["device"] = s.result()
    if engine == "java_l":
        ref = oracle.AlgoL(k, 5)
        ref.sample_all(keys)
        want = ref.result()
    else:
        want, _ = oracle.algo_r(5, 3, k, keys)
    for shape, r in got.items():
        assert np.array_equal(r, want), shape
    # range: the keys are the indices (SamplerTest.scala:117-142 samples 1 to 3000)
    s = Sampler(k, seed=5, stream_id=3, engine=engine)()
    s.sample_all(range(1, n + 1))
    if engine == "java_l":
        ref = oracle.AlgoL(k, 5)
        ref.sample_all_iota(1, n)
        want = ref.result()
    else:
        want, _ = oracle.algo_r(5, 3, k, np.arange(1, n + 1, dtype=np.int64))
    assert np.array_equal(s.result(), want)


def test_indexed_mixed_with_other_batches(cuda, oracle):
    """Per-element samples, device batches and indexed batches interleaved in one stream, reusable
    result() between: identical to one pass over the concatenation."""
    import torch

    from reservoir_amd import Sampler

    k = 256
    keys = oracle.splitmix_keys(3, 900_000)
    want, _ = oracle.algo_r(11, 12, k, keys)
    s = Sampler(k, seed=11, stream_id=12, reusable=True)()
    cuts = [0, 7, 100, 300, 40_000, 41_000, 500_000, 900_000]
    for i, (a, b) in enumerate(zip(cuts, cuts[1:])):
        part = keys[a:b]
        if i % 3 == 0:
            for x in part.tolist():
                s.sample(x)
        elif i % 3 == 1:
            s.sample_all(part)  # indexed
        else:
            s.sample_all(torch.from_numpy(part).to(cuda))
        r, _ = oracle.algo_r(11, 12, k, keys[:b])
        assert np.array_equal(s.result(), r), (a, b)
    assert np.array_equal(s.result(), want)


def test_indexed_c2_shape_maps_only_winners(cuda, oracle):
    """C2's shape (1e9 elements, k = 1024) as a Python range: one K1 pass over the indices, map on
    the <= 1024 winners, reservoir = the oracle's last writers."""
    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    calls = [0]

    def counted(x):
        calls[0] += 1
        return x

    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)(counted)
    s.sample_all(range(n))
    assert calls[0] <= k
    win = oracle.algo_r_last_writers(0xC0FFEE, 0x5A5A, k, 0, n)
    assert np.array_equal(s.result(), win)


def test_keys_owed_state(cuda):
    """Between rsv_sample_indexed and rsv_fill_slots every other call is an IllegalStateException;
    fill_slots with nothing owed is one too; n = 0 reports no change."""
    from reservoir_amd import Sampler, _native as N

    L = N.load()
    s = Sampler(16, seed=1)()
    offs = np.empty(16, dtype=np.int64)
    N.check(L.rsv_sample_indexed(s.handle, 0, offs.ctypes.data_as(C.c_void_p)))
    assert (offs == -1).all()
    N.check(L.rsv_sample_indexed(s.handle, 40, offs.ctypes.data_as(C.c_void_p)))
    assert sorted(offs[offs >= 0].tolist()) == sorted(set(offs[offs >= 0].tolist())) and (offs >= 0).all()
    out = np.empty(16, dtype=np.int64)
    n = C.c_int64()
    assert L.rsv_result(s.handle, out.ctypes.data_as(C.c_void_p), 16, C.byref(n)) == N.E_ILLEGAL_STATE
    assert L.rsv_sample_batch(s.handle, out.ctypes.data_as(C.c_void_p), 1, N.MEM_HOST, None) == N.E_ILLEGAL_STATE
    keys = (offs + 1000).astype(np.int64)
    N.check(L.rsv_fill_slots(s.handle, keys.ctypes.data_as(C.c_void_p)))
    assert L.rsv_fill_slots(s.handle, keys.ctypes.data_as(C.c_void_p)) == N.E_ILLEGAL_STATE
    r = s.result()
    assert np.array_equal(r, keys)
    d = Sampler.distinct(8)()
    assert L.rsv_sample_indexed(d.handle, 5, offs.ctypes.data_as(C.c_void_p)) == N.E_UNSUPPORTED


@pytest.mark.parametrize("engine", ["philox_r", "java_l"])
def test_throwing_map_aborts_the_batch(cuda, oracle, engine):
    """A `map` that throws inside sampleAll(IndexedSeq): the exception propagates, the owed batch is
    dropped (rsv_abort_indexed), and the sampler keeps working -- equal to one that never saw that
    batch (the handle used to stay stuck in IllegalStateException)."""
    from reservoir_amd import Sampler

    k = 64

    class Boom(Exception):
        pass

    def bad(x):
        if x >= 500:
            raise Boom(x)
        return x

    for fresh in (True, False):
        s = Sampler(k, engine=engine, seed=3, stream_id=4)(bad)
        ref = Sampler(k, engine=engine, seed=3, stream_id=4)(bad)
        if not fresh:
            s.sample_all(range(200))
            ref.sample_all(range(200))
        with pytest.raises(Boom):
            s.sample_all(range(100_000))  # evictions land far past 500: map throws
        assert s.is_open and s.count == (0 if fresh else 200)
        s.sample_all(range(300))
        ref.sample_all(range(300))
        assert np.array_equal(s.result(), ref.result())
    from reservoir_amd import _native as N

    L = N.load()
    s = Sampler(8)()
    assert L.rsv_abort_indexed(s.handle) == N.E_ILLEGAL_STATE
