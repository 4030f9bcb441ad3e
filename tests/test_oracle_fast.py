"""The oracle's full-size forms agree with its sequential restatement (CPU only).

or_algo_r_last_writers (the exact R2 shortcut, threaded) must give or_algo_r's res_idx bit for
bit: it is what the full-size C2 GPU check (tests/test_gpu_configs.py) compares against.
"""
import ctypes as C

import numpy as np
import pytest


@pytest.mark.parametrize("k,i0,n", [(1, 0, 5000), (7, 0, 100_000), (1024, 0, 600_000), (100, 3, 2_000_003),
                                    (64, 0, 4096), (1 << 12, 1 << 20, 1_500_000), (1024, 2**32 - 77, 900_001),
                                    (3, 2**40, 1_200_000), (5000, 2_000, 10)])
def test_last_writers_equal_sequential(oracle, k, i0, n):
    keys = np.arange(n, dtype=np.int64)
    res = np.zeros(k, dtype=np.int64)
    idx = np.full(k, -1, dtype=np.int64)
    oracle.lib().or_algo_r(11, 22, k, i0, keys, n, res, idx.ctypes.data_as(C.c_void_p))
    for threads in (1, 3, 0):
        got = oracle.algo_r_last_writers(11, 22, k, i0, n, threads)
        assert np.array_equal(got, idx), threads


def test_segmented_timer_runs_reference_samplers(oracle):
    """The C3 CPU leg's threaded Algorithm-L samplers equal one AlgoL per stream (seed = stream)."""
    S, L, k = 12, 3000, 20
    keys = oracle.splitmix_keys(9, S * L)
    for mode in (0, 1):
        out = np.zeros(S * k, dtype=np.int64)
        t = oracle.lib().or_time_segmented_algo_l(k, keys, S, L, mode, 3, out.ctypes.data_as(C.c_void_p))
        assert t >= 0
        for s in range(S):
            a = oracle.AlgoL(k, s)
            a.sample_all(keys[s * L:(s + 1) * L])
            assert np.array_equal(out[s * k:(s + 1) * k], a.result())


@pytest.mark.parametrize("k,base,n", [(20, 1, 3000), (1, 0, 10), (100, -5, 1_000_000), (1024, 7, 500)])
def test_iota_walk_equals_indexed_walk(oracle, k, base, n):
    """or_algo_l_sample_all_iota (the sampleIndexed walk over a Range, no element array) reads the
    elements or_algo_l_sample_all_indexed reads: same reservoir, in one call and in three; for
    SamplerTest.scala:117-142's setup (k = 20, 1 to 3000, Random(0)) the survey's vector."""
    a = oracle.AlgoL(k, 3)
    a.sample_all(np.arange(base, base + n, dtype=np.int64))
    b = oracle.AlgoL(k, 3)
    b.sample_all_iota(base, n)
    c = oracle.AlgoL(k, 3)
    cuts = [0, n // 3, n // 2, n]
    for lo, hi in zip(cuts, cuts[1:]):
        c.sample_all_iota(base + lo, hi - lo)
    assert np.array_equal(a.result(), b.result()) and np.array_equal(a.result(), c.result())
    if (k, base, n) == (20, 1, 3000):
        d = oracle.AlgoL(20, 0)
        d.sample_all_iota(1, 3000)
        assert d.result().tolist() == [1335, 1173, 2365, 2555, 705, 392, 612, 786, 1639, 2529, 2575, 2058,
                                       176, 780, 339, 607, 1147, 1511, 1218, 222]
