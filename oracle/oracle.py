"""ctypes wrapper of the CPU oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package (reservoir_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

HASH_IDENTITY, HASH_JAVA_LONG, HASH_JAVA_INT = 0, 1, 2

i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class _AlgoL(C.Structure):
    _fields_ = [
        ("k", C.c_int32), ("count", C.c_int64), ("W", C.c_double),
        ("next_sample_count", C.c_int64), ("rand", C.c_uint64),
        ("samples", C.POINTER(C.c_int64)),
        ("ev_pos", C.POINTER(C.c_int64)), ("ev_slot", C.POINTER(C.c_int32)),
        ("ev_n", C.c_int64), ("ev_cap", C.c_int64),
    ]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
        os.path.join(_HERE, "oracle.c")
    ):
        build()
    L = C.CDLL(_LIB_PATH)
    L.or_jr_init.argtypes = [C.c_void_p, C.c_int64]
    L.or_jr_next_int.argtypes = [C.c_void_p]; L.or_jr_next_int.restype = C.c_int32
    L.or_jr_next_int_bound.argtypes = [C.c_void_p, C.c_int32]; L.or_jr_next_int_bound.restype = C.c_int32
    L.or_jr_next_long.argtypes = [C.c_void_p]; L.or_jr_next_long.restype = C.c_int64
    L.or_jr_next_double.argtypes = [C.c_void_p]; L.or_jr_next_double.restype = C.c_double
    L.or_byteswap64.argtypes = [C.c_int64]; L.or_byteswap64.restype = C.c_int64
    L.or_java_long_hashcode.argtypes = [C.c_int64]; L.or_java_long_hashcode.restype = C.c_int64
    L.or_algo_l_init.argtypes = [C.POINTER(_AlgoL), C.c_int32, C.c_int64, C.c_int64]
    L.or_algo_l_init.restype = C.c_int
    L.or_algo_l_free.argtypes = [C.POINTER(_AlgoL)]
    L.or_algo_l_sample.argtypes = [C.POINTER(_AlgoL), C.c_int64]
    L.or_algo_l_sample_all_indexed.argtypes = [C.POINTER(_AlgoL), i64p, C.c_int64]
    L.or_algo_l_sample_all_iota.argtypes = [C.POINTER(_AlgoL), C.c_int64, C.c_int64]
    L.or_algo_l_result.argtypes = [C.POINTER(_AlgoL), i64p]; L.or_algo_l_result.restype = C.c_int64
    L.or_distinct_new.argtypes = [C.c_int32, C.c_int64, C.c_int]; L.or_distinct_new.restype = C.c_void_p
    L.or_distinct_free.argtypes = [C.c_void_p]
    L.or_distinct_sample.argtypes = [C.c_void_p, C.c_int64]
    L.or_distinct_sample_array.argtypes = [C.c_void_p, i64p, C.c_int64]
    L.or_distinct_result.argtypes = [C.c_void_p, i64p, i64p]; L.or_distinct_result.restype = C.c_int64
    L.or_distinct_r0.argtypes = [C.c_void_p]; L.or_distinct_r0.restype = C.c_int64
    L.or_distinct_r1.argtypes = [C.c_void_p]; L.or_distinct_r1.restype = C.c_int64
    L.or_distinct_scramble.argtypes = [C.c_int64, C.c_int64, C.c_int64]
    L.or_distinct_scramble.restype = C.c_int64
    u64v = C.c_void_p
    L.or_drows_new.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.c_int]; L.or_drows_new.restype = C.c_void_p
    L.or_drows_free.argtypes = [C.c_void_p]
    L.or_drows_sample.argtypes = [C.c_void_p, u64v, C.c_int64]
    L.or_drows_sample_array.argtypes = [C.c_void_p, u64v, u64v, C.c_int64]
    L.or_drows_result.argtypes = [C.c_void_p, u64v, u64v]; L.or_drows_result.restype = C.c_int64
    L.or_uuid_hashcode.argtypes = [C.c_uint64, C.c_uint64]; L.or_uuid_hashcode.restype = C.c_int64
    L.or_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.or_draw_u64.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]; L.or_draw_u64.restype = C.c_uint64
    L.or_draw_j.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]; L.or_draw_j.restype = C.c_uint64
    L.or_export_draws.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int64, u64p]
    L.or_algo_r.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, i64p, C.c_int64, i64p,
                            C.c_void_p]
    L.or_algo_r.restype = C.c_int64
    L.or_algo_r_replay.argtypes = [C.c_int32, C.c_uint64, u64p, i64p, C.c_int64, i64p]
    L.or_algo_r_segmented.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, i64p, i64p, C.c_int64, i64p, i64p]
    L.or_time_algo_l_per_element.argtypes = [C.c_int32, C.c_int64, i64p, C.c_int64, C.c_int64, C.c_void_p]
    L.or_time_algo_l_per_element.restype = C.c_double
    L.or_time_algo_l_indexed.argtypes = [C.c_int32, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]
    L.or_time_algo_l_indexed.restype = C.c_double
    L.or_time_distinct.argtypes = [C.c_int32, C.c_int64, C.c_int, i64p, C.c_int64]
    L.or_time_distinct.restype = C.c_double
    L.or_algo_r_last_writers.argtypes = [C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64, C.c_int64, i64p,
                                         C.c_int]
    L.or_time_segmented_algo_l.argtypes = [C.c_int32, i64p, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                           C.c_void_p]
    L.or_time_segmented_algo_l.restype = C.c_double
    L.or_splitmix64.argtypes = [C.c_uint64]; L.or_splitmix64.restype = C.c_uint64
    L.or_fill_splitmix.argtypes = [C.c_uint64, C.c_int64, i64p]
    _lib = L
    return L


# ---------------------------------------------------------------------------------------------
class JavaRandom:
    """java.util.Random restatement (oracle)."""

    def __init__(self, seed: int):
        self._state = C.c_uint64(0)
        lib().or_jr_init(C.byref(self._state), seed)

    def next_int(self, bound: int | None = None) -> int:
        if bound is None:
            return lib().or_jr_next_int(C.byref(self._state))
        return lib().or_jr_next_int_bound(C.byref(self._state), bound)

    def next_long(self) -> int:
        return lib().or_jr_next_long(C.byref(self._state))

    def next_double(self) -> float:
        return lib().or_jr_next_double(C.byref(self._state))


class AlgoL:
    """Algorithm L sampler (Sampler.scala:196-331), seeded like SamplerTest.useConsistentRandom."""

    def __init__(self, k: int, seed: int = 0, event_cap: int = 1 << 20):
        self._s = _AlgoL()
        rc = lib().or_algo_l_init(C.byref(self._s), k, seed, event_cap)
        if rc != 0:
            raise ValueError("bad k")
        self.k = k

    def __del__(self):
        try:
            lib().or_algo_l_free(C.byref(self._s))
        except Exception:
            pass

    def sample(self, x: int) -> None:
        lib().or_algo_l_sample(C.byref(self._s), int(x))

    def sample_all(self, xs) -> None:
        a = np.ascontiguousarray(np.asarray(xs, dtype=np.int64))
        lib().or_algo_l_sample_all_indexed(C.byref(self._s), a, a.size)

    def sample_all_iota(self, base_value: int, n: int) -> None:
        """sampleAll over the Range base_value until base_value + n (the sampleIndexed walk without
        an element array, or_algo_l_sample_all_iota)."""
        lib().or_algo_l_sample_all_iota(C.byref(self._s), int(base_value), int(n))

    def result(self) -> np.ndarray:
        out = np.zeros(self.k, dtype=np.int64)
        m = lib().or_algo_l_result(C.byref(self._s), out)
        return out[:m].copy()

    @property
    def count(self) -> int:
        return self._s.count

    def events(self):
        n = min(self._s.ev_n, self._s.ev_cap)
        pos = np.ctypeslib.as_array(self._s.ev_pos, shape=(self._s.ev_cap,))[:n].copy()
        slot = np.ctypeslib.as_array(self._s.ev_slot, shape=(self._s.ev_cap,))[:n].copy()
        if self._s.ev_n > self._s.ev_cap:
            raise RuntimeError("event log overflow")
        return pos, slot.astype(np.int32)


class Distinct:
    """RandomValues bottom-k sampler (Sampler.scala:383-412)."""

    def __init__(self, k: int, seed: int = 0, hash_kind: int = HASH_IDENTITY):
        self._d = lib().or_distinct_new(k, seed, hash_kind)
        if not self._d:
            raise ValueError("bad k")
        self.k = k

    def __del__(self):
        try:
            lib().or_distinct_free(self._d)
        except Exception:
            pass

    def sample(self, x: int) -> None:
        lib().or_distinct_sample(self._d, int(x))

    def sample_all(self, xs) -> None:
        a = np.ascontiguousarray(np.asarray(xs, dtype=np.int64))
        lib().or_distinct_sample_array(self._d, a, a.size)

    def result(self):
        keys = np.zeros(self.k, dtype=np.int64)
        hs = np.zeros(self.k, dtype=np.int64)
        m = lib().or_distinct_result(self._d, keys, hs)
        return keys[:m].copy(), hs[:m].copy()

    @property
    def r0(self) -> int:
        return lib().or_distinct_r0(self._d)

    @property
    def r1(self) -> int:
        return lib().or_distinct_r1(self._d)


class DistinctRows:
    """RandomValues over fixed-width byte keys (Sampler.scala:383-412 with B = UUID / a case class of
    primitives): rows of ``width`` bytes, equality = equal bytes.  ``hash`` is "precomputed" (the
    caller's per-element Long, passed to sample_all) or "uuid" (java.util.UUID.hashCode of the row,
    laid out [mostSigBits | leastSigBits] as little-endian Longs)."""

    def __init__(self, k: int, seed: int, width: int, hash: str = "precomputed"):
        if width % 8 or width <= 0:
            raise ValueError("width must be a positive multiple of 8")
        self.k, self.width = k, width
        self._d = lib().or_drows_new(k, seed, width // 8, 1 if hash == "uuid" else 0)
        if not self._d:
            raise ValueError("bad k")

    def __del__(self):
        try:
            lib().or_drows_free(self._d)
        except Exception:
            pass

    def sample_all(self, rows, hashes=None) -> None:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.uint8).reshape(-1, self.width))
        hp = None
        if hashes is not None:
            h = np.ascontiguousarray(np.asarray(hashes, dtype=np.int64))
            if h.size != r.shape[0]:
                raise ValueError("one hash per row")
            hp = h.ctypes.data
        lib().or_drows_sample_array(self._d, r.ctypes.data, hp, r.shape[0])

    def result(self):
        """(rows uint8 [m, width], scrambled hashes) sorted by (hash, key words)."""
        rows = np.zeros((self.k, self.width), dtype=np.uint8)
        hs = np.zeros(self.k, dtype=np.int64)
        m = lib().or_drows_result(self._d, rows.ctypes.data, hs.ctypes.data)
        return rows[:m].copy(), hs[:m].copy()


def uuid_hashcode(msb: int, lsb: int) -> int:
    return lib().or_uuid_hashcode(msb & (2**64 - 1), lsb & (2**64 - 1))


def byteswap64(v: int) -> int:
    return lib().or_byteswap64(v)


def scramble(r0: int, r1: int, hashed: int) -> int:
    return lib().or_distinct_scramble(r0, r1, hashed)


def philox4x32_10(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return [o[i] for i in range(4)]


def draw_j(seed: int, stream: int, i: int) -> int:
    return lib().or_draw_j(seed, stream, i)


def draw_u64(seed: int, stream: int, i: int) -> int:
    return lib().or_draw_u64(seed, stream, i)


def export_draws(seed: int, stream: int, i0: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint64)
    lib().or_export_draws(seed, stream, i0, n, out)
    return out


def algo_r(seed: int, stream: int, k: int, keys, i0: int = 0, res=None):
    """Sequential Algorithm R with draw format R2. Returns (reservoir[min(i0+n,k)], replacements)."""
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    if res is None:
        res = np.zeros(k, dtype=np.int64)
    repl = lib().or_algo_r(seed, stream, k, i0, keys, keys.size, res, None)
    m = min(i0 + keys.size, k)
    return res[:m].copy() if m < k else res, repl


def algo_r_last_writers(seed: int, stream: int, k: int, i0: int, n: int, threads: int = 0) -> np.ndarray:
    """Per slot, the global index of its last writer over [i0, i0+n) (-1: none) -- or_algo_r's
    res_idx at full size (exact R2 shortcut, multi-threaded; oracle.c or_algo_r_last_writers)."""
    win = np.empty(k, dtype=np.int64)
    lib().or_algo_r_last_writers(seed, stream, k, i0, n, win, threads)
    return win


def algo_r_replay(k: int, j, keys, i0: int = 0) -> np.ndarray:
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    j = np.ascontiguousarray(np.asarray(j, dtype=np.uint64))
    res = np.zeros(k, dtype=np.int64)
    lib().or_algo_r_replay(k, i0, j, keys, keys.size, res)
    return res[: min(i0 + keys.size, k)]


def algo_r_segmented(seed: int, stream_base: int, k: int, keys, offsets):
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    S = offsets.size - 1
    out = np.zeros(S * k, dtype=np.int64)
    counts = np.zeros(S, dtype=np.int64)
    lib().or_algo_r_segmented(seed, stream_base, k, keys, offsets, S, out, counts)
    return out.reshape(S, k), counts


def splitmix_keys(base: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int64)
    lib().or_fill_splitmix(base, n, out)
    return out
