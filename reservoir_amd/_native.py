"""ctypes binding of libreservoir_hip.so (include/reservoir_hip.h).

This is the Python counterpart of the JNI / Panama FFM stub a Scala binding would declare
(INTEGRATION.md).  It binds exactly the C ABI; no compute happens here.  Loading fails loudly
if the HIP library has not been built -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libreservoir_hip.so")

# rsv_status
OK, E_ILLEGAL_ARGUMENT, E_ILLEGAL_STATE, E_NULL_POINTER, E_DEVICE, E_OUT_OF_MEMORY, E_UNSUPPORTED = range(7)
# enums
KIND_ELEMENTS, KIND_DISTINCT = 0, 1
ENGINE_PHILOX_R, ENGINE_JAVA_L = 0, 1
HASH_DEFAULT, HASH_IDENTITY, HASH_JAVA_LONG, HASH_JAVA_INT, HASH_PRECOMPUTED = range(5)
MEM_HOST, MEM_DEVICE = 0, 1
DISTINCT_AUTO, DISTINCT_SET, DISTINCT_ORDERED = 0, 1, 2

# every symbol include/reservoir_hip.h declares
EXPORTED_SYMBOLS = (
    "rsv_abi_version", "rsv_last_error", "rsv_status_string", "rsv_config_init", "rsv_create",
    "rsv_destroy", "rsv_sample", "rsv_sample_batch", "rsv_result", "rsv_result_device", "rsv_result_take",
    "rsv_host_release",
    "rsv_is_open", "rsv_count", "rsv_set_stream", "rsv_get_stream", "rsv_set_resolve_stream", "rsv_synchronize",
    "rsv_seek",
    "rsv_export_state", "rsv_merge_state", "rsv_sample_segmented", "rsv_replay_events",
    "rsv_export_draws", "rsv_profile_enable", "rsv_profile_read", "rsv_export_packed",
    "rsv_merge_packed", "rsv_profile_global", "rsv_profile_global_read", "rsv_stage_acquire",
    "rsv_stage_commit", "rsv_get_distinct_info", "rsv_export_log", "rsv_merge_log",
    "rsv_sample_indexed", "rsv_fill_slots", "rsv_abort_indexed", "rsv_retain_log", "rsv_commit_indexed",
)


class RsvConfig(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("kind", C.c_int32),
        ("max_sample_size", C.c_int32),
        ("key_width", C.c_int32),
        ("reusable", C.c_int32),
        ("pre_allocate", C.c_int32),
        ("engine", C.c_int32),
        ("hash_kind", C.c_int32),
        ("device", C.c_int32),
        ("distinct_order", C.c_int32),
        ("seed", C.c_uint64),
        ("stream_id", C.c_uint64),
    ]


class RsvDistinctInfo(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("ordered", C.c_int32),
        ("tied", C.c_int32),
        ("log_retained", C.c_int32),
        ("size", C.c_int64),
        ("max_hash", C.c_int64),
        ("log_entries", C.c_int64),
        ("sched_passes", C.c_int64),
        ("sched_fallbacks", C.c_int64),
    ]


class ReservoirError(RuntimeError):
    """Device / runtime failure (RSV_E_DEVICE, RSV_E_OUT_OF_MEMORY, RSV_E_UNSUPPORTED)."""


class IllegalArgumentException(ValueError):
    """Mirror of java.lang.IllegalArgumentException (Sampler.scala:80-81)."""


class IllegalStateException(RuntimeError):
    """Mirror of java.lang.IllegalStateException (Sampler.scala:186)."""


class NullPointerException(TypeError):
    """Mirror of java.lang.NullPointerException (Sampler.scala:82, :94)."""


_lib = None


def load():
    """Load the HIP engine; raises ImportError if it was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()')"
        )
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    L.rsv_abi_version.restype = i32
    L.rsv_last_error.restype = C.c_char_p
    L.rsv_status_string.argtypes = [i32]
    L.rsv_status_string.restype = C.c_char_p
    L.rsv_config_init.argtypes = [C.POINTER(RsvConfig)]
    L.rsv_create.argtypes = [C.POINTER(RsvConfig), C.POINTER(vp)]
    L.rsv_destroy.argtypes = [vp]
    L.rsv_destroy.restype = None
    L.rsv_sample.argtypes = [vp, vp, vp]
    L.rsv_sample_batch.argtypes = [vp, vp, i64, i32, vp]
    L.rsv_result.argtypes = [vp, vp, i64, C.POINTER(i64)]
    L.rsv_result_device.argtypes = [vp, vp, i64, C.POINTER(i64)]
    L.rsv_result_take.argtypes = [vp, C.POINTER(vp), C.POINTER(i64)]
    L.rsv_host_release.argtypes = [vp]
    L.rsv_host_release.restype = None
    L.rsv_is_open.argtypes = [vp]
    L.rsv_is_open.restype = i32
    L.rsv_count.argtypes = [vp]
    L.rsv_count.restype = i64
    L.rsv_set_stream.argtypes = [vp, vp]
    L.rsv_get_stream.argtypes = [vp]
    L.rsv_get_stream.restype = vp
    L.rsv_set_resolve_stream.argtypes = [vp, vp]
    L.rsv_synchronize.argtypes = [vp]
    L.rsv_seek.argtypes = [vp, i64]
    L.rsv_export_state.argtypes = [vp, vp, vp, vp, C.POINTER(i64)]
    L.rsv_merge_state.argtypes = [vp, vp, vp, vp, vp, i32, i64, i64]
    L.rsv_export_packed.argtypes = [vp, vp]
    L.rsv_merge_packed.argtypes = [vp, vp, i32, i64, i64]
    L.rsv_sample_segmented.argtypes = [vp, vp, i64, i32, i32, u64, u64, vp, vp, vp]
    L.rsv_replay_events.argtypes = [vp, i64, i32, i64, vp, vp, i64, i32, vp, vp]
    L.rsv_export_draws.argtypes = [u64, u64, u64, i64, vp, vp]
    L.rsv_profile_enable.argtypes = [vp, i32]
    L.rsv_profile_read.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(i64)]
    L.rsv_profile_global.argtypes = [i32]
    L.rsv_profile_global_read.argtypes = [C.POINTER(C.c_double), C.POINTER(i64)]
    L.rsv_stage_acquire.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(i64)]
    L.rsv_stage_commit.argtypes = [vp, i64]
    L.rsv_get_distinct_info.argtypes = [vp, C.POINTER(RsvDistinctInfo)]
    L.rsv_export_log.argtypes = [vp, i64, vp, vp, i64, C.POINTER(i64)]
    L.rsv_merge_log.argtypes = [vp, vp, vp, i64, i64]
    L.rsv_sample_indexed.argtypes = [vp, i64, vp]
    L.rsv_fill_slots.argtypes = [vp, vp]
    L.rsv_abort_indexed.argtypes = [vp]
    L.rsv_commit_indexed.argtypes = [vp]
    L.rsv_retain_log.argtypes = [vp, i32]
    for name in ("rsv_config_init", "rsv_create", "rsv_sample", "rsv_sample_batch", "rsv_result",
                 "rsv_result_device", "rsv_result_take", "rsv_set_stream", "rsv_set_resolve_stream",
                 "rsv_synchronize", "rsv_seek",
                 "rsv_export_state", "rsv_merge_state", "rsv_sample_segmented", "rsv_replay_events",
                 "rsv_export_draws", "rsv_profile_enable", "rsv_profile_read", "rsv_export_packed",
                 "rsv_merge_packed", "rsv_profile_global", "rsv_profile_global_read", "rsv_stage_acquire",
                 "rsv_stage_commit", "rsv_get_distinct_info", "rsv_export_log", "rsv_merge_log",
                 "rsv_sample_indexed", "rsv_fill_slots", "rsv_abort_indexed", "rsv_retain_log",
                 "rsv_commit_indexed"):
        getattr(L, name).restype = i32
    if L.rsv_abi_version() != 1:
        raise ImportError("libreservoir_hip.so ABI version mismatch")
    _lib = L
    return L


def check(status: int) -> None:
    """Map an rsv_status onto the reference's exception types (include/reservoir_hip.h)."""
    if status == OK:
        return
    msg = load().rsv_last_error().decode(errors="replace")
    if status == E_ILLEGAL_ARGUMENT:
        raise IllegalArgumentException(msg)
    if status == E_ILLEGAL_STATE:
        raise IllegalStateException(msg)
    if status == E_NULL_POINTER:
        raise NullPointerException(msg)
    if status == E_OUT_OF_MEMORY:
        raise MemoryError(msg)
    raise ReservoirError(f"{load().rsv_status_string(status).decode()}: {msg}")
