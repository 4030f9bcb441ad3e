"""The C-ABI library: it loads, exports every symbol include/reservoir_hip.h declares, and validates
arguments (the reference's IllegalArgument/NullPointer cases) before touching a device.  CPU only."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "reservoir_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rsv_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def native():
    from reservoir_amd import _native

    return _native


def test_every_declared_symbol_is_exported(native):
    L = native.load()
    decl = declared_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(native.EXPORTED_SYMBOLS) == decl


def test_library_is_a_gfx950_hip_object():
    path = os.path.join(ROOT, "reservoir_amd", "libreservoir_hip.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob  # the embedded code object targets MI355X


def test_config_layout_matches_header(native):
    L = native.load()
    cfg = native.RsvConfig()
    assert L.rsv_config_init(C.byref(cfg)) == native.OK
    assert cfg.struct_size == C.sizeof(native.RsvConfig) == 56
    assert (cfg.kind, cfg.max_sample_size, cfg.key_width, cfg.engine, cfg.device) == (0, 1, 8, 0, -1)


@pytest.mark.parametrize("k,err", [(0, 1), (-1, 1), (2**31 - 1, 1), (2**31 - 2, 1)])
def test_create_rejects_bad_sizes_without_a_device(native, k, err):
    """validateSharedParams (Sampler.scala:79-83) runs before any HIP call."""
    L = native.load()
    cfg = native.RsvConfig()
    L.rsv_config_init(C.byref(cfg))
    cfg.max_sample_size = k
    h = C.c_void_p()
    assert L.rsv_create(C.byref(cfg), C.byref(h)) == native.E_ILLEGAL_ARGUMENT
    assert not h.value
    msg = L.rsv_last_error().decode()
    assert "maxSampleSize" in msg


def test_null_pointer_and_state_checks(native):
    L = native.load()
    assert L.rsv_create(None, None) == native.E_NULL_POINTER
    n = C.c_int64()
    assert L.rsv_result(None, None, 0, C.byref(n)) == native.E_NULL_POINTER
    assert L.rsv_is_open(None) == 0
    assert L.rsv_sample_segmented(None, None, 1, 8, 0, 0, 0, None, None, None) == native.E_ILLEGAL_ARGUMENT
    assert L.rsv_sample_segmented(None, None, 1, 8, 4, 0, 0, None, None, None) == native.E_NULL_POINTER
    with pytest.raises(native.IllegalArgumentException):
        native.check(native.E_ILLEGAL_ARGUMENT)
    with pytest.raises(native.IllegalStateException):
        native.check(native.E_ILLEGAL_STATE)


def test_status_strings(native):
    L = native.load()
    assert L.rsv_status_string(native.E_ILLEGAL_STATE) == b"illegal state"
    assert L.rsv_abi_version() == 1


def test_create_rejects_unknown_distinct_order_without_a_device(native):
    L = native.load()
    cfg = native.RsvConfig()
    L.rsv_config_init(C.byref(cfg))
    assert cfg.distinct_order == native.DISTINCT_AUTO
    cfg.kind = native.KIND_DISTINCT
    cfg.max_sample_size = 10
    cfg.distinct_order = 7
    h = C.c_void_p()
    assert L.rsv_create(C.byref(cfg), C.byref(h)) == native.E_ILLEGAL_ARGUMENT
    assert not h.value
    assert "distinct order" in L.rsv_last_error().decode()


def test_process_wide_profiler_without_launches(native):
    """rsv_profile_global on/off and a read with no timed launch: zero totals, no device needed."""
    L = native.load()
    assert L.rsv_profile_global(1) == native.OK
    assert L.rsv_profile_global(0) == native.OK
    ms, n = C.c_double(-1), C.c_int64(-1)
    assert L.rsv_profile_global_read(C.byref(ms), C.byref(n)) == native.OK
    assert (ms.value, n.value) == (0.0, 0)
    assert L.rsv_profile_global_read(None, None) == native.E_NULL_POINTER
