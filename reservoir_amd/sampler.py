"""Host-side mirror of ``lgbt.princess.reservoir.Sampler`` over the HIP engine.

Reference: core/src/main/scala/lgbt/princess/reservoir/Sampler.scala (NthPortal/reservoir).

    Sampler(max_sample_size, pre_allocate=False, reusable=False)(map)      # Sampler.apply  :128-136
    Sampler.distinct(max_sample_size, reusable=False)(map, hash=default)   # Sampler.distinct :171-180

    s.sample(x)        # Sampler.sample    :37-38
    s.sample_all(xs)   # Sampler.sampleAll :49-50
    s.result()         # Sampler.result    :59-60
    s.is_open          # Sampler.isOpen    :67

Names, argument meaning and exceptions follow the reference (IllegalArgumentException for a
bad size, NullPointerException for a missing ``map``/``hash``, IllegalStateException after
``result()`` on a single-use sampler).  ``map`` runs on the host (the reference allows it to be
called more than ``maxSampleSize`` times, Sampler.scala:115-116); the extracted primitive keys go
to the GPU in batches.  Keys already resident in HBM (a torch CUDA tensor) are sampled in place.

Extensions (keyword-only, defaulted so reference-style calls are unchanged):
    key_type  "long" (B = Long, 8-byte keys, default), "int" (B = Int, 4-byte keys), or "bytesN"
              (fixed-width byte keys with value equality, N a multiple of 8 in 16..256, e.g.
              "bytes16" for java.util.UUID laid out [mostSigBits | leastSigBits] as little-endian
              Longs; numpy arrays of shape (n, N) uint8 or dtype "VN", torch CUDA uint8 tensors of
              shape (n, N)).  Sampler.distinct over byte keys dedups by the bytes and takes a
              callable ``hash`` (the JVM's ``hash: B => Long``) -- or, for "bytes16", the default
              java.util.UUID.hashCode
    engine    "philox_r" (default: data-parallel Algorithm R) or "java_l" (the reference's own
              Algorithm L over java.util.Random(seed): bit-identical results to the reference)
    seed      RNG seed (default: fresh entropy, like ``new Random()`` at Sampler.scala:199)
    stream_id Philox stream of a "philox_r" sampler
    device    HIP device ordinal (default: current device)
    order     distinct only: "auto" (default), "set" or "ordered" -- how hash ties are resolved
              (include/reservoir_hip.h rsv_distinct_order): "ordered" reproduces the reference's
              sequential heap for any hash, "set" is the order-independent bottom-k by (hash, key)
    retain_log  distinct "ordered" only: keep the replayed candidates on the host for the exact
              multi-rank merge (export_log; reservoir_amd.distributed.combine needs it on every
              rank whose boundary hash bucket may tie)

sample_all over an indexable host sequence (a list, tuple, range or host numpy array -- the
reference's IndexedSeq) samples by index first and maps only the elements that end in the
reservoir, as the reference's sampleIndexed does (Sampler.scala:261-273): no key crosses PCIe but
the <= k winners (rsv_sample_indexed / rsv_fill_slots).
"""
from __future__ import annotations

import ctypes as C
import os
from collections.abc import Sequence
from typing import Any, Callable, Iterable

import numpy as np

from . import _native as N
from ._native import IllegalArgumentException, IllegalStateException, NullPointerException

MAX_SIZE = 2**31 - 1 - 2  # Sampler.scala:71


def identity(x):
    return x


_KEY = {"long": (8, np.int64), "int": (4, np.int32)}


def _wide_width(key_type) -> int:
    """Width of a "bytesN" key type (N a multiple of 8 in 16..256), else 0."""
    if isinstance(key_type, str) and key_type.startswith("bytes") and key_type[5:].isdigit():
        w = int(key_type[5:])
        if 16 <= w <= 256 and w % 8 == 0:
            return w
    return 0
_ENGINE = {"philox_r": N.ENGINE_PHILOX_R, "java_l": N.ENGINE_JAVA_L}
_ORDER = {"auto": N.DISTINCT_AUTO, "set": N.DISTINCT_SET, "ordered": N.DISTINCT_ORDERED}


def _fresh_seed() -> int:
    return int.from_bytes(os.urandom(8), "little")


def _validate_shared(max_sample_size: int, map_fn) -> None:
    # validateSharedParams, Sampler.scala:79-83
    if max_sample_size > MAX_SIZE:
        raise IllegalArgumentException("requirement failed: maxSampleSize exceeds VM limit")
    if max_sample_size <= 0:
        raise IllegalArgumentException("requirement failed: maxSampleSize must be positive")
    if map_fn is None:
        raise NullPointerException("`map` cannot be `null`")


_TORCH = None


def _torch():
    global _TORCH
    if _TORCH is None:
        import torch

        _TORCH = torch
    return _TORCH


def _is_torch_cuda(x) -> bool:
    t = type(x)
    return t.__module__.startswith("torch") and t.__name__ == "Tensor" and getattr(x, "is_cuda", False)


def _indexed(elements) -> bool:
    """The reference's IndexedSeq with a known size (Sampler.scala:294-307): a host sequence with
    len() and O(1) indexing -- not a string, not bytes, not a torch tensor (those take the batch
    paths)."""
    if isinstance(elements, np.ndarray):
        return elements.ndim == 1
    if isinstance(elements, (str, bytes, bytearray)) or type(elements).__module__.startswith("torch"):
        return False
    return isinstance(elements, (range, list, tuple, Sequence))


def _current_raw_stream(torch, t) -> int:
    """torch's current HIP stream on t's device as an integer handle (cheap form when available)."""
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return int(raw(t.device.index))
    return torch.cuda.current_stream(t.device).cuda_stream



class _HostBuffer:
    """A pinned result buffer handed over by rsv_result_take: exposed to numpy as raw bytes, released
    (rsv_host_release) when the last array viewing it is gone."""

    def __init__(self, lib, ptr: int, nbytes: int):
        self._lib = lib
        self._ptr = ptr
        # (numpy wants a non-NULL address even for an empty view)
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "version": 3,
                                    "data": (ptr or 1, False)}

    def __del__(self):
        ptr, self._ptr = self._ptr, 0
        if ptr:
            try:
                self._lib.rsv_host_release(C.c_void_p(ptr))
            except Exception:  # interpreter shutdown: the process frees it
                pass

class GpuSampler:
    """A ``Sampler[A, B]`` whose state lives on an MI355X (one opaque C-ABI handle)."""

    def __init__(self, kind: int, max_sample_size: int, map_fn: Callable, *, reusable: bool,
                 pre_allocate: bool = False, hash_fn=None, hash_kind: int = N.HASH_DEFAULT,
                 key_type: str = "long", engine: str = "philox_r", seed: int | None = None,
                 stream_id: int = 0, device: int | None = None, order: str = "auto",
                 retain_log: bool = False):
        self._objects = key_type == "object"
        if self._objects:
            if kind != N.KIND_ELEMENTS:
                raise IllegalArgumentException("key_type 'object' is for Sampler.apply (distinct needs keys)")
            key_type = "long"  # the handle's key width; its slots never hold keys (rsv_commit_indexed)
        if key_type not in _KEY and not _wide_width(key_type):
            raise IllegalArgumentException(f"key_type must be one of {sorted(_KEY)}, 'bytesN' or 'object'")
        if engine not in _ENGINE:
            raise IllegalArgumentException(f"engine must be one of {sorted(_ENGINE)}")
        if order not in _ORDER:
            raise IllegalArgumentException(f"order must be one of {sorted(_ORDER)}")
        self._L = N.load()
        self._map = map_fn
        self._hash_fn = hash_fn
        if key_type in _KEY:
            self._width, self._dtype = _KEY[key_type]
        else:
            self._width = _wide_width(key_type)
            self._dtype = np.dtype(f"V{self._width}")
        self._kind = kind
        self._k = max_sample_size
        self._reusable = bool(reusable)
        cfg = N.RsvConfig()
        N.check(self._L.rsv_config_init(C.byref(cfg)))
        cfg.kind = kind
        cfg.max_sample_size = max_sample_size
        cfg.key_width = self._width
        cfg.reusable = 1 if reusable else 0
        cfg.pre_allocate = 1 if pre_allocate else 0
        cfg.engine = _ENGINE[engine]
        cfg.hash_kind = hash_kind
        cfg.distinct_order = _ORDER[order]
        cfg.device = -1 if device is None else int(device)
        cfg.seed = (_fresh_seed() if seed is None else int(seed)) & (2**64 - 1)
        cfg.stream_id = int(stream_id) & (2**64 - 1)
        self.seed = cfg.seed
        h = C.c_void_p()
        N.check(self._L.rsv_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self._stream = int(self._L.rsv_get_stream(h) or 0)
        self._rstream = 0  # set_resolve_stream
        self._precomputed = hash_kind == N.HASH_PRECOMPUTED
        self._rows = None  # the last merge_packed's rows (a distinct merge reads them until it settles)
        self._ordered = False
        if self._objects:  # ObjectSampler's state: the slot array and the buffered mapped elements
            self._slots: list = []
            self._pending: list = []
            self._obj_count = 0
        if kind == N.KIND_DISTINCT:
            self._ordered = bool(self.distinct_info()["ordered"])  # no device work at creation
            if retain_log:
                N.check(self._L.rsv_retain_log(h, 1))

    # -- lifecycle ----------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.rsv_destroy(self._h)
            self._h = None
        self._rows = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def is_open(self) -> bool:
        return bool(self._L.rsv_is_open(self._h))

    isOpen = is_open

    @property
    def count(self) -> int:
        return int(self._L.rsv_count(self._h))

    @property
    def stream(self) -> int:
        return self._stream

    def set_stream(self, hip_stream: int) -> None:
        """Run this sampler's work on ``hip_stream`` (e.g. torch.cuda.current_stream().cuda_stream)."""
        N.check(self._L.rsv_set_stream(self._h, C.c_void_p(hip_stream)))
        self._stream = int(hip_stream)

    def set_resolve_stream(self, hip_stream: int | None) -> None:
        """Pipelining (element samplers, batches > 2^27 keys): the slot resolve + result publication
        run on ``hip_stream`` after the batch's K1, so the next sampler's K1 on this stream does not
        queue behind them (include/reservoir_hip.h rsv_set_resolve_stream).  The batch's keys must
        stay unchanged until result() returns."""
        N.check(self._L.rsv_set_resolve_stream(self._h, C.c_void_p(hip_stream or 0)))
        self._rstream = int(hip_stream or 0)

    def synchronize(self) -> None:
        N.check(self._L.rsv_synchronize(self._h))

    # -- Sampler trait --------------------------------------------------------------------------
    def _key_hash(self, element):
        key = self._map(element)
        hv = None
        if self._precomputed:
            hv = C.c_int64(int(self._hash_fn(key)))
        return key, hv

    # -- any B (key_type="object"): bindings/scala/core/.../gpu/ObjectSampler.scala's protocol ----
    _OBJ_BATCH = 65536

    def _obj_check_open(self) -> None:
        if self._h is None or not self._L.rsv_is_open(self._h):
            raise IllegalStateException("use of sampler after calling `result()`")

    def _obj_place(self, offs, values_at) -> None:
        """the batch's new slot holders into the slot array (values_at(offset) -> B)"""
        for j in np.flatnonzero(offs >= 0).tolist():
            if j >= len(self._slots):
                self._slots.extend([None] * (j + 1 - len(self._slots)))
            self._slots[j] = values_at(int(offs[j]))

    def _obj_flush(self) -> None:
        n = len(self._pending)
        if not n:
            return
        offs = np.empty(self._k, dtype=np.int64)
        N.check(self._L.rsv_sample_indexed(self._h, n, offs.ctypes.data_as(C.c_void_p)))
        N.check(self._L.rsv_commit_indexed(self._h))
        pending, self._pending = self._pending, []
        self._obj_place(offs, pending.__getitem__)
        self._obj_count += n

    def _obj_sample_indexed(self, seq) -> None:
        self._obj_flush()
        n = len(seq)
        offs = np.empty(self._k, dtype=np.int64)
        N.check(self._L.rsv_sample_indexed(self._h, n, offs.ctypes.data_as(C.c_void_p)))
        try:  # map the new holders first: the slots change only once all of them are mapped
            vals = {int(o): self._map(seq[int(o)]) for o in offs[offs >= 0].tolist()}
        except BaseException:
            N.check(self._L.rsv_abort_indexed(self._h))
            raise
        N.check(self._L.rsv_commit_indexed(self._h))
        self._obj_place(offs, vals.__getitem__)
        self._obj_count += n

    def sample(self, element: Any) -> None:
        """Sampler.sample (Sampler.scala:37-38)."""
        if self._objects:
            self._obj_check_open()
            self._pending.append(self._map(element))
            if len(self._pending) == self._OBJ_BATCH:
                self._obj_flush()
            return
        if not self._L.rsv_is_open(self._h):
            raise IllegalStateException("use of sampler after calling `result()`")
        key, hv = self._key_hash(element)
        if self._width > 8:
            kbuf = self._key_bytes(key)
        else:
            kbuf = self._dtype(key).tobytes() if not isinstance(key, (bytes, bytearray)) else key
        N.check(self._L.rsv_sample(self._h, C.c_char_p(kbuf),
                                   C.byref(hv) if hv is not None else None))

    def sample_all(self, elements: Iterable, hashes=None) -> None:
        """Sampler.sampleAll (Sampler.scala:49-50): same result as sample() on each element.

        ``hashes``: a distinct sampler with a callable ``hash`` over device-resident keys takes the
        hashes precomputed as an int64 CUDA tensor (one per key, e.g. computed by torch on the
        device) instead of calling ``hash`` per element on the host."""
        if hashes is not None:
            self._sample_device_hashed(elements, hashes)
            return
        if self._objects:
            self._obj_check_open()
            if _indexed(elements) and len(elements) > 0:
                self._obj_sample_indexed(elements)
            else:
                for x in elements:
                    self.sample(x)
            return
        if _is_torch_cuda(elements) and self._map is identity and not self._precomputed:
            # device fast path; checkOpen() first, as the reference does before any other work
            # (Sampler.scala:186, :417-419): a single-use sampler closed by result() keeps its handle
            if self._h is None or not self._L.rsv_is_open(self._h):
                raise IllegalStateException("use of sampler after calling `result()`")
            torch = _torch()
            t = elements if elements.is_contiguous() else elements.contiguous()
            cur = _current_raw_stream(torch, t)
            if cur != self._stream:
                self._wait_torch(t)  # produced on torch's stream
                # and torch must not hand the block to another tensor while this handle's stream
                # still reads it (the caller may drop `elements` as soon as we return)
                t.record_stream(torch.cuda.ExternalStream(self._stream, device=t.device))
            if self._rstream and self._rstream != cur:
                # the batch's resolve reads the keys on the resolve stream, after this call returns
                t.record_stream(torch.cuda.ExternalStream(self._rstream, device=t.device))
            if self._width <= 8:
                if t.element_size() != self._width:
                    raise IllegalArgumentException("device tensor dtype does not match key_type")
                n_keys = t.numel()
            else:  # fixed-width byte keys: any dtype, rows of exactly key_width bytes
                if t.dim() < 2 or t.shape[-1] * t.element_size() != self._width:
                    raise IllegalArgumentException("device tensor rows must hold key_width bytes")
                n_keys = t.numel() * t.element_size() // self._width
            N.check(self._L.rsv_sample_batch(self._h, C.c_void_p(t.data_ptr()), n_keys,
                                             N.MEM_DEVICE, None))
            return
        if not self._L.rsv_is_open(self._h):
            raise IllegalStateException("use of sampler after calling `result()`")
        if self._kind == N.KIND_ELEMENTS and self._width <= 8 and _indexed(elements):
            self._sample_indexed(elements)
            return
        if self._width > 8:
            keys = self._wide_keys(elements)
        elif isinstance(elements, np.ndarray) and self._map is identity:
            keys = np.ascontiguousarray(elements, dtype=self._dtype)
        else:
            keys = np.fromiter((self._map(x) for x in elements), dtype=self._dtype)
        hashes = None
        if self._precomputed:
            hashes = np.ascontiguousarray(
                np.fromiter((int(self._hash_fn(k)) for k in keys.tolist()), dtype=np.int64,
                            count=keys.size))
        N.check(self._L.rsv_sample_batch(
            self._h, keys.ctypes.data_as(C.c_void_p), keys.size, N.MEM_HOST,
            hashes.ctypes.data_as(C.c_void_p) if hashes is not None else None))

    sampleAll = sample_all

    def _sample_device_hashed(self, keys, hashes) -> None:
        """Device keys + their precomputed hashes (RSV_HASH_PRECOMPUTED) in one rsv_sample_batch."""
        if self._h is None or not self._L.rsv_is_open(self._h):
            raise IllegalStateException("use of sampler after calling `result()`")
        if not self._precomputed:
            raise IllegalArgumentException("hashes= needs a distinct sampler with a callable hash")
        if not (_is_torch_cuda(keys) and _is_torch_cuda(hashes)) or self._map is not identity:
            raise IllegalArgumentException("hashes= takes device tensors of keys (identity map) and int64 hashes")
        torch = _torch()
        t = keys if keys.is_contiguous() else keys.contiguous()
        hv = hashes if hashes.is_contiguous() else hashes.contiguous()
        if hv.dtype != torch.int64:
            raise IllegalArgumentException("hashes must be int64")
        if self._width <= 8:
            if t.element_size() != self._width:
                raise IllegalArgumentException("device tensor dtype does not match key_type")
            n_keys = t.numel()
        else:
            if t.dim() < 2 or t.shape[-1] * t.element_size() != self._width:
                raise IllegalArgumentException("device tensor rows must hold key_width bytes")
            n_keys = t.numel() * t.element_size() // self._width
        if hv.numel() != n_keys:
            raise IllegalArgumentException("one hash per key")
        cur = _current_raw_stream(torch, t)
        if cur != self._stream:
            self._wait_torch(t)
            ext = torch.cuda.ExternalStream(self._stream, device=t.device)
            t.record_stream(ext)
            hv.record_stream(ext)
        N.check(self._L.rsv_sample_batch(self._h, C.c_void_p(t.data_ptr()), n_keys, N.MEM_DEVICE,
                                         C.c_void_p(hv.data_ptr())))

    def _sample_indexed(self, seq) -> None:
        """sampleAll over an IndexedSeq (Sampler.scala:289-312 -> sampleIndexed :261-273): the engine
        samples the len(seq) indices, and only the elements that now hold a slot are mapped."""
        n = len(seq)
        offs = np.empty(self._k, dtype=np.int64)
        N.check(self._L.rsv_sample_indexed(self._h, n, offs.ctypes.data_as(C.c_void_p)))
        if n == 0:
            return
        sel = np.flatnonzero(offs >= 0)
        keys = np.zeros(self._k, dtype=self._dtype)
        try:
            if isinstance(seq, np.ndarray) and self._map is identity:
                keys[sel] = seq[offs[sel]]
            else:
                for j in sel.tolist():
                    keys[j] = self._map(seq[int(offs[j])])
        except BaseException:
            # `map` threw (or a key does not fit the key type): drop the batch, keep the sampler
            # usable, and propagate the exception as the reference's sampleIndexed does
            N.check(self._L.rsv_abort_indexed(self._h))
            raise
        N.check(self._L.rsv_fill_slots(self._h, keys.ctypes.data_as(C.c_void_p)))

    def _wide_keys(self, elements) -> np.ndarray:
        """Host batch of fixed-width byte keys as a contiguous array of dtype VN."""
        if isinstance(elements, np.ndarray) and self._map is identity:
            a = np.ascontiguousarray(elements)
        else:
            a = np.array([self._key_bytes(self._map(x)) for x in elements], dtype=np.uint8).reshape(-1, self._width)
        if a.dtype != self._dtype:
            if a.dtype != np.uint8 or a.ndim != 2 or a.shape[1] != self._width:
                raise IllegalArgumentException(f"byte keys must be uint8 rows of {self._width} bytes")
            a = np.ascontiguousarray(a).view(self._dtype).reshape(-1)
        return a

    def _key_bytes(self, key) -> bytes:
        b = bytes(key) if not isinstance(key, (bytes, bytearray)) else bytes(key)
        if len(b) != self._width:
            raise IllegalArgumentException(f"key is {len(b)} bytes, key_width is {self._width}")
        return b

    def result(self) -> np.ndarray:
        """Sampler.result (Sampler.scala:59-60). Slot order for element samplers."""
        if self._objects:  # a list of the B values in slot order
            self._obj_check_open()
            self._obj_flush()
            out = list(self._slots[: min(self._obj_count, self._k)])
            if not self._reusable:
                self.close()
            return out
        if self._h is None or not self._L.rsv_is_open(self._h):
            raise IllegalStateException("use of sampler after calling `result()`")
        if not self._reusable:
            # the published keys handed over instead of copied (rsv_result_take); the array owns the
            # pinned buffer and releases it when the last view of it goes (byte keys: (n, key_width)
            # uint8 rows over it -- a 65536-key UUID set is 1 MB, two host copies saved)
            buf, n = C.c_void_p(), C.c_int64(0)
            st = self._L.rsv_result_take(self._h, C.byref(buf), C.byref(n))
            if st == N.OK:
                raw = np.asarray(_HostBuffer(self._L, buf.value or 0, n.value * self._width))
                return raw.reshape(-1, self._width) if self._width > 8 else raw.view(self._dtype)
            if st != N.E_UNSUPPORTED:
                N.check(st)
        out = np.empty(self._k, dtype=self._dtype)
        n = C.c_int64(0)
        N.check(self._L.rsv_result(self._h, out.ctypes.data_as(C.c_void_p), self._k, C.byref(n)))
        if self._width > 8:  # fixed-width byte keys: (n, key_width) uint8 rows, slot order
            return out[: n.value].view(np.uint8).reshape(-1, self._width).copy()
        return out if n.value == self._k else out[: n.value].copy()

    def result_device(self, out_tensor) -> int:
        """Write the result into a device tensor (no host round trip); returns its length."""
        self._order_after_torch(out_tensor)
        n = C.c_int64(0)
        N.check(self._L.rsv_result_device(self._h, C.c_void_p(out_tensor.data_ptr()),
                                          out_tensor.numel(), C.byref(n)))
        return n.value

    def _order_after_torch(self, t) -> None:
        """Device tensors handed to the engine were written (or allocated and filled) by torch on
        its current stream; unless this handle runs on that stream, order the handle's stream after
        it first -- the engine's own stream is not ordered after torch's."""
        if _is_torch_cuda(t):
            torch = _torch()
            if _current_raw_stream(torch, t) != self._stream:
                self._wait_torch(t)

    def _wait_torch(self, t) -> None:
        """An event recorded on torch's current stream, waited for by this handle's stream
        (hipStreamWaitEvent): stream-ordered, no host wait.  The event is kept until the next
        hand-over."""
        torch = _torch()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        torch.cuda.ExternalStream(self._stream, device=t.device).wait_event(ev)
        self._torch_ev = ev

    # -- multi-GPU helpers (reservoir_amd.distributed) ------------------------------------------
    @property
    def is_distinct(self) -> bool:
        return self._kind == N.KIND_DISTINCT

    @property
    def max_sample_size(self) -> int:
        return self._k

    @property
    def key_width(self) -> int:
        return self._width

    @property
    def key_dtype(self):
        return self._dtype

    def seek(self, index: int) -> None:
        """Next element has global index ``index`` (index-range split across ranks)."""
        N.check(self._L.rsv_seek(self._h, int(index)))

    def export_state(self, device):
        """Partial state as device tensors (idx[k], keys[k], hashes[k], n)."""
        import torch

        idx = torch.full((self._k,), -1, dtype=torch.int64, device=device)
        if self._width > 8:
            keys = torch.zeros((self._k, self._width), dtype=torch.uint8, device=device)
        else:
            keys = torch.zeros(self._k, dtype=torch.int64 if self._width == 8 else torch.int32, device=device)
        hashes = torch.zeros(self._k, dtype=torch.int64, device=device)
        self._order_after_torch(hashes)
        n = C.c_int64(0)
        N.check(self._L.rsv_export_state(self._h, C.c_void_p(idx.data_ptr()),
                                         C.c_void_p(keys.data_ptr()), C.c_void_p(hashes.data_ptr()),
                                         C.byref(n)))
        return idx, keys, hashes, n.value

    @property
    def key_words(self) -> int:
        """int64 words one key takes in a packed row (1 for Int/Long keys, key_width / 8 for byte keys)."""
        return self._width // 8 if self._width > 8 else 1

    @property
    def packed_width(self) -> int:
        """Length of this sampler's rsv_export_packed row (int64 words)."""
        if self.is_distinct:
            return self._k * (self.key_words + 1) + 6
        return self._k * (1 + self.key_words)

    def export_packed(self, row) -> None:
        """Write the packed row (include/reservoir_hip.h rsv_export_packed) into the int64 device
        tensor ``row``: ``[idx(k) | keys as int64 (k)]`` for element samplers, ``[keys (k) | hashes
        (k) | n, count, tied, max_hash, log_retained, ordered]`` for distinct ones (one kernel,
        stream-ordered on a caller stream)."""
        self._order_after_torch(row)
        N.check(self._L.rsv_export_packed(self._h, C.c_void_p(row.data_ptr())))

    def merge_packed(self, rows, total_count: int) -> None:
        """Merge the packed rows of a ``[parts, width]`` int64 device tensor: per slot the last
        writer (elements), the bottom-k of the union (distinct: on the device, no host wait; the
        rows are kept referenced until the next merge, as the engine may re-read them)."""
        if rows.dim() != 2 or not rows.is_contiguous():
            raise IllegalArgumentException("rows must be a contiguous [parts, width] tensor")
        self._order_after_torch(rows)
        if self.is_distinct:
            self._rows = rows
        N.check(self._L.rsv_merge_packed(self._h, C.c_void_p(rows.data_ptr()), int(rows.shape[0]),
                                         int(rows.shape[1]), int(total_count)))

    def distinct_info(self) -> dict:
        """Distinct samplers: set size, largest hash, whether the boundary hash bucket is
        oversubscribed (``tied``), and the candidate log's status (include/reservoir_hip.h)."""
        info = N.RsvDistinctInfo()
        info.struct_size = C.sizeof(N.RsvDistinctInfo)
        N.check(self._L.rsv_get_distinct_info(self._h, C.byref(info)))
        return {f: int(getattr(info, f)) for f, _ in N.RsvDistinctInfo._fields_[1:]}

    @property
    def is_ordered(self) -> bool:
        """RSV_DISTINCT_ORDERED semantics (fixed at creation: no device state is read)."""
        return self._ordered

    def retain_log(self, on: bool = True) -> None:
        """Ordered distinct samplers: keep the candidate log for export_log (before sampling)."""
        N.check(self._L.rsv_retain_log(self._h, 1 if on else 0))

    def export_log(self, bound: int = 2**63 - 1):
        """Ordered distinct samplers: every logged candidate with hash < ``bound`` in arrival order
        as host arrays (hashes int64, keys of the key type)."""
        n = C.c_int64(0)
        # count first (cap 0): the buffers are sized for what the bound keeps, not the whole log
        N.check(self._L.rsv_export_log(self._h, int(bound), None, None, 0, C.byref(n)))
        cap = n.value
        h = np.empty(max(cap, 1), dtype=np.int64)
        k = np.empty(max(cap, 1), dtype=self._dtype)
        if cap:
            N.check(self._L.rsv_export_log(self._h, int(bound), h.ctypes.data_as(C.c_void_p),
                                           k.ctypes.data_as(C.c_void_p), cap, C.byref(n)))
        return h[: n.value].copy(), k[: n.value].copy()

    def merge_log(self, hashes, keys, total_count: int) -> None:
        """Ordered distinct samplers: become a fresh RandomValues replica run over the candidate
        run (host arrays, global arrival order)."""
        h = np.ascontiguousarray(hashes, dtype=np.int64)
        k = np.ascontiguousarray(keys, dtype=self._dtype)
        if h.size != k.size:
            raise IllegalArgumentException("hashes and keys differ in length")
        N.check(self._L.rsv_merge_log(self._h, h.ctypes.data_as(C.c_void_p), k.ctypes.data_as(C.c_void_p),
                                      h.size, int(total_count)))

    def merge_state(self, idx, keys, hashes, part_n, total_count: int) -> None:
        """Merge gathered partial states ([parts, k] device tensors) into this sampler."""
        parts = int(keys.shape[0])
        self._order_after_torch(keys)
        pn = np.ascontiguousarray(np.asarray(part_n, dtype=np.int64))
        N.check(self._L.rsv_merge_state(
            self._h, C.c_void_p(idx.data_ptr()), C.c_void_p(keys.data_ptr()),
            C.c_void_p(hashes.data_ptr()), pn.ctypes.data_as(C.c_void_p), parts,
            int(keys.shape[1]), int(total_count)))


def Sampler(max_sample_size: int, pre_allocate: bool = False, reusable: bool = False, **ext):
    """``Sampler.apply`` (Sampler.scala:128-136): ``Sampler(k)(map)``."""

    def make(map_fn: Callable = identity) -> GpuSampler:
        _validate_shared(max_sample_size, map_fn)  # validateNonDistinctParams :85-88
        return GpuSampler(N.KIND_ELEMENTS, max_sample_size, map_fn, reusable=reusable,
                          pre_allocate=pre_allocate, **ext)

    return make


_DEFAULT_HASH = object()


def _resolve_hash(hash):
    """validateDistinctParams (Sampler.scala:90-95) + mapping onto rsv_hash_kind."""
    if hash is None:
        raise NullPointerException("`hash` cannot be `null`")
    if hash is _DEFAULT_HASH:
        return N.HASH_DEFAULT, None
    if isinstance(hash, str):
        kinds = {"identity": N.HASH_IDENTITY, "java_long": N.HASH_JAVA_LONG, "java_int": N.HASH_JAVA_INT}
        if hash not in kinds:
            raise IllegalArgumentException(f"unknown hash kind {hash!r}")
        return kinds[hash], None
    if callable(hash):
        return N.HASH_PRECOMPUTED, hash
    raise IllegalArgumentException("hash must be callable or a known hash kind")


def distinct(max_sample_size: int, reusable: bool = False, **ext):
    """``Sampler.distinct`` (Sampler.scala:171-180): ``Sampler.distinct(k)(map, hash)``.

    ``hash`` defaults to ``B#hashCode().toLong`` (Sampler.scala:75); pass ``"identity"`` for the
    bijective Long identity hash, or any callable (evaluated on the host, shipped as int64).
    """

    def make(map_fn: Callable = identity, hash=_DEFAULT_HASH) -> GpuSampler:
        _validate_shared(max_sample_size, map_fn)  # validateDistinctParams :90-95
        hk, hf = _resolve_hash(hash)
        return GpuSampler(N.KIND_DISTINCT, max_sample_size, map_fn, reusable=reusable,
                          hash_fn=hf, hash_kind=hk, **ext)

    return make


Sampler.distinct = distinct  # type: ignore[attr-defined]
Sampler.apply = Sampler  # type: ignore[attr-defined]
