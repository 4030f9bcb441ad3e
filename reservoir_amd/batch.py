"""Stateless batch entry points of the HIP engine over device tensors.

torch is used only for device memory and streams (plumbing); the compute runs in
libreservoir_hip.so.  Every function raises if the engine is unavailable.

    sample_segmented  -- K2: S independent samplers in one launch (one wave per stream)
    replay_events     -- K1': apply the reference's Algorithm-L eviction events on the GPU
    export_draws      -- the per-element draw sequence j_i of draw format R2
"""
from __future__ import annotations

import ctypes as C

from . import _native as N


def _stream_ptr(torch, device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def sample_segmented(keys, offsets, k: int, seed: int, stream_base: int = 0):
    """Sample each of S streams keys[offsets[s]:offsets[s+1]] independently (Algorithm R).

    Returns (out[S, k], counts[S]) device tensors; stream s is bit-identical to a single
    "philox_r" Sampler with stream_id = stream_base + s fed the same keys.
    """
    import torch

    L = N.load()
    if not (keys.is_cuda and offsets.is_cuda):
        raise N.IllegalArgumentException("keys and offsets must be device tensors")
    if keys.dtype not in (torch.int64, torch.int32) or offsets.dtype != torch.int64:
        raise N.IllegalArgumentException("keys must be int64/int32 and offsets int64")
    keys = keys.contiguous()
    offsets = offsets.contiguous()
    S = offsets.numel() - 1
    # the kernel writes every slot (empty ones as 0) and every count: no zero-fill (at C3's shape
    # torch.zeros was a 512 MB memset beside the 1.7 ms launch)
    out = torch.empty((max(S, 0), k), dtype=keys.dtype, device=keys.device)
    counts = torch.empty(max(S, 0), dtype=torch.int64, device=keys.device)
    if S <= 0:
        return out, counts
    N.check(L.rsv_sample_segmented(
        C.c_void_p(keys.data_ptr()), C.c_void_p(offsets.data_ptr()), S, keys.element_size(), k,
        seed & (2**64 - 1), stream_base & (2**64 - 1), C.c_void_p(out.data_ptr()),
        C.c_void_p(counts.data_ptr()), _stream_ptr(torch, keys.device)))
    return out, counts


def replay_events(keys, base_index: int, ev_pos, ev_slot, k: int, reservoir=None):
    """Apply (1-based position, slot) eviction events to the keys at [base, base+n)."""
    import torch

    L = N.load()
    keys = keys.contiguous()
    if reservoir is None:
        reservoir = torch.zeros(k, dtype=keys.dtype, device=keys.device)
    ev_pos = ev_pos.to(device=keys.device, dtype=torch.int64).contiguous()
    ev_slot = ev_slot.to(device=keys.device, dtype=torch.int32).contiguous()
    N.check(L.rsv_replay_events(
        C.c_void_p(keys.data_ptr()), keys.numel(), keys.element_size(), base_index,
        C.c_void_p(ev_pos.data_ptr()), C.c_void_p(ev_slot.data_ptr()), ev_pos.numel(), k,
        C.c_void_p(reservoir.data_ptr()), _stream_ptr(torch, keys.device)))
    return reservoir


def export_draws(seed: int, stream_id: int, i0: int, n: int, device=None):
    """j_i for i in [i0, i0+n) as a uint64-valued int64 device tensor."""
    import torch

    L = N.load()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    N.check(L.rsv_export_draws(seed & (2**64 - 1), stream_id & (2**64 - 1), i0, n,
                               C.c_void_p(out.data_ptr()), _stream_ptr(torch, dev)))
    return out
