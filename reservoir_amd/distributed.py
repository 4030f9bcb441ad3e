"""Multi-GPU sampling: one process per GPU, torch.distributed (RCCL over xGMI) for the one exchange.

The reference has no multi-device story.  Two shardings are exact here:

* one giant stream of an element sampler ("philox_r"): rank r samples its contiguous index
  range [offset_r, offset_r + n_r) after ``seek(offset_r)``; because a draw depends only on
  (seed, stream, global index), the union of the per-rank last writers, taken per slot by the
  largest global index, is bit-identical to one sampler fed the whole stream.
* a distinct sampler: bottom-k is mergeable, any split of the elements works.

``combine`` is the only collective: every rank exports its k-slot partial state, one
``all_gather_into_tensor`` moves it (k x 16 B per rank: latency-bound, not link-bound), and each
rank merges all parts with the engine's merge kernel.  Independent streams (segmented sampling)
need no collective at all.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous index range [lo, hi) of rank ``rank`` for a stream of ``n_total`` elements."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_streams(offsets, rank: int, world: int):
    """Independent streams (segmented sampling): this rank's contiguous slice of
    streams as (first_stream, local offsets rebased to 0, element range [lo, hi)).  No collective:
    rank r samples its streams with ``stream_base = first_stream`` and the outputs concatenate."""
    n_streams = len(offsets) - 1
    s0, s1 = shard_range(n_streams, rank, world)
    lo, hi = int(offsets[s0]), int(offsets[s1])
    return s0, offsets[s0:s1 + 1] - lo, (lo, hi)


def sample_shard(sampler, keys_local, global_offset: int) -> None:
    """Sample this rank's shard of one stream (keys at [global_offset, +len))."""
    if not sampler.is_distinct:
        sampler.seek(global_offset)
    sampler.sample_all(keys_local)


def combine(sampler, group=None, device=None, total_count: int | None = None) -> None:
    """All-gather the partial states of every rank and merge them into ``sampler`` (on all ranks).

    One collective: each rank packs its partial state into one int64 row -- element samplers
    ``[idx(k) | keys(k)]`` (16 KB at k = 1024), distinct samplers ``[keys(k) | hashes(k) | n]`` --
    so the exchange pays one RCCL latency.  ``total_count`` (the global stream length) saves a
    second exchange for element samplers; without it the per-rank counts ride along in the row.
    """
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    if not sampler.is_distinct:
        _combine_elements(sampler, world, group, device, total_count)
        return
    idx, keys, hashes, n = sampler.export_state(device)
    k = keys.numel()
    dev = idx.device
    width = 2 * k + 2
    row = torch.empty(width, dtype=torch.int64, device=dev)
    row[:k] = keys.to(torch.int64)
    row[k:2 * k] = hashes
    row[2 * k:] = torch.tensor([n, sampler.count], dtype=torch.int64).to(dev, non_blocking=True)
    flat = torch.empty(world * width, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(flat, row, group=group)  # flat output: gloo and RCCL both accept
    rows = flat.view(world, width)
    g_keys = rows[:, :k].to(keys.dtype).contiguous()
    meta = rows[:, 2 * k:].cpu()
    part_n = meta[:, 0].tolist()
    total = int(meta[:, 1].sum()) if total_count is None else int(total_count)
    sampler.merge_state(torch.empty((world, k), dtype=torch.int64, device=dev), g_keys,
                        rows[:, k:2 * k].contiguous(), part_n, total)


def _combine_elements(sampler, world, group, device, total_count) -> None:
    """Element sampler: one kernel packs ``[idx(k) | keys(k)]`` (+ the count when the global
    length is unknown), one all-gather, one merge kernel over the gathered rows in place."""
    k = sampler.max_sample_size
    kw = getattr(sampler, "key_width", 8)
    body = k * (1 + (kw // 8 if kw > 8 else 1))  # [idx(k) | keys: one int64 each, or kw/8 words]
    width = body + (0 if total_count is not None else 1)
    row = torch.empty(width, dtype=torch.int64, device=device)
    sampler.export_packed(row)
    if total_count is None:
        row[body] = sampler.count
    flat = torch.empty(world * width, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(flat, row, group=group)
    rows = flat.view(world, width)
    total = int(rows[:, body].max().item()) if total_count is None else int(total_count)
    sampler.merge_packed(rows, total)
