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

import warnings

import numpy as np
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


def combine(sampler, group=None, device=None, total_count: int | None = None) -> bool:
    """All-gather the partial states of every rank and merge them into ``sampler`` (on all ranks).

    One collective: each rank packs its partial state into one int64 row -- element samplers
    ``[idx(k) | keys(k)]`` (16 KB at k = 1024), distinct samplers ``[keys(k) | hashes(k) | meta]``
    -- so the exchange pays one RCCL latency.  ``total_count`` (the global stream length) saves a
    second exchange for element samplers; without it the per-rank counts ride along in the row.

    Ordered distinct samplers (the reference's default ``hashCode``) whose merged boundary hash
    bucket is oversubscribed take one more exchange, the exact replay: rank r holds the r-th piece
    of the stream, and the result is the reference's sequential set.  Returns whether it ran.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    if not sampler.is_distinct:
        _combine_elements(sampler, world, group, device, total_count)
        return False
    row = _distinct_row(sampler, device)
    flat = torch.empty(world * row.numel(), dtype=torch.int64, device=row.device)
    dist.all_gather_into_tensor(flat, row, group=group)  # flat output: gloo and RCCL both accept
    rows = flat.view(world, row.numel())
    meta = _merge_distinct_rows(sampler, rows, total_count)
    if _ordered_replay_needed(sampler, meta):
        bounds = replay_bounds(rows, meta, sampler.max_sample_size)
        h, keys = sampler.export_log(bounds[rank])
        part = torch.from_numpy(np.concatenate([h, keys.astype(np.int64)])).to(row.device)
        sizes = torch.empty(world, dtype=torch.int64, device=row.device)
        dist.all_gather_into_tensor(sizes, torch.tensor([h.size], dtype=torch.int64).to(row.device), group=group)
        sz = sizes.cpu().numpy()
        mx = int(sz.max())
        buf = torch.zeros(2 * mx, dtype=torch.int64, device=row.device)
        buf[: h.size] = part[: h.size]
        buf[mx: mx + h.size] = part[h.size:]
        logs = torch.empty(world * 2 * mx, dtype=torch.int64, device=row.device)
        dist.all_gather_into_tensor(logs, buf, group=group)
        lg = logs.view(world, 2 * mx).cpu().numpy()
        _merge_logs(sampler, [(lg[r, : sz[r]], lg[r, mx: mx + sz[r]]) for r in range(world)], meta)
        return True
    return False


def merge_local(target, shards, total_count: int | None = None) -> bool:
    """``combine`` without a process group: ``shards`` are samplers that each saw one contiguous
    piece of a stream, in order (shard r = rank r), all on one device; their merged state goes into
    ``target`` (a fresh sampler, or one of the shards).  Same rows, merge calls and exact ordered
    replay as ``combine`` -- e.g. C4's 8-way split rehearsed on one GPU.  Returns whether the exact
    ordered replay ran."""
    if not target.is_distinct:
        k = target.max_sample_size
        kw = getattr(target, "key_width", 8)
        body = k * (1 + (kw // 8 if kw > 8 else 1))
        dev = torch.device("cuda", torch.cuda.current_device())
        rows = torch.empty((len(shards), body), dtype=torch.int64, device=dev)
        for r, s in enumerate(shards):
            s.export_packed(rows[r])
        total = sum(s.count for s in shards) if total_count is None else int(total_count)
        target.merge_packed(rows, total)
        return False
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    rows = torch.stack([_distinct_row(s, dev) for s in shards])
    meta = _merge_distinct_rows(target, rows, total_count)
    if _ordered_replay_needed(target, meta):
        bounds = replay_bounds(rows, meta, target.max_sample_size)
        parts = []
        for r, s in enumerate(shards):
            h, keys = s.export_log(bounds[r])
            parts.append((h, keys.astype(np.int64)))
        _merge_logs(target, parts, meta)
        return True
    return False


# distinct row: [keys(k) | hashes(k) | n, count, tied, max_hash, log_retained, ordered]
_META = 6


def _distinct_row(sampler, device) -> torch.Tensor:
    info = sampler.distinct_info()
    idx, keys, hashes, n = sampler.export_state(device)
    k = keys.numel()
    row = torch.empty(2 * k + _META, dtype=torch.int64, device=idx.device)
    row[:k] = keys.to(torch.int64)
    row[k:2 * k] = hashes
    meta = [n, sampler.count, info["tied"], info["max_hash"], info["log_retained"], info["ordered"]]
    row[2 * k:] = torch.tensor(meta, dtype=torch.int64).to(idx.device, non_blocking=True)
    return row


def _merge_distinct_rows(sampler, rows, total_count):
    """Bottom-k of the union by (hash, key) (rsv_merge_state); returns the per-rank meta (host)."""
    k = sampler.max_sample_size
    world = rows.shape[0]
    dtype = torch.int64 if sampler.key_width == 8 else torch.int32
    meta = rows[:, 2 * k:].cpu().numpy()
    total = int(meta[:, 1].sum()) if total_count is None else int(total_count)
    sampler.merge_state(torch.empty((world, k), dtype=torch.int64, device=rows.device),
                        rows[:, :k].to(dtype).contiguous(), rows[:, k:2 * k].contiguous(),
                        meta[:, 0].tolist(), total)
    return meta


def _ordered_replay_needed(sampler, meta) -> bool:
    """Ordered samplers only: the merged set is the reference's unless more distinct elements share
    the merged maximum hash than it keeps -- seen in the union (``tied`` after the merge) or inside
    one rank whose own set was tied at that maximum (it exported only part of its bucket)."""
    if not all(int(m[5]) for m in meta):
        return False
    info = sampler.distinct_info()
    k = sampler.max_sample_size
    if info["size"] < k:
        return False  # fewer than k distinct elements overall: the set holds all of them
    M = info["max_hash"]
    need = bool(info["tied"]) or any(int(m[2]) and int(m[3]) == M and int(m[0]) == k for m in meta)
    if need and not all(int(m[4]) for m in meta):
        warnings.warn("ordered distinct combine: a rank did not retain its candidate log; the merged set "
                      "resolves the boundary hash bucket by (hash, key) instead of arrival order",
                      RuntimeWarning)
        return False
    return need


def replay_bounds(rows, meta, k: int) -> list:
    """Per rank r, the bound its exported candidates must stay under: the k-th smallest hash of the
    distinct elements in the pieces before it (from the gathered bottom-k sets), else no bound.
    Inside rank r's piece the reference's heap maximum is at most that hash, and it admits only
    elements strictly below its maximum (Sampler.scala:403)."""
    world = rows.shape[0]
    h_all = rows[:, k:2 * k].cpu().numpy()
    k_all = rows[:, :k].cpu().numpy()
    no_bound = np.iinfo(np.int64).max
    bounds = [no_bound]
    ph = np.empty(0, dtype=np.int64)
    pk = np.empty(0, dtype=np.int64)
    for r in range(1, world):
        n = int(meta[r - 1][0])
        uk, first = np.unique(np.concatenate([pk, k_all[r - 1, :n]]), return_index=True)
        uh = np.concatenate([ph, h_all[r - 1, :n]])[first]
        order = np.lexsort((uk, uh))[:k]
        ph, pk = uh[order], uk[order]
        bounds.append(int(ph[k - 1]) if ph.size == k else no_bound)
    return bounds


def _merge_logs(sampler, parts, meta) -> None:
    """Exact ordered merge: every rank's exported candidates, concatenated in rank order, through a
    fresh replica of the reference's RandomValues (rsv_merge_log)."""
    h = np.concatenate([np.asarray(p[0], dtype=np.int64) for p in parts]) if parts else np.empty(0, np.int64)
    keys = np.concatenate([np.asarray(p[1], dtype=np.int64) for p in parts]) if parts else np.empty(0, np.int64)
    sampler.merge_log(h, keys.astype(sampler.key_dtype), int(sampler.count))


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
