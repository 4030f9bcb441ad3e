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
    """Sample this rank's shard of one stream (keys at [global_offset, +len)).  An ordered distinct
    sampler retains its candidate log from its first shard on (combine's exact replay reads it)."""
    if not sampler.is_distinct:
        sampler.seek(global_offset)
    elif sampler.is_ordered and sampler.count == 0 and hasattr(sampler, "retain_log"):
        sampler.retain_log(True)
    sampler.sample_all(keys_local)


def _mark(marks) -> None:
    if marks is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append(ev)


def combine(sampler, group=None, device=None, total_count: int | None = None, marks: list | None = None,
            strict: bool = True) -> bool:
    """All-gather the partial states of every rank and merge them into ``sampler`` (on all ranks).

    One collective: each rank packs its partial state into one int64 row (rsv_export_packed) --
    element samplers ``[idx(k) | keys(k)]`` (16 KB at k = 1024), distinct samplers ``[keys(k) |
    hashes(k) | meta]`` -- so the exchange pays one RCCL latency, and one device merge
    (rsv_merge_packed) folds the gathered rows in, stream-ordered: a set-mode distinct or element
    combine never waits on the host.  ``total_count`` (the global stream length) saves reading the
    per-rank counts back.

    Ordered distinct samplers (the reference's default ``hashCode``) read the merged state back
    once; when its boundary hash bucket is oversubscribed they take one more exchange, the exact
    replay: rank r holds the r-th piece of the stream, and the result is the reference's
    sequential set (every rank needs ``retain_log``; ``sample_shard`` sets it).  When the replay is
    needed and a rank did not retain its log, ``strict`` (default) raises IllegalStateException --
    the reference's set cannot be formed -- and ``strict=False`` warns and keeps the (hash, key)
    bottom-k instead.  The tie is only known once the device merge has run, so when it raises,
    ``sampler`` already holds that merged (hash, key) bottom-k (as with ``strict=False``); callers
    that want the old warn-and-continue behaviour (before round 6 the default) pass
    ``strict=False``.  Returns whether the replay ran.
    ``marks`` (a list): CUDA events are appended after the export, the all-gather and the merge.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    if not sampler.is_distinct:
        _combine_elements(sampler, world, group, device, total_count)
        return False
    width = sampler.packed_width
    row = torch.empty(width, dtype=torch.int64, device=device)
    sampler.export_packed(row)
    _mark(marks)
    flat = torch.empty(world * width, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(flat, row, group=group)  # flat output: gloo and RCCL both accept
    _mark(marks)
    rows = flat.view(world, width)
    k = sampler.max_sample_size
    mo = _meta_off(sampler)
    total = int(rows[:, mo + 1].sum().item()) if total_count is None else int(total_count)
    sampler.merge_packed(rows, total)
    _mark(marks)
    if not sampler.is_ordered:
        return False
    meta = _ordered_replay_meta(sampler, rows, strict)
    if meta is None:
        return False
    w = _key_words(sampler)
    bounds = replay_bounds(rows, meta, k, w)
    h, keys = sampler.export_log(bounds[rank])
    part = torch.from_numpy(np.concatenate([h, _as_words(keys)])).to(device)
    sizes = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(sizes, torch.tensor([h.size], dtype=torch.int64).to(device), group=group)
    sz = sizes.cpu().numpy()
    parts = []
    for r in range(world):  # exact sizes, one broadcast per rank (no padding to the largest log)
        buf = part if r == rank else torch.empty((1 + w) * int(sz[r]), dtype=torch.int64, device=device)
        if sz[r]:
            dist.broadcast(buf, src=dist.get_global_rank(group, r) if group is not None else r, group=group)
        lg = buf.cpu().numpy()
        parts.append((lg[: sz[r]], lg[sz[r]:]))  # hashes, then the keys' int64 words
    _merge_logs(sampler, parts)
    return True


def merge_local(target, shards, total_count: int | None = None, strict: bool = True) -> bool:
    """``combine`` without a process group: ``shards`` are samplers that each saw one contiguous
    piece of a stream, in order (shard r = rank r), all on one device; their merged state goes into
    ``target`` (a fresh sampler, or one of the shards).  Same rows, merge kernels and exact ordered
    replay as ``combine`` -- e.g. C4's 8-way split rehearsed on one GPU.  Returns whether the exact
    ordered replay ran (``strict`` as in ``combine``)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    rows = torch.empty((len(shards), target.packed_width), dtype=torch.int64, device=dev)
    for r, s in enumerate(shards):
        s.export_packed(rows[r])
    if not target.is_distinct:
        total = sum(s.count for s in shards) if total_count is None else int(total_count)
        target.merge_packed(rows, total)
        return False
    k = target.max_sample_size
    mo = _meta_off(target)
    total = int(rows[:, mo + 1].sum().item()) if total_count is None else int(total_count)
    target.merge_packed(rows, total)
    if not target.is_ordered:
        return False
    meta = _ordered_replay_meta(target, rows, strict)
    if meta is None:
        return False
    bounds = replay_bounds(rows, meta, k, _key_words(target))
    parts = []
    for r, s in enumerate(shards):
        h, keys = s.export_log(bounds[r])
        parts.append((h, _as_words(keys)))
    _merge_logs(target, parts)
    return True


# distinct row (rsv_export_packed): [keys(k) | hashes(k) | n, count, tied, max_hash, log_retained, ordered];
# a key is one int64 word (Int / Long, widened) or key_width / 8 words (fixed-width byte keys)
_META = 6


def _key_words(sampler) -> int:
    return int(getattr(sampler, "key_words", 1))


def _meta_off(sampler) -> int:
    return sampler.max_sample_size * (_key_words(sampler) + 1)


def _as_words(keys) -> np.ndarray:
    """Host keys as int64 words: Int / Long keys widened, byte keys (dtype VN) N / 8 words each."""
    keys = np.ascontiguousarray(keys)
    if keys.dtype.kind == "V":
        return keys.view(np.int64).reshape(-1)
    return keys.astype(np.int64)


def _ordered_replay_meta(sampler, rows, strict: bool = True):
    """After the device merge of an ordered sampler: the per-rank meta (host) when the exact replay
    is needed, else None.  The merged set is the reference's unless more distinct elements share its
    maximum hash than it keeps -- seen in the union, or inside one rank whose own boundary bucket
    was oversubscribed at that maximum (the engine folds both into ``tied``)."""
    info = sampler.distinct_info()  # settles the merge: one wait for its published words
    if not info["tied"]:
        return None
    meta = rows[:, _meta_off(sampler):].cpu().numpy()
    if not all(int(m[5]) for m in meta):
        return None  # some rank ran in set mode: the (hash, key) set is the defined result
    if not all(int(m[4]) for m in meta):
        msg = ("ordered distinct combine: the boundary hash bucket is oversubscribed and a rank did not retain "
               "its candidate log (Sampler.distinct(..., retain_log=True), or distributed.sample_shard), so the "
               "reference's arrival-order set cannot be formed")
        if strict:
            from ._native import IllegalStateException

            raise IllegalStateException(msg)
        warnings.warn(msg + "; strict=False: the merged set resolves the bucket by (hash, key)", RuntimeWarning)
        return None
    return meta


def replay_bounds(rows, meta, k: int, key_words: int = 1) -> list:
    """Per rank r, the bound its exported candidates must stay under: the k-th smallest hash of the
    distinct elements in the pieces before it (from the gathered bottom-k sets), else no bound.
    Inside rank r's piece the reference's heap maximum is at most that hash, and it admits only
    elements strictly below its maximum (Sampler.scala:403).  Elements are distinct by (hash, key
    words); equal keys have equal hashes."""
    world = rows.shape[0]
    kw = k * key_words
    h_all = rows[:, kw:kw + k].cpu().numpy()
    k_all = rows[:, :kw].cpu().numpy().reshape(world, k, key_words)
    no_bound = np.iinfo(np.int64).max
    bounds = [no_bound]
    acc = np.empty((0, key_words + 1), dtype=np.int64)  # rows [h, key words...], bottom-k so far
    for r in range(1, world):
        n = int(meta[r - 1][0])
        ent = np.concatenate([h_all[r - 1, :n, None], k_all[r - 1, :n]], axis=1)
        acc = np.unique(np.concatenate([acc, ent]), axis=0)[:k]  # sorted by (h, key words)
        bounds.append(int(acc[k - 1, 0]) if acc.shape[0] == k else no_bound)
    return bounds


def _merge_logs(sampler, parts) -> None:
    """Exact ordered merge: every rank's exported candidates, concatenated in rank order, through a
    fresh replica of the reference's RandomValues (rsv_merge_log).  ``parts``: (hashes, key words)."""
    h = np.concatenate([np.asarray(p[0], dtype=np.int64) for p in parts]) if parts else np.empty(0, np.int64)
    words = np.concatenate([np.asarray(p[1], dtype=np.int64) for p in parts]) if parts else np.empty(0, np.int64)
    dt = np.dtype(sampler.key_dtype)
    keys = np.ascontiguousarray(words).view(dt) if dt.kind == "V" else words.astype(dt)
    sampler.merge_log(h, keys, int(sampler.count))


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
