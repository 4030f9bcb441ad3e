"""N > 1 path of reservoir_amd.distributed on CPU: world_size-2 gloo, oracle-backed shard samplers.

The shard samplers here are CPU stand-ins built on the oracle (they implement the same
seek / sample_all / export_packed / merge_packed protocol as GpuSampler -- the packed rows of
include/reservoir_hip.h rsv_export_packed); what is under test is the sharding arithmetic and the
one-collective combine of reservoir_amd.distributed.  The engine's own merge kernels are covered on
the GPU (test_gpu_elements / test_gpu_distinct *_merge tests, test_gpu_distributed).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleElements:
    """Algorithm R (draw format R2) shard sampler on the oracle."""

    is_distinct = False

    def __init__(self, k, seed, stream):
        from oracle import oracle as O

        self.O, self.k, self.seed, self.stream = O, k, seed, stream
        self.res = np.zeros(k, dtype=np.int64)
        self.idx = np.full(k, -1, dtype=np.int64)
        self.count = 0

    def seek(self, i):
        assert i >= self.count
        self.count = i

    def sample_all(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        import ctypes as C

        self.O.lib().or_algo_r(self.seed, self.stream, self.k, self.count, keys, keys.size, self.res,
                               self.idx.ctypes.data_as(C.c_void_p))
        self.count += keys.size

    def export_state(self, device):
        return (torch.from_numpy(self.idx.copy()), torch.from_numpy(self.res.copy()),
                torch.zeros(self.k, dtype=torch.int64), self.k)

    def merge_state(self, idx, keys, hashes, part_n, total):
        for p in range(idx.shape[0]):
            better = idx[p].numpy() > self.idx
            self.idx[better] = idx[p].numpy()[better]
            self.res[better] = keys[p].numpy()[better]
        self.count = max(self.count, total)

    # packed row protocol of GpuSampler.export_packed / merge_packed: [idx(k) | keys(k)]
    @property
    def max_sample_size(self):
        return self.k

    @property
    def packed_width(self):
        return 2 * self.k

    def export_packed(self, row):
        row[: self.k] = torch.from_numpy(self.idx)
        row[self.k: 2 * self.k] = torch.from_numpy(self.res)

    def merge_packed(self, rows, total):
        k = self.k
        self.merge_state(rows[:, :k], rows[:, k:2 * k], None, None, total)

    def result(self):
        return self.res[: min(self.count, self.k)].copy()


def _write_row(row, k, keys, hs, meta):
    """A distinct packed row: [keys(k) | hashes(k) | n, count, tied, max_hash, log_retained, ordered]."""
    n = keys.size
    row[:] = 0
    row[k: 2 * k] = 2**63 - 1
    row[:n] = torch.from_numpy(np.asarray(keys, dtype=np.int64))
    row[k: k + n] = torch.from_numpy(np.asarray(hs, dtype=np.int64))
    row[2 * k:] = torch.tensor(meta, dtype=torch.int64)


def _row_entries(rows, k):
    """(h, key) entries of every gathered row and each row's meta."""
    ents, metas = set(), []
    for r in range(rows.shape[0]):
        meta = rows[r, 2 * k:].tolist()
        n = meta[0]
        ents |= set(zip(rows[r, k: k + n].tolist(), rows[r, :n].tolist()))
        metas.append(meta)
    return sorted(ents), metas


class OracleDistinct:
    is_distinct = True
    is_ordered = False
    key_width = 8
    key_dtype = np.int64

    def __init__(self, k, seed):
        from oracle import oracle as O

        self.O, self.k, self.seed = O, k, seed
        self.d = O.Distinct(k, seed, O.HASH_IDENTITY)
        self.entries = None
        self.count = 0

    def sample_all(self, keys):
        self.d.sample_all(keys)
        self.count += len(keys)

    @property
    def max_sample_size(self):
        return self.k

    @property
    def packed_width(self):
        return 2 * self.k + 6

    def export_packed(self, row):
        keys, hs = self.d.result()
        o = np.lexsort((keys, hs))
        keys, hs = keys[o], hs[o]
        _write_row(row, self.k, keys, hs, [keys.size, self.count, 0, int(hs[-1]) if keys.size else -2**63, 0, 0])

    def merge_packed(self, rows, total):
        ents, _ = _row_entries(rows, self.k)
        self.entries = ents[: self.k]
        self.count = total

    def result(self):
        return np.array([v for _, v in self.entries], dtype=np.int64)


def _java_long_hashes(O, r0, r1, vals):
    """RandomValues' scrambled hash of Long.hashCode (Sampler.scala:75, :396) per element."""
    u = np.asarray(vals, dtype=np.int64).view(np.uint64)
    hc = ((u ^ (u >> np.uint64(32))) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32).astype(np.int64)
    return np.array([O.scramble(r0, r1, int(x)) for x in hc], dtype=np.int64)


class OracleOrdered:
    """Ordered (default-hash) distinct shard sampler on the oracle, with GpuSampler's exact-merge
    protocol: distinct_info / export_log / merge_log.  Its "log" is every element of the piece, a
    superset of what any sequential run admits from it (the engine logs fewer)."""

    is_distinct = True
    is_ordered = True
    key_width = 8
    key_dtype = np.int64

    def __init__(self, k, seed):
        from oracle import oracle as O

        self.O, self.k, self.seed = O, k, seed
        self.d = O.Distinct(k, seed, O.HASH_JAVA_LONG)
        self.seen = np.empty(0, dtype=np.int64)
        self.count = 0
        self.merged = None  # (keys, hashes) ascending after merge_state
        self.tied_merge = False

    @property
    def max_sample_size(self):
        return self.k

    def sample_all(self, keys):
        self.d.sample_all(keys)
        self.seen = np.concatenate([self.seen, np.asarray(keys, dtype=np.int64)])
        self.count += len(keys)

    def _state(self):
        if self.merged is not None:
            return self.merged
        keys, hs = self.d.result()
        o = np.lexsort((keys, hs))
        return keys[o], hs[o]

    def distinct_info(self):
        keys, hs = self._state()
        m = keys.size
        mx = int(hs[-1]) if m else -2**63
        if self.merged is not None:
            tied = self.tied_merge
        else:  # more distinct elements of the piece with h <= max than the set keeps
            u = np.unique(self.seen)
            tied = m == self.k and int((_java_long_hashes(self.O, self.d.r0, self.d.r1, u) <= mx).sum()) > m
        return {"ordered": 1, "tied": int(tied), "log_retained": 1, "size": m, "max_hash": mx,
                "log_entries": self.seen.size}

    @property
    def packed_width(self):
        return 2 * self.k + 6

    def export_packed(self, row):
        keys, hs = self._state()
        info = self.distinct_info()
        _write_row(row, self.k, keys, hs, [keys.size, self.count, info["tied"], info["max_hash"], 1, 1])

    def merge_packed(self, rows, total):
        """As the engine's device merge: the (h, key) bottom-k of the union; tied when the union
        oversubscribes the merged maximum's bucket or a full rank was tied at it."""
        ents, metas = _row_entries(rows, self.k)
        top = ents[: self.k]
        full = len(top) == self.k
        M = top[-1][0] if top else None
        self.tied_merge = full and (sum(1 for h, _ in ents if h <= M) > self.k or
                                    any(m[2] and m[0] == self.k and m[3] == M for m in metas))
        self.merged = (np.array([v for _, v in top], dtype=np.int64), np.array([h for h, _ in top], dtype=np.int64))
        self.count = total

    def export_log(self, bound):
        h = _java_long_hashes(self.O, self.d.r0, self.d.r1, self.seen)
        keep = h < bound if bound != 2**63 - 1 else np.ones(h.size, dtype=bool)
        return h[keep], self.seen[keep]

    def merge_log(self, hashes, keys, total):
        self.d = self.O.Distinct(self.k, self.seed, self.O.HASH_JAVA_LONG)
        self.d.sample_all(keys)
        self.merged = None
        self.seen = np.empty(0, dtype=np.int64)
        self.count = total

    def result(self):
        return self._state()[0]


def _colliding(rng, n, buckets):
    """Long keys whose Long.hashCode takes `buckets` values (many distinct keys per hash)."""
    hi = rng.integers(0, 2**31, size=n, dtype=np.int64)
    lo = (hi ^ rng.integers(0, buckets, size=n, dtype=np.int64)) & 0xFFFFFFFF
    return (hi << 32) | lo


def _ordered_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from reservoir_amd import distributed as D

        outs = []
        for seed in range(6):
            rng = np.random.default_rng(50 + seed)
            vals = _colliding(rng, 6000, 150)
            vals = np.concatenate([vals, vals[rng.integers(0, vals.size, 1500)]])
            lo, hi = D.shard_range(vals.size, rank, world)
            s = OracleOrdered(40, seed)
            s.sample_all(vals[lo:hi])
            replayed = D.combine(s, device="cpu")
            outs.append((sorted(s.result().tolist()), s.count, replayed))
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ordered_exact_combine(oracle, world):
    """Default-hash distinct split in rank order: combine's exact replay (bounds from the gathered
    sets, per-rank candidate export, one more all-gather, replica merge) equals the reference's
    sequential RandomValues over the whole stream -- tie bucket included."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ordered_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    replays = 0
    for seed in range(6):
        rng = np.random.default_rng(50 + seed)
        vals = _colliding(rng, 6000, 150)
        vals = np.concatenate([vals, vals[rng.integers(0, vals.size, 1500)]])
        ref = oracle.Distinct(40, seed, oracle.HASH_JAVA_LONG)
        ref.sample_all(vals)
        want = sorted(ref.result()[0].tolist())
        for rank, res in outs:
            got, cnt, replayed = res[seed]
            assert got == want and cnt == vals.size, (rank, seed)
            replays += bool(replayed)
    assert replays > 0  # the boundary bucket was oversubscribed (40 slots, ~40 keys per hash value)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, k, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from reservoir_amd import distributed as D

        keys = O.splitmix_keys(0x5EED0000, n)
        lo, hi = D.shard_range(n, rank, world)
        s = OracleElements(k, 0xC0FFEE, 0x5A5A)
        D.sample_shard(s, keys[lo:hi], lo)
        D.combine(s, device="cpu")
        s2 = OracleElements(k, 0xC0FFEE, 0x5A5A)  # bench.py's form: global length known
        D.sample_shard(s2, keys[lo:hi], lo)
        D.combine(s2, device="cpu", total_count=n)
        assert s2.result().tolist() == s.result().tolist() and s2.count == n
        vals = np.random.default_rng(3).integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
        vals = np.concatenate([vals, vals[: n // 3]])
        dlo, dhi = D.shard_range(vals.size, rank, world)
        d = OracleDistinct(k, 9)
        D.sample_shard(d, vals[dlo:dhi], dlo)
        D.combine(d, device="cpu")
        q.put((rank, s.result().tolist(), s.count, sorted(d.result().tolist()), d.count))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_index_range_split_combine(oracle, world):
    n, k = 50_003, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys = oracle.splitmix_keys(0x5EED0000, n)
    want, _ = oracle.algo_r(0xC0FFEE, 0x5A5A, k, keys)
    vals = np.random.default_rng(3).integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    vals = np.concatenate([vals, vals[: n // 3]])
    ref = oracle.Distinct(k, 9, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    for rank, res, cnt, dres, dcnt in outs:
        assert res == want.tolist() and cnt == n  # every rank holds the merged reservoir
        assert dres == sorted(ref.result()[0].tolist()) and dcnt == vals.size


def test_shard_range_partitions():
    from reservoir_amd.distributed import shard_range

    for n in [0, 1, 7, 1000, 10**9 + 7]:
        for w in [1, 2, 3, 8]:
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_shard_streams_partitions(oracle):
    """Segmented shards: concatenating the per-rank outputs (stream_base = first stream) equals one
    launch over every stream (checked on the oracle's segmented Algorithm R)."""
    from reservoir_amd.distributed import shard_streams

    rng = np.random.default_rng(2)
    lens = rng.integers(0, 700, size=101)
    offs = np.r_[0, np.cumsum(lens)].astype(np.int64)
    keys = oracle.splitmix_keys(4, int(offs[-1]))
    want, wcnt = oracle.algo_r_segmented(9, 50, 16, keys, offs)
    for world in (1, 2, 3, 8):
        outs, cnts = [], []
        for r in range(world):
            s0, local, (lo, hi) = shard_streams(offs, r, world)
            o, c = oracle.algo_r_segmented(9, 50 + s0, 16, keys[lo:hi], local)
            outs.append(o.reshape(-1, 16))
            cnts.append(c)
        assert np.array_equal(np.concatenate(outs).reshape(-1), want.reshape(-1))
        assert np.array_equal(np.concatenate(cnts), wcnt)
