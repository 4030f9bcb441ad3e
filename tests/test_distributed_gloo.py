"""N > 1 path of reservoir_amd.distributed on CPU: world_size-2 gloo, oracle-backed shard samplers.

The shard samplers here are CPU stand-ins built on the oracle (they implement the same
seek / sample_all / export_state / merge_state protocol as GpuSampler); what is under test is the
sharding arithmetic and the one-collective combine of reservoir_amd.distributed.  The engine's
own merge kernel is covered on the GPU (test_gpu_elements / test_gpu_distinct *_merge tests).
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

    def export_packed(self, row):
        row[: self.k] = torch.from_numpy(self.idx)
        row[self.k: 2 * self.k] = torch.from_numpy(self.res)

    def merge_packed(self, rows, total):
        k = self.k
        self.merge_state(rows[:, :k], rows[:, k:2 * k], None, None, total)

    def result(self):
        return self.res[: min(self.count, self.k)].copy()


class OracleDistinct:
    is_distinct = True

    def __init__(self, k, seed):
        from oracle import oracle as O

        self.O, self.k, self.seed = O, k, seed
        self.d = O.Distinct(k, seed, O.HASH_IDENTITY)
        self.entries = None
        self.count = 0

    def sample_all(self, keys):
        self.d.sample_all(keys)
        self.count += len(keys)

    def export_state(self, device):
        keys, hs = self.d.result()
        n = keys.size
        pad = lambda a: torch.from_numpy(np.concatenate([a, np.zeros(self.k - n, dtype=np.int64)]))
        return torch.full((self.k,), -1, dtype=torch.int64), pad(keys), pad(hs), n

    def merge_state(self, idx, keys, hashes, part_n, total):
        ents = set()
        for p, n in enumerate(part_n):
            ents |= set(zip(hashes[p, :n].tolist(), keys[p, :n].tolist()))
        self.entries = sorted(ents)[: self.k]
        self.count = total

    def result(self):
        return np.array([v for _, v in self.entries], dtype=np.int64)


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
