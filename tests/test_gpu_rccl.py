"""reservoir_amd.distributed over RCCL (torch.distributed backend "nccl"), on one GPU.

RCCL puts at most one rank on a device, so the one-GPU box runs a world of ONE rank: the same
calls bench.py makes at N GPUs -- ``init_process_group("nccl", device_id=...)``, the element
combine on a communication stream after the sampler's ``rsv_set_stream`` hand-over (bench.py
``issue()``), ``all_gather_into_tensor`` of the packed rows, the device merge, and for ordered
distinct samplers the exact replay's size all-gather + broadcasts -- all through RCCL's kernels
instead of gloo's host copies.  Results must equal the oracle's single sampler.
The child is a spawned process so the test process keeps no process group.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _twins(n, seed):
    """Long keys whose Long.hashCode collides in ~3000-key groups (the boundary bucket ties)."""
    rng = np.random.default_rng(500 + seed)
    hi = rng.integers(0, 2**31, size=n, dtype=np.int64)
    lo = (hi ^ rng.integers(0, 3000, size=n, dtype=np.int64)) & 0xFFFFFFFF
    v = (hi << 32) | lo
    return np.concatenate([v, v[rng.integers(0, n, n // 4)]])


def _child(port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    try:
        from oracle import oracle as O
        from reservoir_amd import Sampler
        from reservoir_amd import distributed as D

        out = {"backend": dist.get_backend()}
        n, k = 5_000_011, 1024
        kd = torch.from_numpy(O.splitmix_keys(0x5EED0000, n)).to(dev)
        stream = torch.cuda.current_stream(dev)
        comm = torch.cuda.Stream(device=dev)
        # bench.py issue() at N > 1, two steps in flight on the same streams
        samplers = []
        for _ in range(2):
            s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
            s.set_stream(stream.cuda_stream)
            s.seek(0)
            s.sample_all(kd)
            s.set_stream(comm.cuda_stream)
            with torch.cuda.stream(comm):
                D.combine(s, device=dev, total_count=n)
            samplers.append(s)
        out["elements_comm"] = [(s.result().tolist(), s.count) for s in samplers]
        # the count carried in the row (total_count unknown)
        s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
        D.sample_shard(s, kd, 0)
        D.combine(s, device=dev)
        out["elements_row_count"] = (s.result().tolist(), s.count)
        # distinct, set mode (identity hash): one all_gather + the device merge
        vals = np.random.default_rng(4).integers(-2**63, 2**63 - 1, size=300_000, dtype=np.int64)
        vals = np.concatenate([vals, vals[:90_000]])
        d = Sampler.distinct(4000, seed=9)(hash="identity")
        D.sample_shard(d, torch.from_numpy(vals).to(dev), 0)
        D.combine(d, device=dev)
        out["distinct_set"] = (sorted(d.result().tolist()), d.count)
        # distinct, ordered (Long.hashCode) with a tied boundary bucket: the exact replay's
        # size all-gather and broadcast go through RCCL too
        cv = _twins(200_000, 1)
        o = Sampler.distinct(300, seed=1, retain_log=True)()
        D.sample_shard(o, torch.from_numpy(cv).to(dev), 0)
        tied = bool(o.distinct_info()["tied"])
        replayed = D.combine(o, device=dev)
        out["ordered"] = (o.result().tolist(), o.count, tied, bool(replayed))
        torch.cuda.synchronize()
        q.put(out)
    except BaseException as ex:  # noqa: BLE001 -- reported to the parent
        q.put(repr(ex))
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_world1_combine(cuda, oracle):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=110)
    p.join(timeout=60)
    assert isinstance(out, dict), out
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    n, k = 5_000_011, 1024
    want, _ = oracle.algo_r(0xC0FFEE, 0x5A5A, k, oracle.splitmix_keys(0x5EED0000, n))
    for got in out["elements_comm"] + [out["elements_row_count"]]:
        assert got == (want.tolist(), n)
    vals = np.random.default_rng(4).integers(-2**63, 2**63 - 1, size=300_000, dtype=np.int64)
    vals = np.concatenate([vals, vals[:90_000]])
    ref = oracle.Distinct(4000, 9, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    assert out["distinct_set"] == (sorted(ref.result()[0].tolist()), vals.size)
    cv = _twins(200_000, 1)
    ref = oracle.Distinct(300, 1, oracle.HASH_JAVA_LONG)
    ref.sample_all(cv)
    got, cnt, tied, replayed = out["ordered"]
    assert sorted(got) == sorted(ref.result()[0].tolist()) and cnt == cv.size
    assert tied and replayed  # the exact replay ran through RCCL
