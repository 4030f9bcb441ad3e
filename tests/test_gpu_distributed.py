"""reservoir_amd.distributed with the REAL engine: 2 and 3 gloo ranks sharing one GPU.

Each rank samples its index range of one stream with a GpuSampler (seek + sample_all on device
keys), then distributed.combine runs the one-collective exchange: export_packed -> all_gather ->
merge_packed, for element and distinct samplers alike (the distinct merge runs on the device).
Every rank must end with the oracle's single-stream result (oracle.algo_r, oracle.Distinct) --
including default-hash (ordered) distinct samplers whose boundary hash bucket is oversubscribed,
which take combine's exact replay (export_log -> all_gather -> merge_log).
RCCL cannot put two ranks on one device, so this rehearsal uses gloo (CUDA tensors through host
copies); bench.py at N GPUs uses RCCL with one rank per GPU and the same calls.
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


def _colliding_vals(seed):
    rng = np.random.default_rng(300 + seed)
    hi = rng.integers(0, 2**31, size=400_000, dtype=np.int64)
    lo = (hi ^ rng.integers(0, 3000, size=hi.size, dtype=np.int64)) & 0xFFFFFFFF
    v = (hi << 32) | lo
    return np.concatenate([v, v[rng.integers(0, v.size, 100_000)]])


def _wide_stream():
    """24-byte keys (ids with repeats) and a colliding precomputed hash (97 values): the ordered
    combine's boundary bucket ties"""
    rng = np.random.default_rng(17)
    ids = np.concatenate([np.arange(120_000), rng.integers(0, 120_000, 40_000)])
    rng.shuffle(ids)
    words = np.stack([ids, ids * 7 + 1, ~ids], axis=1).astype(np.int64)
    rows = np.ascontiguousarray(words).view(np.uint8).reshape(-1, 24)
    return rows, {"set": (ids * 1_000_003 + 17).astype(np.int64), "ordered": (ids % 97 - 48).astype(np.int64)}


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from reservoir_amd import Sampler
        from reservoir_amd import distributed as D

        out = {}
        n, k = 3_000_017, 1024
        keys = O.splitmix_keys(0x5EED0000, n)
        lo, hi = D.shard_range(n, rank, world)
        for kt in ("long", "int"):
            dt = torch.int64 if kt == "long" else torch.int32
            kd = torch.from_numpy(keys[lo:hi]).to(dev).to(dt)
            s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, key_type=kt)()
            D.sample_shard(s, kd, lo)
            D.combine(s, device=dev)  # count rides along in the row
            out[f"elements_{kt}"] = (s.result().astype(np.int64).tolist(), s.count)
            s2 = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, key_type=kt)()
            D.sample_shard(s2, kd, lo)
            D.combine(s2, device=dev, total_count=n)
            out[f"elements_{kt}_total"] = (s2.result().astype(np.int64).tolist(), s2.count)
            # bench.py's form: sampled on torch's stream, combined on a communication stream that
            # the sampler hands over to (rsv_set_stream: an event wait, no host wait)
            comm = torch.cuda.Stream(device=dev)
            s3 = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, key_type=kt)()
            s3.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            s3.seek(lo)
            s3.sample_all(kd)
            s3.set_stream(comm.cuda_stream)
            with torch.cuda.stream(comm):
                D.combine(s3, device=dev, total_count=n)
            out[f"elements_{kt}_comm"] = (s3.result().astype(np.int64).tolist(), s3.count)
        vals = np.random.default_rng(3).integers(-2**63, 2**63 - 1, size=400_000, dtype=np.int64)
        vals = np.concatenate([vals, vals[: 150_000]])
        dlo, dhi = D.shard_range(vals.size, rank, world)
        d = Sampler.distinct(5000, seed=9)(hash="identity")
        D.sample_shard(d, torch.from_numpy(vals[dlo:dhi]).to(dev), dlo)
        D.combine(d, device=dev)
        out["distinct"] = (sorted(d.result().tolist()), d.count)
        # default hash (ordered): the exact combine, boundary bucket included
        for seed in range(3):
            cv = _colliding_vals(seed)
            clo, chi = D.shard_range(cv.size, rank, world)
            o = Sampler.distinct(300, seed=seed, retain_log=True)()
            o.sample_all(torch.from_numpy(cv[clo:chi]).to(dev))
            replayed = D.combine(o, device=dev)
            out[f"ordered{seed}"] = (o.result().tolist(), o.count, bool(replayed))
        # fixed-width byte keys (24 B): set mode under a 64-bit hash, ordered mode under a colliding
        # one (the exact replay's broadcasts carry the key words)
        rows, hs = _wide_stream()
        wlo, whi = D.shard_range(rows.shape[0], rank, world)
        rd = torch.from_numpy(rows[wlo:whi]).to(dev)
        for order, hv in hs.items():
            w = Sampler.distinct(700, key_type="bytes24", seed=3, order=order,
                                 retain_log=order == "ordered")(hash=lambda b: 0)
            w.sample_all(rd, hashes=torch.from_numpy(hv[wlo:whi]).to(dev))
            replayed = D.combine(w, device=dev)
            got = sorted(bytes(r) for r in w.result())
            out[f"wide_{order}"] = (got, w.count, bool(replayed))
        q.put((rank, out))
    except BaseException as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_real_engine(cuda, oracle, world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, out in outs:
        assert isinstance(out, dict), out
    for p in procs:
        assert p.exitcode == 0
    n, k = 3_000_017, 1024
    keys = oracle.splitmix_keys(0x5EED0000, n)
    want, _ = oracle.algo_r(0xC0FFEE, 0x5A5A, k, keys)
    want32, _ = oracle.algo_r(0xC0FFEE, 0x5A5A, k, keys.astype(np.int32).astype(np.int64))
    vals = np.random.default_rng(3).integers(-2**63, 2**63 - 1, size=400_000, dtype=np.int64)
    vals = np.concatenate([vals, vals[: 150_000]])
    ref = oracle.Distinct(5000, 9, oracle.HASH_IDENTITY)
    ref.sample_all(vals)
    for rank, out in outs:
        for key in ("elements_long", "elements_long_total", "elements_long_comm"):
            assert out[key] == (want.tolist(), n), (rank, key)
        for key in ("elements_int", "elements_int_total", "elements_int_comm"):
            assert out[key] == (want32.tolist(), n), (rank, key)
        assert out["distinct"] == (sorted(ref.result()[0].tolist()), vals.size), rank
    replays = 0
    for seed in range(3):
        cv = _colliding_vals(seed)
        ref = oracle.Distinct(300, seed, oracle.HASH_JAVA_LONG)
        ref.sample_all(cv)
        for rank, out in outs:
            got, cnt, replayed = out[f"ordered{seed}"]
            assert got == ref.result()[0].tolist() and cnt == cv.size, (rank, seed)
            replays += replayed
    assert replays > 0
    rows, hs = _wide_stream()
    for order, hv in hs.items():
        ref = oracle.DistinctRows(700, 3, 24)
        ref.sample_all(rows, hv)
        want = sorted(bytes(r) for r in ref.result()[0])
        for rank, out in outs:
            got, cnt, replayed = out[f"wide_{order}"]
            assert got == want and cnt == rows.shape[0], (rank, order)
            if order == "ordered":
                assert replayed, rank
