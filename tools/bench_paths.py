"""Secondary measurements of the other hot-path configs: not the bench.py line.

  C3  segmented: 2^20 streams x 4096 int64 keys, k = 64 (K2)
  C4g distinct, one GPU's share of C4: 5e8 int64 keys, 30 % duplicates, k = 65536, identity hash
      (K3 filter + merge); also the default Long.hashCode
  C2L the reference's Algorithm L (engine java_l) on C2: 1e9 keys, k = 1024 (K1' replay)

Prints one JSON line per config with the kernel time (HIP events on the launch stream) and the
8-B-per-element HBM roofline fraction.  Usage: python tools/bench_paths.py [--only c3,c4,c2l]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import splitmix_fill  # noqa: E402

HBM = 8000.0


def timed(fn, reps=5, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def c3(dev):
    from reservoir_amd import batch

    S, L, k = 1 << 20, 4096, 64
    n = S * L
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0)
    offs = torch.arange(0, n + 1, L, dtype=torch.int64, device=dev)
    t = timed(lambda: batch.sample_segmented(keys, offs, k, seed=1), reps=5)
    bytes_alg = n * 8 + S * k * 8
    return {"config": "C3 segmented 2^20 x 4096, k=64", "elements": n, "seconds": t,
            "Gelem_s": n / t / 1e9, "alg_bytes_per_elem": bytes_alg / n,
            "achieved_GBs": bytes_alg / t / 1e9, "hbm_frac": bytes_alg / t / 1e9 / HBM}


def c4_data(n, dev):
    D = int(n * 0.7)
    v = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(v[:D], 0xD15C << 32)
    # duplicates: element i >= D copies a pseudo-random earlier distinct value
    idx = (torch.arange(D, n, dtype=torch.int64, device=dev) * 2654435761) % D
    v[D:] = v[idx]
    # scatter positions by an affine bijection of [0, n)
    a = 1_000_000_007
    perm = (torch.arange(n, dtype=torch.int64, device=dev) * a + 12345) % n
    out = torch.empty_like(v)
    out[perm] = v
    return out


def c4(dev, hash_kind="identity", order="auto"):
    from reservoir_amd import Sampler, _native

    n, k = 500_000_000, 65536
    vals = c4_data(n, dev)
    torch.cuda.synchronize()
    L = _native.load()
    times, kern = [], []
    for rep in range(4):
        mk = Sampler.distinct(k, seed=7, order=order)
        d = mk(hash=hash_kind) if hash_kind != "default" else mk()
        d.set_stream(torch.cuda.current_stream().cuda_stream)
        _native.check(L.rsv_profile_enable(d.handle, 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.sample_all(vals)
        r = d.result()
        t1 = time.perf_counter()
        ms, cnt = C.c_double(), C.c_int64()
        _native.check(L.rsv_profile_read(d.handle, C.byref(ms), C.byref(cnt)))
        if rep:
            times.append(t1 - t0)
            kern.append((ms.value / 1e3, cnt.value))
        assert r.size == k
        d.close()
    t = sorted(times)[len(times) // 2]
    kt, passes = kern[0]
    ordered = order == "ordered" or (order == "auto" and hash_kind == "default")
    read = n * 8 if ordered else n * 8 * passes  # ordered: one chunked pass; set: every pass reads all
    return {"config": f"C4 (one GPU's share) distinct 5e8 keys 30% dup, k=65536, hash={hash_kind}, order={order}",
            "elements": n, "seconds_end_to_end": t, "Gelem_s": n / t / 1e9,
            "filter_launches": passes, "filter_seconds_total": kt,
            "filter_achieved_GBs": read / kt / 1e9, "hbm_frac_filter": read / kt / 1e9 / HBM}


def c2l(dev):
    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0x5EED0000)
    torch.cuda.synchronize()
    ts = []
    for rep in range(4):
        s = Sampler(k, engine="java_l", seed=0)()
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.sample_all(keys)
        s.result()
        ts.append(time.perf_counter() - t0)
        s.close()
    t = sorted(ts[1:])[1]
    return {"config": "C2 on engine java_l (reference Algorithm L, events replayed on GPU)",
            "elements": n, "seconds": t, "Gelem_s": n / t / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c3,c4,c2l")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    todo = args.only.split(",")
    if "c3" in todo:
        print(json.dumps(c3(dev)), flush=True)
        torch.cuda.empty_cache()
    if "c4" in todo:
        print(json.dumps(c4(dev, "identity")), flush=True)
        print(json.dumps(c4(dev, "default", "set")), flush=True)
        print(json.dumps(c4(dev, "default")), flush=True)  # auto -> ordered (exact ties)
        torch.cuda.empty_cache()
    if "c4o" in todo:  # default hash, auto -> ordered only (for traces)
        print(json.dumps(c4(dev, "default")), flush=True)
    if "c4i" in todo:  # identity hash only (for traces)
        print(json.dumps(c4(dev, "identity")), flush=True)
    if "c2l" in todo:
        print(json.dumps(c2l(dev)), flush=True)


if __name__ == "__main__":
    main()
