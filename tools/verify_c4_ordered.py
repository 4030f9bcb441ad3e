"""Full-size parity of the ordered distinct path (development check, not part of the test suite):
C4's per-GPU share (5e8 keys, 30 % duplicates, k = 65536) under the default Long.hashCode, one
sampler seed per run, GPU set vs the oracle's sequential RandomValues restatement
(oracle/oracle.c, Sampler.scala:394-409) over the same keys in the same order.  Also reports the
GPU wall time of sampleAll + result per seed: the seeds whose boundary hash bucket is
oversubscribed pay the host replay of the logged candidates (ordered mode).

  python tools/verify_c4_ordered.py [--n 500000000] [--seeds 7,8,9,...]   -> one JSON line per seed
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000_000)
    ap.add_argument("--k", type=int, default=65536)
    ap.add_argument("--seeds", default="7,8,9,10,11,12,13,14")
    args = ap.parse_args()
    from bench_paths import c4_data

    from oracle import oracle as O
    from reservoir_amd import Sampler

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    vals = c4_data(args.n, dev)
    host = vals.cpu().numpy()
    for seed in (int(s) for s in args.seeds.split(",")):
        d = Sampler.distinct(args.k, seed=seed)()  # Long.hashCode -> order "auto" = ordered
        d.set_stream(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.sample_all(vals)
        got = d.result()
        t1 = time.perf_counter()
        ref = O.Distinct(args.k, seed, O.HASH_JAVA_LONG)
        c0 = time.perf_counter()
        ref.sample_all(host)
        want, wh = ref.result()
        c1 = time.perf_counter()
        top = int(wh.max())
        print(json.dumps({"seed": seed, "n": args.n, "k": args.k, "gpu_ms": round((t1 - t0) * 1e3, 3),
                          "oracle_s": round(c1 - c0, 2), "match": sorted(got.tolist()) == sorted(want.tolist()),
                          "size": int(got.size), "tied_at_max_in_result": int((wh == top).sum())}), flush=True)


if __name__ == "__main__":
    main()
