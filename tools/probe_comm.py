"""The N>1 bench step's stream hand-over without a collective (development probe): a fresh Sampler
samples 1e9 device keys on stream A, then its combine kernels (export_packed -> merge_packed, the
all_gather left out) run on stream B after rsv_set_stream; two steps in flight, as bench.py.
Modes: "same" (everything on A) and "comm" (the combine on B).  Prints ms per step for each."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import workloads  # noqa: E402
from reservoir_amd import Sampler  # noqa: E402

dev = torch.device("cuda", 0)
n, k = 1_000_000_000, 1024
keys = torch.empty(n, dtype=torch.int64, device=dev)
workloads.splitmix_fill(keys, 0x5EED0000, 1 << 27)
A = torch.cuda.current_stream(dev)
B = torch.cuda.Stream(dev)
torch.cuda.synchronize()


def issue(mode):
    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
    s.set_stream(A.cuda_stream)
    s.sample_all(keys)
    strm = A if mode == "same" else B
    if mode != "same":
        s.set_stream(B.cuda_stream)
    with torch.cuda.stream(strm):
        rows = torch.empty((2, 2 * k), dtype=torch.int64, device=dev)
        s.export_packed(rows[0])
        s.export_packed(rows[1])
        s.merge_packed(rows, n)
    return s


def run(mode, steps):
    pending = None
    for _ in range(steps):
        s = issue(mode)
        if pending is not None:
            pending.result()
            pending.close()
        pending = s
    pending.result()
    pending.close()


for rnd in range(2):
    for mode in ("same", "comm"):
        run(mode, 300)  # ramp
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(mode, 200)
        torch.cuda.synchronize()
        print(f'{{"mode": "{mode}", "round": {rnd}, "ms_per_step": {(time.perf_counter() - t0) / 200 * 1e3:.4f}}}', flush=True)
