"""K1 launch time vs the stream (HW queue) it is launched on (development probe, run under
rocprofv3 --kernel-trace; tools/trace_phases.py groups the durations).

  python3 tools/probe_k1env.py

After a 0.3 s ramp, three rounds of: 40 bench steps (fresh Sampler, sample_all over 1e9 device
keys, result(), close) on the sampler's own stream, on torch's current (null) stream, and on a
created torch stream, separated by 1-element torch fill kernels (phase markers).
"""
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
mark = torch.zeros(1, device=dev)
torch.cuda.synchronize()

t = time.perf_counter()
s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, reusable=True)()
while time.perf_counter() - t < 0.3:
    s.sample_all(keys)
    torch.cuda.synchronize()
s.close()
created = torch.cuda.Stream(dev)
for rnd in range(3):
    for label, strm in (("own", None), ("null", torch.cuda.current_stream(dev)), ("created", created)):
        mark.fill_(1)
        torch.cuda.synchronize()
        for _ in range(40):
            s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
            if strm is not None:
                s.set_stream(strm.cuda_stream)
            s.sample_all(keys)
            s.result()
            s.close()
        torch.cuda.synchronize()
        print(rnd, label, flush=True)
mark.fill_(1)
torch.cuda.synchronize()
