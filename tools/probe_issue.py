"""Host time of one bench step's issue() by part (development probe): Sampler creation, set_stream,
seek, sample_all; and finish(): result, close.  Medians over 2000 steps, GPU busy throughout."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import splitmix_fill  # noqa: E402
from reservoir_amd import Sampler  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, k = 1_000_000_000, 1024
keys = torch.empty(n, dtype=torch.int64, device=dev)
splitmix_fill(keys, 0x5EED0000)
stream = torch.cuda.current_stream(dev).cuda_stream
parts = {p: [] for p in ("create", "set_stream", "seek", "sample_all", "result", "close")}
prev = None
for it in range(2200):
    t0 = time.perf_counter()
    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, device=0)()
    t1 = time.perf_counter()
    s.set_stream(stream)
    t2 = time.perf_counter()
    s.seek(0)
    t3 = time.perf_counter()
    s.sample_all(keys)
    t4 = time.perf_counter()
    if prev is not None:
        t5 = time.perf_counter()
        prev.result()
        t6 = time.perf_counter()
        prev.close()
        t7 = time.perf_counter()
        if it >= 200:
            parts["result"].append(t6 - t5)
            parts["close"].append(t7 - t6)
    if it >= 200:
        for name, a, b in (("create", t0, t1), ("set_stream", t1, t2), ("seek", t2, t3), ("sample_all", t3, t4)):
            parts[name].append(b - a)
    prev = s
prev.result()
prev.close()
for name, v in parts.items():
    print(f"{name:12s} median {1e6 * statistics.median(v):6.1f} us  p90 {1e6 * sorted(v)[len(v) * 9 // 10]:6.1f} us")
