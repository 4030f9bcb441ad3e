"""Fixed cost of bench.py's timed region (development probe): host time of one step's issue() and
finish(), and the timed region at K = 20 and K = 100 with the bench's own step functions."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import splitmix_fill  # noqa: E402
from reservoir_amd import Sampler  # noqa: E402
import collections  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, k = 1_000_000_000, 1024
keys = torch.empty(n, dtype=torch.int64, device=dev)
splitmix_fill(keys, 0x5EED0000)
stream = torch.cuda.current_stream(dev).cuda_stream


def issue():
    s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, device=0)()
    s.set_stream(stream)
    s.seek(0)
    s.sample_all(keys)
    return s


def finish(s):
    r = s.result()
    s.close()
    return r


def run_steps(count, depth=2):
    pending = collections.deque()
    for _ in range(count):
        pending.append(issue())
        if len(pending) >= depth:
            finish(pending.popleft())
    while pending:
        finish(pending.popleft())


for _ in range(3000):  # ramp
    finish(issue())
run_steps(200)
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = issue()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    finish(s)
    t3 = time.perf_counter()
    print(f"issue host {1e6 * (t1 - t0):.1f} us, to GPU idle {1e6 * (t2 - t0):.1f} us, finish after idle {1e6 * (t3 - t2):.1f} us",
          flush=True)
for K in (20, 100, 20, 100, 20, 100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(K)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"K={K}: {1e6 * t:.0f} us, {1e6 * t / K:.1f} us/step", flush=True)
