"""Host-side cost of each call in one bench step (development probe): perf_counter around every
call of the C2 step, averaged over many steps."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import splitmix_fill  # noqa: E402
from reservoir_amd import Sampler, _native  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, k = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000, 1024
keys = torch.empty(n, dtype=torch.int64, device=dev)
splitmix_fill(keys, 0x5EED0000)
stream = torch.cuda.current_stream(dev).cuda_stream
L = _native.load()
names = ["create", "set_stream", "prof_on", "seek", "sample_all", "result", "prof_read", "close"]
acc = {x: 0.0 for x in names}


def step(timed, prof):
    t = [time.perf_counter()]
    s = Sampler(k, seed=1, stream_id=2, device=0)()
    t.append(time.perf_counter())
    s.set_stream(stream)
    t.append(time.perf_counter())
    if prof:
        _native.check(L.rsv_profile_enable(s.handle, 1))
    t.append(time.perf_counter())
    s.seek(0)
    t.append(time.perf_counter())
    s.sample_all(keys)
    t.append(time.perf_counter())
    s.result()
    t.append(time.perf_counter())
    if prof:
        ms, cnt = C.c_double(), C.c_int64()
        _native.check(L.rsv_profile_read(s.handle, C.byref(ms), C.byref(cnt)))
    t.append(time.perf_counter())
    s.close()
    t.append(time.perf_counter())
    if timed:
        for i, x in enumerate(names):
            acc[x] += t[i + 1] - t[i]


for prof in (False, True):
    for _ in range(50):
        step(False, prof)
    for x in names:
        acc[x] = 0.0
    reps = 200
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step(True, prof)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / reps
    print(f"n={n} profile={prof}: step {tot * 1e6:.1f} us; " +
          ", ".join(f"{x} {acc[x] / reps * 1e6:.1f}" for x in names), flush=True)
