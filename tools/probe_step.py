"""Where does a bench step's time go beyond K1?  (development probe)"""
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
n, k = 1_000_000_000, 1024
keys = torch.empty(n, dtype=torch.int64, device=dev)
splitmix_fill(keys, 0x5EED0000)
st = torch.cuda.current_stream()
L = _native.load()


def mk():
    s = Sampler(k, seed=1, stream_id=2)()
    s.set_stream(st.cuda_stream)
    return s


def run(label, fn, reps=20):
    ss = [mk() for _ in range(reps + 3)]
    for s in ss[:3]:
        fn(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in ss[3:]:
        fn(s)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    print(f"{label:40s} {t * 1e6:8.1f} us/step", flush=True)


run("sample_all only", lambda s: s.sample_all(keys))
run("sample_all + result", lambda s: (s.sample_all(keys), s.result()))
run("seek + sample_all + result", lambda s: (s.seek(0), s.sample_all(keys), s.result()))


def raw(s):
    L.rsv_sample_batch(s.handle, C.c_void_p(keys.data_ptr()), n, 1, None)
    out = (C.c_int64 * k)()
    m = C.c_int64()
    L.rsv_result(s.handle, out, k, C.byref(m))


run("raw ctypes sample_batch + result", raw)
small = keys[:1_000_000]
run("1e6 keys: sample_all + result", lambda s: (s.sample_all(small), s.result()))
tiny = keys[:1000]
run("1e3 keys: sample_all + result", lambda s: (s.sample_all(tiny), s.result()))


def timed_loop(label, body, reps=50):
    for _ in range(5):
        body()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        body()
    torch.cuda.synchronize()
    print(f"{label:40s} {(time.perf_counter() - t0) / reps * 1e6:8.1f} us/step", flush=True)


timed_loop("create(private stream) + close", lambda: Sampler(k, seed=1, stream_id=2)().close())
timed_loop("create + set_stream + close", lambda: mk().close())
rs = Sampler(k, seed=1, stream_id=2, reusable=True)()
rs.set_stream(st.cuda_stream)
timed_loop("reusable: 1e3 keys sample_all + result", lambda: (rs.sample_all(tiny), rs.result()))
timed_loop("reusable: 1e9 keys sample_all + result", lambda: (rs.sample_all(keys), rs.result()))


def full(x):
    s = mk()
    s.seek(0)
    s.sample_all(x)
    r = s.result()
    s.close()
    return r


timed_loop("full step incl create/close, 1e3", lambda: full(tiny))
timed_loop("full step incl create/close, 1e9", lambda: full(keys))
