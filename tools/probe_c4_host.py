"""Host-side split of one C4 ordered sampleAll + result(): where the end-to-end time goes beyond the
kernels (dev probe; bench_paths.py c4 reports the end-to-end figure)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from workloads import c4_data  # noqa: E402


def main():
    import ctypes as C

    from reservoir_amd import Sampler, _native as N

    L = N.load()

    dev = torch.device("cuda", 0)
    n, k = 500_000_000, 65536
    vals = c4_data(n, dev)
    torch.cuda.synchronize()
    for order, hk in (("auto", "default"), ("auto", "identity")):
        rows = []
        for rep in range(16):
            mk = Sampler.distinct(k, seed=7, order=order)
            d = mk() if hk == "default" else mk(hash=hk)
            d.set_stream(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d.sample_all(vals)
            t1 = time.perf_counter()
            if rep % 2:
                r = d.result()
                t2 = time.perf_counter()
                tc = 0.0
            else:  # the C call alone, into a buffer touched beforehand
                out = np.ones(k, dtype=np.int64)
                n_ = C.c_int64(0)
                t1 = time.perf_counter()
                N.check(L.rsv_result(d.handle, out.ctypes.data_as(C.c_void_p), k, C.byref(n_)))
                t2 = time.perf_counter()
                tc = 1.0
            d.close()
            if rep >= 2:
                rows.append((t1 - t0, t2 - t1, tc))
        a = np.array(rows)
        py = a[a[:, 2] == 0] * 1e6
        cc = a[a[:, 2] == 1] * 1e6
        print(f"{hk}/{order}: sample_all median {np.median(a[:, 0]) * 1e6:.1f} us, result() median {np.median(py[:, 1]):.1f} us, "
              f"rsv_result alone {np.median(cc[:, 1]):.1f} us")
    # the Python mirror's share: sample_all vs the bare ctypes call with its arguments prepared
    for hk in ("identity", "default"):
        rows = []
        for rep in range(14):
            mk = Sampler.distinct(k, seed=7)
            d = mk() if hk == "default" else mk(hash=hk)
            d.set_stream(torch.cuda.current_stream().cuda_stream)
            ptr = C.c_void_p(vals.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if rep % 2:
                d.sample_all(vals)
            else:
                N.check(L.rsv_sample_batch(d.handle, ptr, n, N.MEM_DEVICE, None))
            t1 = time.perf_counter()
            d.result()
            d.close()
            if rep >= 2:
                rows.append((t1 - t0, rep % 2))
        a = np.array(rows)
        print(f"{hk}: sample_all {np.median(a[a[:, 1] == 1, 0]) * 1e6:.1f} us, bare rsv_sample_batch "
              f"{np.median(a[a[:, 1] == 0, 0]) * 1e6:.1f} us")
    # the copy alone: 512 KB from a fresh numpy buffer vs a reused one
    src = torch.empty(k, dtype=torch.int64, pin_memory=True)
    ts, tr = [], []
    buf = np.empty(k, dtype=np.int64)
    s = src.numpy()
    for _ in range(20):
        t0 = time.perf_counter()
        o = np.empty(k, dtype=np.int64)
        o[:] = s
        t1 = time.perf_counter()
        buf[:] = s
        t2 = time.perf_counter()
        ts.append(t1 - t0)
        tr.append(t2 - t1)
    print(f"512 KB copy from pinned: into a fresh array {np.median(ts) * 1e6:.1f} us, into a reused one {np.median(tr) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
