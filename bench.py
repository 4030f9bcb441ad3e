"""Headline benchmark: C2 = one stream of 1e9 int64 keys per GPU, k = 1024, Algorithm R (philox_r).

A step is one full pass of the hot path over the batch: a fresh Sampler (Sampler.apply, created
and closed inside the step) samples the device-resident keys (K1 last-writer kernel + resolve),
then result() brings the k-slot reservoir to the host.  With N GPUs the stream is N x 1e9 elements split by index range (each
rank seeks to its offset, weak scaling) and the per-rank reservoirs are combined with one RCCL
all_gather + merge kernel inside the step.

Prints ONE JSON line on rank 0 (contract in the task statement), including
  roofline      -- K1's average launch time, measured with HIP events on the sampler's stream
  cpu_baseline  -- the oracle's C restatement of the reference (Algorithm L) on one host core
  secondary     -- (N = 1) the other configs of BASELINE.json, measured after the headline:
                   C3 segmented, C4 distinct (identity; Long.hashCode in set and ordered order),
                   C2 on engine java_l, and the CPU distinct baseline (tools/bench_paths.py)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import mmap
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "elements sampled/sec (Gelem/s) + % HBM roofline, 1B Long keys k=1024, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_ELEM = 8     # each 64-bit key charged once


def splitmix_fill(out: torch.Tensor, base: int, chunk: int = 1 << 27) -> None:
    """key[i] = splitmix64(0x5EED0000 + i), generated on the device."""
    def s64(c):
        return c - (1 << 64) if c >= 1 << 63 else c

    g, m1, m2 = s64(0x9E3779B97F4A7C15), s64(0xBF58476D1CE4E5B9), s64(0x94D049BB133111EB)
    n = out.numel()
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        z = torch.arange(base + a, base + b, dtype=torch.int64, device=out.device) + g
        z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * m1
        z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * m2
        out[a:b] = z ^ ((z >> 31) & ((1 << 33) - 1))


def cpu_baseline(k: int, n_stream: int, seed: int) -> dict:
    """Time the oracle (C restatement of Sampler.scala) on one host core, bounded to ~10 s."""
    from oracle import oracle as O

    L = O.lib()
    buf_n = 20_000_000
    keys = O.splitmix_keys(0x5EED0000, buf_n)
    out = np.zeros(k, dtype=np.int64)
    t = L.or_time_algo_l_per_element(k, seed, keys, buf_n, 1, out.ctypes.data_as(C.c_void_p))
    reps = max(1, min(int(n_stream // buf_n), int(8.0 / max(t, 1e-3))))
    t = L.or_time_algo_l_per_element(k, seed, keys, buf_n, reps, out.ctypes.data_as(C.c_void_p))
    per_elem = reps * buf_n / t / 1e9
    # sampleAll(IndexedSeq) skip path over the full stream: an untouched zero-page mapping stands in
    # for the 8 GB array (the path reads only ~k ln(n/k) elements)
    zbuf = mmap.mmap(-1, n_stream * 8)
    addr = C.addressof(C.c_char.from_buffer(zbuf))
    ts = L.or_time_algo_l_indexed(k, seed, C.c_void_p(addr), n_stream, out.ctypes.data_as(C.c_void_p))
    del addr
    zbuf.close()
    return {
        "value": round(per_elem, 4),
        "unit": "Gelem/s",
        "cores": 1,
        "kind": "port",
        "sample": f"per-element sample() (Algorithm L, Sampler.scala:248-259) over one stream of "
                  f"{reps * buf_n:.3g} keys (a {buf_n:.0e}-key C2 prefix replayed {reps}x), k={k}",
        "skip_path": {"value": round(n_stream / ts / 1e9, 2), "unit": "Gelem/s",
                      "sample": f"sampleAll(IndexedSeq) skip path (Sampler.scala:261-273) over "
                                f"{n_stream:.0e} elements; touches ~k ln(n/k) of them"},
    }


def valu_roofline(n: int, k1_s: float) -> dict:
    """K1's binding limit: Philox4x32-10 evaluations per second vs the gfx950 VALU peak.

    Per call: 20 v_mad_u64_u32 (3.2 full-rate issue slots each, measured by tools/micro_k1.hip)
    + 20 v_bitop3 = 84 slots; peak = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 84.  Calls per launch
    (expected): one level-0 call per 16 indices, a recompute for the 6.07 % of blocks holding a zero
    byte, and one level-1 call per candidate (1 in 256 indices).
    """
    level0 = n / 16
    calls = level0 * (1 + (1 - (255 / 256) ** 16)) + n / 256
    peak = 256 * 4 * 32 * 2.4e9 / 84 / 1e9
    achieved = calls / k1_s / 1e9
    return {"bound": "valu", "achieved": round(achieved, 1), "peak": round(peak, 1),
            "unit": "GPhilox/s", "frac": round(achieved / peak, 4),
            "calls_per_launch": int(calls)}


def load_traffic(n: int):
    """HBM bytes per K1 launch from the committed PMC pass (profiles/), if one matches n."""
    path = os.path.join(ROOT, "profiles", "pmc_k1.json")
    try:
        d = json.load(open(path))
        if int(d.get("n", -1)) == n:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def secondary(dev, with_cpu: bool) -> list:
    """The other hot-path configs of BASELINE.json (not the headline `value`): C3 segmented,
    C4 distinct (one GPU's share; identity hash, and Long.hashCode in set and ordered order), C2 on
    the reference's Algorithm L (engine java_l).  Same measurement code as tools/bench_paths.py;
    a failure here is reported in the entry, never fails the headline line."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_paths as P

    out = []
    jobs = [("C3", lambda: P.c3(dev)), ("C4 identity", lambda: P.c4(dev, "identity")),
            ("C4 default/set", lambda: P.c4(dev, "default", "set")),
            ("C4 default/ordered", lambda: P.c4(dev, "default")), ("C2 java_l", lambda: P.c2l(dev))]
    for name, fn in jobs:
        try:
            r = fn()
        except Exception as ex:  # noqa: BLE001 -- reported, not raised
            r = {"config": name, "error": f"{type(ex).__name__}: {ex}"}
        out.append({kk: (round(v, 6) if isinstance(v, float) else v) for kk, v in r.items()})
        torch.cuda.empty_cache()
    if with_cpu:
        from oracle import oracle as O

        keys = O.splitmix_keys(0xD15C, 10_000_000)
        t = O.lib().or_time_distinct(65536, 7, O.HASH_IDENTITY, keys, keys.size)
        out.append({"config": "CPU baseline: Sampler.distinct per element (RandomValues restated, "
                              "Sampler.scala:394-409), k=65536, identity hash, 1e7 keys, 1 core",
                    "Gelem_s": round(keys.size / t / 1e9, 4), "kind": "port", "cores": 1})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--keys-per-gpu", dest="n", type=int, default=1_000_000_000)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=0xC0FFEE)
    ap.add_argument("--stream-id", type=int, default=0x5A5A)
    ap.add_argument("--time-every", type=int, default=4,
                    help="HIP events around every N-th K1 launch of the timed steps (1 = every launch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the other hot-path configs (C3 segmented, C4 distinct, C2 on java_l)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RSV_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU
    backend = os.environ.get("RSV_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from reservoir_amd import Sampler, _native
    from reservoir_amd import distributed as D

    n, k = args.n, args.k
    offset = rank * n
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0x5EED0000 + offset)
    stream = torch.cuda.current_stream(dev).cuda_stream

    L = _native.load()
    prof = [0.0, 0]  # K1 milliseconds, launches (timed steps)

    def step():
        # a fresh Sampler per step (Sampler.apply): creation and close are inside the step
        s = Sampler(k, seed=args.seed, stream_id=args.stream_id, device=local)()
        s.set_stream(stream)
        s.seek(offset)
        s.sample_all(keys)
        if world > 1:
            D.combine(s, device=dev, total_count=n * world)
        r = s.result()
        s.close()
        return r

    def profile_read():
        ms, cnt = C.c_double(), C.c_int64()
        _native.check(L.rsv_profile_global_read(C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    # Device warm-up (untimed): under sustained load the K1 launch time falls from ~152 to ~140 us
    # over the first ~30 ms as clocks ramp (rocprofv3 trace); run steps for 0.2 s
    # before the W warmup steps so the timed region sees the steady state.
    # Every step holds a collective at N>1, so all ranks must run the same number of steps: the
    # count comes from one timed step, agreed as the max over ranks.
    t_w = time.perf_counter()
    step()
    torch.cuda.synchronize()
    n_ramp = max(1, int(0.2 / max(time.perf_counter() - t_w, 1e-4)))
    if world > 1:
        t = torch.tensor([min(n_ramp, 10_000)], dtype=torch.int64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_ramp = int(t.item())
    for _ in range(min(n_ramp, 10_000)):
        step()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # K1 timing: HIP events around every N-th K1 launch of the timed steps (process-wide list,
    # drained after the timed region; rsv_profile_global in include/reservoir_hip.h).  Each event
    # pair adds ~5 us of marker packets to its step, so by default one step in four carries them.
    _native.check(L.rsv_profile_global(max(1, args.time_every)))
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _native.check(L.rsv_profile_global(0))
    prof[0], prof[1] = profile_read()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # K1 launch time (HIP events on the launch stream), averaged over the timed steps
    k1_s = prof[0] / max(prof[1], 1) / 1e3
    assert res is not None and res.size == k

    if rank == 0:
        total = n * world * args.steps
        achieved = BYTES_PER_ELEM * n / k1_s / 1e9
        line = {
            "metric": METRIC,
            "value": round(total / elapsed / 1e9, 3),
            "unit": "Gelem/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "C2: single stream, 1e9 int64 keys per GPU (splitmix64), k=1024, "
                            "Algorithm R last-writer (engine philox_r); step = create Sampler, "
                            "sampleAll over device-resident keys, result() to host, close",
                "keys_per_gpu": n, "k": k, "stream_elements": n * world,
                "parallelism": f"index-range split over {world} GPU(s), RCCL all_gather combine"
                               if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(n),
                "kernel": "k1_resolve_publish",
                "launch_avg_us": round(k1_s * 1e6, 2),
                "launches_timed": prof[1],
                "note": "achieved charges 8 B per element (SURVEY.md 8(d)); K1 reads no key "
                        "(draws depend only on the index), so it is bound by Philox integer "
                        "VALU work, not HBM -- see the valu_roofline object and DESIGN.md",
            },
            "valu_roofline": valu_roofline(n, k1_s),
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(k, n, args.seed)
        if world == 1 and not args.no_secondary:
            del keys
            torch.cuda.empty_cache()
            line["secondary"] = secondary(dev, with_cpu=not args.no_cpu_baseline)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
