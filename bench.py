"""Headline benchmark: C2 = one stream of 1e9 int64 keys per GPU, k = 1024, Algorithm R (philox_r).

A step is one full pass of the hot path over the batch: a fresh Sampler (Sampler.apply, created
and closed inside the step) samples the device-resident keys (K1 last-writer kernel + resolve),
then result() brings the k-slot reservoir to the host.  Two steps are in flight (step t+1's
sampling is queued on the stream before step t's result is read, so the host turnaround overlaps
the GPU); the one-at-a-time figure is reported beside it ("serial"; --serial times that instead).
(RSV_BENCH_RESOLVE_STREAM=1 moves each step's one-workgroup slot resolve + publication to a second
stream after its K1, rsv_set_resolve_stream: measured slower, off by default.)  With N GPUs the stream is N x 1e9 elements
split by index range (each rank seeks to its offset, weak scaling) and the per-rank reservoirs are
combined with one all_gather + merge kernel inside the step.

  python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N > 1 without a torch.distributed environment (WORLD_SIZE unset) launches N ranks itself
(a torch.distributed.run child process; this process never touches the GPU).  Inside a launched
job WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0 (contract in the task statement), including
  roofline      -- K1's VALU roofline (tools/roofline.py): algorithmic Philox calls per launch over
                   the fused kernel's average launch time, measured with HIP events on the
                   sampler's stream, against the gfx950 issue peak; HBM traffic from PMC
  cpu_baseline  -- the oracle's C restatement of the reference (Algorithm L / RandomValues) on the
                   host cores, median of 5 runs per leg (C2 headline leg on one core; C1, C3 on
                   all cores, C4 prefix)
  secondary     -- (N = 1) the other configs of BASELINE.json: C3 segmented (roofline on its
                   binding bound, the winners' 128-B HBM lines, beside K2's VALU model), C4
                   distinct (identity; Long.hashCode in set and ordered order; the ordered replay
                   branch; 16-byte UUID keys), C2 on engine java_l (tools/bench_paths.py), C5
                   sustained elem/s at k = 1 Mi (tools/bench_c5)
  c4            -- (N > 1) C4 at its own definition: N x 5e8 keys split by rank (4e9 at N = 8),
                   distinct sampling + distributed.combine inside the timed step, both hashes, the
                   merged set checked against one sampler over the whole stream (c4_leg)
"""
from __future__ import annotations

import argparse
import collections
import ctypes as C
import json
import mmap
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "elements sampled/sec (Gelem/s) + % HBM roofline, 1B Long keys k=1024, 1/2/4/8 GPU"


def splitmix_fill(out, base: int, chunk: int = 1 << 27) -> None:
    """key[i] = splitmix64(0x5EED0000 + i), generated on the device."""
    import workloads

    workloads.splitmix_fill(out, base, chunk)


def _median(fn, reps: int = 5) -> float:
    return statistics.median(fn() for _ in range(reps))


def host_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs this job may use per the cgroup v2 cpu.max quota (None when unlimited / unreadable)."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(k: int, n_stream: int, seed: int, c4_host=None) -> dict:
    """The oracle (C restatement of Sampler.scala) on the host, median of 5 runs per leg.

    The headline leg (`value`) is C2's streaming path: per-element sample() (Sampler.scala:248-259,
    what the akka operator calls) on ONE core -- the reference sampler is single-threaded
    (Sampler.scala:18-19).  Bounded samples keep the whole baseline at ~15-30 s of CPU work.
    """
    from oracle import oracle as O

    L = O.lib()
    quota = cpu_quota()
    out = np.zeros(max(k, 1 << 10), dtype=np.int64)
    op = out.ctypes.data_as(C.c_void_p)
    legs = []

    # C2, per-element: a 2.5e8-element sample of the stream (a 2e7-key prefix replayed)
    buf_n = 20_000_000
    keys = O.splitmix_keys(0x5EED0000, buf_n)
    reps = 12
    t = _median(lambda: L.or_time_algo_l_per_element(k, seed, keys, buf_n, reps, op))
    per_elem = reps * buf_n / t / 1e9
    # C2, sampleAll(IndexedSeq) skip path over the full 1e9 length: an untouched zero-page mapping
    # stands in for the 8 GB array (the path reads only ~k ln(n/k) elements, all of them zeros)
    zbuf = mmap.mmap(-1, n_stream * 8)
    addr = C.addressof(C.c_char.from_buffer(zbuf))
    # one untimed pass first: it maps every page the walk reads (the same ~14 k elements each run,
    # same seed), so the timed runs read resident memory as the reference's array would be
    L.or_time_algo_l_indexed(k, seed, C.c_void_p(addr), n_stream, op)
    ts = _median(lambda: L.or_time_algo_l_indexed(k, seed, C.c_void_p(addr), n_stream, op))
    del addr
    zbuf.close()
    legs.append({"config": "C2 sampleAll(IndexedSeq) skip path (Sampler.scala:261-273)", "cores": 1,
                 "Gelem_s": round(n_stream / ts / 1e9, 2),
                 "sample": f"{n_stream:.0e} elements, k={k}; input = a zero-page mapping whose pages the walk "
                           "reads were mapped by an untimed first pass (the path touches ~k ln(n/k) elements, "
                           "so their values do not matter)"})

    # C1: 10 M Longs (the first 1e7 of the C2 stream), k = 100, both samplers
    n1, k1 = 10_000_000, 100
    c1 = keys[:n1]
    t = _median(lambda: L.or_time_algo_l_per_element(k1, seed, c1, n1, 1, op))
    legs.append({"config": "C1 Sampler(100) per-element sample()", "cores": 1, "Gelem_s": round(n1 / t / 1e9, 4),
                 "sample": "1e7 keys"})
    t = _median(lambda: L.or_time_algo_l_indexed(k1, seed, c1.ctypes.data_as(C.c_void_p), n1, op))
    legs.append({"config": "C1 Sampler(100) sampleAll(IndexedSeq)", "cores": 1, "Gelem_s": round(n1 / t / 1e9, 2),
                 "sample": "1e7 keys"})
    for hk, name in ((O.HASH_JAVA_LONG, "Long.hashCode (default)"), (O.HASH_IDENTITY, "identity")):
        t = _median(lambda: L.or_time_distinct(k1, seed, hk, c1, n1))
        legs.append({"config": f"C1 Sampler.distinct(100), hash = {name}, per element", "cores": 1,
                     "Gelem_s": round(n1 / t / 1e9, 4), "sample": "1e7 keys"})

    # C3: one reference sampler per stream (4096 Longs, k = 64) on every host core (nproc
    # affinity cores), and on the CPU quota the box grants this job (cgroup cpu.max) when it is smaller
    S3, L3 = 1 << 16, 4096
    k3 = O.splitmix_keys(0, S3 * L3)
    counts = [host_cores()]
    if quota and quota < host_cores():
        counts.append(max(1, int(quota)))
    for threads in counts:
        for mode, name in ((0, "per-element sample()"), (1, "sampleAll(IndexedSeq)")):
            t = _median(lambda: L.or_time_segmented_algo_l(64, k3, S3, L3, mode, threads, None), 3)
            legs.append({"config": f"C3 one Sampler(64) per stream, {name}", "cores": threads,
                         "Gelem_s": round(S3 * L3 / t / 1e9, 3),
                         "sample": f"2^16 of the 2^20 streams x {L3} keys on {threads} threads"
                                   + (" (all affinity cores)" if threads == host_cores() else
                                      " (the job's cgroup CPU quota)")})
    del k3

    # C4: Sampler.distinct(65536) over a prefix of one GPU's C4 share, both hashes of BASELINE.md
    if c4_host is not None:
        n4 = c4_host.size
        for hk, name in ((O.HASH_JAVA_LONG, "Long.hashCode (default)"), (O.HASH_IDENTITY, "identity")):
            t = _median(lambda: L.or_time_distinct(65536, 7, hk, c4_host, n4), 3)
            legs.append({"config": f"C4 Sampler.distinct(65536), hash = {name}, per element", "cores": 1,
                         "Gelem_s": round(n4 / t / 1e9, 4),
                         "sample": f"the first {n4:.1e} keys of C4's per-GPU share (30 % duplicates, Feistel order); "
                                   "median of 3"})
    return {
        "value": round(per_elem, 4),
        "unit": "Gelem/s",
        "cores": 1,
        "kind": "port",
        "sample": f"per-element sample() (Algorithm L, Sampler.scala:248-259) over one stream of "
                  f"{reps * buf_n:.3g} keys (a {buf_n:.0e}-key C2 prefix replayed {reps}x), k={k}; median of 5",
        "host_cores": host_cores(),
        "cpu_quota_cores": quota,
        "legs": legs,
    }


def secondary(dev) -> list:
    """The other hot-path configs of BASELINE.json (not the headline `value`).  Same measurement
    code as tools/bench_paths.py; a failure here is reported in the entry, never fails the line."""
    import torch

    import bench_paths as P

    out = []
    jobs = [("C3", lambda: P.c3(dev)), ("C4 identity", lambda: P.c4(dev, "identity")),
            ("C4 default/set", lambda: P.c4(dev, "default", "set")),
            ("C4 default/ordered", lambda: P.c4(dev, "default")),
            ("C4 default/ordered replay branch", lambda: P.c4_replay(dev)),
            ("C2 java_l", lambda: P.c2l(dev)), ("C2 indexed", lambda: P.c2_indexed(dev)),
            ("C2 host buffer", lambda: P.c2_host(dev)),
            ("C4 combine", lambda: P.c4_merge(dev)),
            ("C4 16-byte UUID keys, set", lambda: P.c4_wide(dev, "set")),
            ("C4 16-byte UUID keys, ordered", lambda: P.c4_wide(dev, "uuid"))]
    for name, fn in jobs:
        try:
            rs = fn()
        except Exception as ex:  # noqa: BLE001 -- reported, not raised
            rs = {"config": name, "error": f"{type(ex).__name__}: {ex}"}
        for r in (rs if isinstance(rs, list) else [rs]):
            out.append({kk: (round(v, 6) if isinstance(v, float) else v) for kk, v in r.items()})
        torch.cuda.empty_cache()
    return out


def c5_legs(n: int = 200_000_000) -> list:
    """C5 (BASELINE.json configs[4]): sustained elem/s of a per-element source feeding the sampler
    through the C ABI at k = 1 Mi -- rsv_sample per element (what SampleImpl.onPush does,
    SampleImpl.scala:27-31) and zero-copy pinned batches (rsv_stage_acquire/commit), both engines.
    tools/bench_c5 (built by __graft_entry__.build) prints one JSON object per leg."""
    exe = os.path.join(ROOT, "tools", "bench_c5")
    if not os.path.exists(exe):
        return [{"config": "C5", "error": f"{exe} not built (__graft_entry__.build)"}]
    r = subprocess.run([exe, str(n), str(1 << 20)], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return [{"config": "C5", "error": f"bench_c5 rc={r.returncode}: {r.stderr[-400:]}"}]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def c4_leg(args, rank: int, world: int, dev, backend: str) -> dict:
    """C4 (BASELINE.json configs[3]) at N ranks: a stream of N x 5e8 Long keys (30 % duplicates; at
    N = 8 the 4e9-key workload) split by rank, k = 65536.  A step: every rank creates a distinct
    sampler, samples its contiguous 5e8 piece (device-resident), distributed.combine merges the
    ranks' sets (one all_gather; the exact replay for the default hash when its boundary bucket is
    tied), result() to the host, close.  Timed like the headline (barrier + synchronize, max over
    ranks); afterwards rank 0 checks the merged set against ONE sampler fed the whole stream."""
    import torch
    import torch.distributed as dist

    import workloads
    from reservoir_amd import Sampler
    from reservoir_amd import distributed as D

    piece, k = args.c4_keys, 65536
    total = piece * world
    keys = workloads.c4_slice(total, rank * piece, (rank + 1) * piece, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = {"workload": f"C4: distinct over {total:.2e} Long keys (30% duplicates, Feistel order), k=65536, "
                       f"{world} ranks x {piece:.1e} contiguous keys, merged by distributed.combine",
           "ranks": world, "backend": backend, "legs": []}

    def make(hash_kind):
        mk = Sampler.distinct(k, seed=7, retain_log=hash_kind == "default")  # the exact replay reads the log
        return mk(hash="identity") if hash_kind == "identity" else mk()

    for hash_kind in ("identity", "default"):
        replays = 0
        marks = []  # per timed step: events before sampling / before the combine / inside it / after it

        def step(mark=False):
            nonlocal replays
            s = make(hash_kind)
            s.set_stream(stream)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if mark else None
            if ev:
                ev[0].record()
            s.sample_all(keys)
            if ev:
                ev[1].record()
            inner = [] if mark else None  # after the export / the all-gather / the device merge
            replays += D.combine(s, device=dev, total_count=total, marks=inner)
            if ev:
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[2].record()
                marks.append(ev + inner)
            r = s.result()
            s.close()
            return r

        for _ in range(args.c4_warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        replays = 0
        t0 = time.perf_counter()
        res = None
        for _ in range(args.c4_steps):
            res = step(mark=True)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        # the step split on the stream's own clock (events around sample_all and around combine:
        # the all-gather, the device merge, and for the default hash its one host read-back)
        samp = statistics.median(m[0].elapsed_time(m[1]) for m in marks)
        comb = statistics.median(m[1].elapsed_time(m[2]) for m in marks)
        gather = statistics.median(m[3].elapsed_time(m[4]) for m in marks)
        merge = statistics.median(m[4].elapsed_time(m[5]) for m in marks)
        export = statistics.median(m[1].elapsed_time(m[3]) for m in marks)
        leg = {"hash": hash_kind + (" (Long.hashCode, ordered: exact sequential set)" if hash_kind == "default"
                                    else " (set mode, bit-exact bottom-k)"),
               "steps": args.c4_steps, "ms_per_step": round(elapsed / args.c4_steps * 1e3, 4),
               "Gelem_s": round(total * args.c4_steps / elapsed / 1e9, 3), "exact_replays": replays,
               "sample_ms_median": round(samp, 4), "combine_ms_median": round(comb, 4),
               "combine_split_ms": {"export_row": round(export, 4), "all_gather": round(gather, 4),
                                    "device_merge": round(merge, 4)},
               "split_clock": "HIP events on the sampler's (torch's) stream, this rank"}
        if rank == 0:  # the merged set vs one sampler over the whole stream (same seed, same hash)
            full = workloads.c4_slice(total, 0, total, dev)
            one = make(hash_kind)
            one.sample_all(full)
            want = np.sort(one.result())
            one.close()
            del full
            torch.cuda.empty_cache()
            leg["matches_single_sampler"] = bool(np.array_equal(np.sort(res), want))
        out["legs"].append(leg)
    del keys
    torch.cuda.empty_cache()
    return out


def load_traffic(n: int):
    """HBM bytes per K1 launch from the committed PMC pass (profiles/), if one matches n."""
    for path in (os.path.join(ROOT, "profiles", r, "pmc_k1.json") for r in ("r05", "r04", "r03", "r02", "")):
        try:
            d = json.load(open(path))
            if int(d.get("n", -1)) == n:
                return d.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    return None


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args) -> int:
    """--gpus N > 1 outside a torch.distributed job: run N ranks (one per GPU) in a child
    torch.distributed.run.  Nothing here initialises the GPU (device_count does not, on ROCm)."""
    import torch

    have = torch.cuda.device_count()
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this node has {have}; "
              "refusing to run fewer ranks than requested", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--keys-per-gpu", dest="n", type=int, default=1_000_000_000)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=0xC0FFEE)
    ap.add_argument("--stream-id", type=int, default=0x5A5A)
    ap.add_argument("--time-every", type=int, default=2,
                    help="HIP events around every N-th K1 launch of the timed steps (1 = every launch): "
                         "every 2nd times 10 launches of the driver's 20-step form; against every 6th (3 "
                         "launches) the headline moved < 0.5 %% (profiles/r06/bench_time_every_ab.jsonl)")
    ap.add_argument("--serial", action="store_true",
                    help="one step at a time (no second sampler in flight) for the timed steps")
    ap.add_argument("--depth", type=int, default=int(os.environ.get("RSV_BENCH_DEPTH", "2")),
                    help="samplers in flight (each step still creates, samples, reads and closes its own)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the other hot-path configs (C3 segmented, C4 distinct, C2 on java_l, C5)")
    ap.add_argument("--c4-keys", type=int, default=500_000_000, help="C4 keys per rank (N > 1 leg)")
    ap.add_argument("--c4-steps", type=int, default=10)
    ap.add_argument("--c4-warmup", type=int, default=2)
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 leg at N > 1")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

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
    import roofline as R

    n, k = args.n, args.k
    offset = rank * n
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0x5EED0000 + offset)
    stream = torch.cuda.current_stream(dev).cuda_stream
    # N > 1 over RCCL: each step's combine (export, all-gather, merge) runs on a communication
    # stream, handed over from the sampling stream by an event (rsv_set_stream), so the next step's
    # K1 is not queued behind this step's collective.  (Not under gloo: its all-gather of CUDA
    # tensors waits on the host for the stream it runs on, which then serialises the steps -- the
    # 2-rank rehearsal ran 0.54 -> 1.05 ms per step with it.)
    comm = torch.cuda.Stream(device=dev) if world > 1 and backend == "nccl" else None
    # RSV_BENCH_RESOLVE_STREAM=1: each step's slot resolve + result publication (a one-workgroup
    # dispatch, ~5 us) on a second stream after its K1 (rsv_set_resolve_stream), so the next step's
    # K1 need not queue behind it.  Off by default: measured slower (r05j, same box, A/B/A/B: 0.0915
    # and 0.0919 ms per step without, 0.0939 and 0.0963 with; K1 86.8 -> 89-90 us -- the dispatch
    # running beside K1 costs K1 more than the queueing it saves)
    rstream = (torch.cuda.Stream(device=dev).cuda_stream
               if os.environ.get("RSV_BENCH_RESOLVE_STREAM", "0") == "1" else None)

    L = _native.load()

    def issue():
        # a fresh Sampler per step (Sampler.apply): creation and close are inside the step.  On the
        # caller's stream sample_all and the combine are stream-ordered: nothing here waits
        s = Sampler(k, seed=args.seed, stream_id=args.stream_id, device=local)()
        s.set_stream(stream)
        if rstream is not None:
            s.set_resolve_stream(rstream)
        s.seek(offset)
        s.sample_all(keys)
        if comm is not None:
            s.set_stream(comm.cuda_stream)
            with torch.cuda.stream(comm):
                D.combine(s, device=dev, total_count=n * world)
        elif world > 1:
            D.combine(s, device=dev, total_count=n * world)
        return s

    def finish(s):
        r = s.result()  # waits for this step's published reservoir
        s.close()
        return r

    def step():
        return finish(issue())

    def run_steps(count: int, depth: int):
        """`count` steps with `depth` samplers in flight: step t + depth - 1 is issued (its kernels
        queue behind the earlier steps' on the stream) before step t's result() is read, so the
        host's result / close / create turnaround overlaps the GPU's next steps instead of idling
        it.  Every step still creates its sampler, samples all keys, reads its result and closes."""
        res = None
        pending = collections.deque()
        for _ in range(count):
            pending.append(issue())
            if len(pending) >= depth:
                res = finish(pending.popleft())
        while pending:
            res = finish(pending.popleft())
        return res

    def profile_read():
        ms, cnt = C.c_double(), C.c_int64()
        _native.check(L.rsv_profile_global_read(C.byref(ms), C.byref(cnt)))
        return ms.value, cnt.value

    # Device warm-up (untimed): under sustained load the K1 launch time falls as clocks ramp (98-104
    # -> 88-90 us over tens of ms, tools/probe_k1env.py); run steps for 0.3 s before the W warmup
    # steps so the timed region sees the steady state.  Every step holds a collective at N>1, so
    # all ranks run the same number of steps, agreed as the max over ranks.  The count comes from
    # steps timed AFTER the first one: the first carries the one-time module load and pool
    # allocations, and timed alone it shrank the ramp to a handful of steps (the timed region
    # then ran K1 at ~96 us on a still-ramping clock).
    step()
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    run_steps(8, 1)
    torch.cuda.synchronize()
    n_ramp = max(1, int(0.3 / max((time.perf_counter() - t_w) / 8, 1e-5)))
    if world > 1:
        t = torch.tensor([min(n_ramp, 10_000)], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_ramp = int(t.item())
    depth = 1 if args.serial else max(1, args.depth)
    run_steps(min(n_ramp, 10_000), depth)
    run_steps(args.warmup, depth)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # K1 timing: HIP events around every N-th K1 launch of the timed steps (process-wide list,
    # drained after the timed region; rsv_profile_global in include/reservoir_hip.h).  Each event
    # pair adds marker packets to its step; every 2nd step carries them (the 20-step form: 10 launches).
    # (the library times the (every/2)-th launch first: a region's first launch finds the GPU idle
    # and its event pair would include the host's submission latency)
    _native.check(L.rsv_profile_global(max(1, min(args.time_every, args.steps // 2))))
    t0 = time.perf_counter()
    res = run_steps(args.steps, depth)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _native.check(L.rsv_profile_global(0))
    k1_ms, k1_launches = profile_read()
    # the same steps one at a time (issue -> result -> close, nothing in flight): reported beside
    # the pipelined figure, same barrier / synchronize bracketing, not the headline
    serial_steps = min(args.steps, 40)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run_steps(serial_steps, 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed_serial = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([elapsed, elapsed_serial], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_serial = float(t[0].item()), float(t[1].item())

    k1_s = k1_ms / max(k1_launches, 1) / 1e3  # K1 launch time (HIP events on the launch stream)
    assert res is not None and res.size == k

    c4 = None
    if world > 1 and not args.no_c4:
        del keys
        torch.cuda.empty_cache()
        c4 = c4_leg(args, rank, world, dev, backend)

    if rank == 0:
        total = n * world * args.steps
        l0, l1 = R.k1_calls(n, k, offset)
        # the runtime fuses K1 with the slot resolve only up to 2^27 draws (rsv_runtime.hip rsv_sample_all)
        fused = os.environ.get("RSV_K1_FUSE") == "1" or (os.environ.get("RSV_K1_FUSE") != "0" and n <= 1 << 27)
        kname = ("k1_resolve_publish (K1 + the last workgroup's resolve/publish tail)" if fused else
                 "k1_last_writer (K1 alone; the slot resolve/publish is a separate one-workgroup dispatch)")
        roof = R.valu_roofline(
            l0, l1, k1_s, kname,
            note="bound = integer VALU (Philox): K1 reads only the k winning keys (draws depend on the index "
                 "alone, like the reference's sampleAll(IndexedSeq) skip, Sampler.scala:261-273), so the "
                 "SURVEY 8(d) 8 B/elem HBM convention would read " +
                 f"{8 * n / k1_s / 1e9:.0f} GB/s (> the 8 TB/s peak): it is not this kernel's bound")
        roof["traffic"] = load_traffic(n)
        roof["launches_timed"] = k1_launches
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
                "parallelism": (f"index-range split over {world} ranks, "
                                f"{'RCCL' if backend == 'nccl' else backend} all_gather combine")
                               if world > 1 else "single GPU",
            },
            "roofline": roof,
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "steps_in_flight": depth,
            "resolve_stream": rstream is not None,
            "serial": {"steps": serial_steps, "ms_per_step": round(elapsed_serial / serial_steps * 1e3, 4),
                       "value": round(n * world * serial_steps / elapsed_serial / 1e9, 3),
                       "what": "the same step run one at a time (result read and sampler closed before the "
                               "next is created): the host turnaround between steps idles the GPU"},
        }
        if c4 is not None:
            line["c4"] = c4
        c4_host = None
        if world == 1 and not args.no_secondary:
            del keys
            torch.cuda.empty_cache()
            line["secondary"] = secondary(dev)
            try:
                line["secondary"] += c5_legs()
            except Exception as ex:  # noqa: BLE001 -- reported, not raised
                line["secondary"].append({"config": "C5", "error": f"{type(ex).__name__}: {ex}"})
        if world == 1 and not args.no_cpu_baseline:
            import workloads

            c4 = workloads.c4_data(500_000_000, dev)
            c4_host = c4[:400_000_000].cpu().numpy()
            del c4
            torch.cuda.empty_cache()
            try:
                line["cpu_baseline"] = cpu_baseline(k, n, args.seed, c4_host)
            except Exception as ex:  # noqa: BLE001 -- the headline line is printed regardless
                line["cpu_baseline"] = {"error": f"{type(ex).__name__}: {ex}"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
