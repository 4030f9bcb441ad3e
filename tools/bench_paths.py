"""Secondary measurements of the other hot-path configs: not the bench.py line.

  C3  segmented: 2^20 streams x 4096 int64 keys, k = 64 (K2)
  C4g distinct, one GPU's share of C4: 5e8 int64 keys, 30 % duplicates, k = 65536, identity hash
      (K3 filter + merge); also the default Long.hashCode
  C2L the reference's Algorithm L (engine java_l) on C2: 1e9 keys, k = 1024 (K1' replay)
  C2I C2 through the boundary as the JVM binding's sampleAll(IndexedSeq): a 1e9-element host
      sequence sampled by index (rsv_sample_indexed), map + keys only for the <= 1024 winners
  C3K K2 past the LDS winner table (k = 8192, global tables) beside k = 4096 on 4096 x 2^17 keys
  C4M C4's combine on one GPU: 8 shard sets of k = 65536 merged by distributed.merge_local
      (8 x rsv_export_packed + the device rsv_merge_packed), both hashes
  C4W C4's share as 16-byte UUID keys (rsv_wide.hip): a precomputed 64-bit hash in set mode (the
      filter reads the 8-B hashes only), UUID.hashCode in ordered mode (the filter reads the 16-B
      rows), and UUID hash twins (the ordered host replay)

Prints one JSON line per config with the kernel time (HIP events on the launch stream) and the
8-B-per-element HBM roofline fraction.  Usage: python tools/bench_paths.py [--only c3,c4,c2l]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

sys.path.insert(0, os.path.join(ROOT, "tools"))
import roofline as R  # noqa: E402
from workloads import c4_data, hash_twins, splitmix_fill  # noqa: E402

HBM = 8000.0


def ramp(fn, seconds=0.3):
    """Run fn back to back for `seconds` (untimed): VALU-bound launches run ~10 % slower until the
    clock has ramped under sustained load (tools/probe_k1env.py)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        torch.cuda.synchronize()


def timed(fn, reps=5, warm=1):
    ramp(fn)
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def c3(dev):
    from reservoir_amd import batch

    S, L, k = 1 << 20, 4096, 64
    n = S * L
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0)
    offs = torch.arange(0, n + 1, L, dtype=torch.int64, device=dev)
    t = timed(lambda: batch.sample_segmented(keys, offs, k, seed=1), reps=9)
    l0, l1 = R.k2_calls(S, L, k)
    # the memory floor: K2 must fetch each stream's 64 winning keys, ~57 distinct random 128-B lines
    # of its 32 KB segment (7.5 GB per launch by FETCH_SIZE, profiles/r02).  Timed here as a plain
    # gather of 64 uniform random positions per 4096-key row (the last writer of a slot is uniform on
    # [0, n)); tools/micro_gather.hip times the same access as a hand-written kernel (1.40-1.47 ms)
    g = torch.Generator(device=dev)
    g.manual_seed(12345)
    idx = torch.randint(0, L, (S, k), device=dev, generator=g)
    rows = keys.view(S, L)
    t_g = timed(lambda: torch.gather(rows, 1, idx), reps=5)
    del idx
    # The binding bound: HBM lines.  A lone 8-B load moves its whole 128-B line (tools/micro_gather
    # line probes, profiles/r05/gather_line_probe_time.jsonl: both 64-B halves of 32 lines cost what
    # one half twice costs), so a stream's winners cost 128 B per DISTINCT line: 64 uniform positions
    # without replacement in 256 lines touch 256 (1 - C(4080, 64) / C(4096, 64)) ~ 56.6 of them.
    # Plus the output rows (k keys per stream) and the offsets, so the algorithmic bytes and the PMC
    # traffic (reads + writes) count the same things.
    lines = 256.0 * (1.0 - math.exp(sum(math.log((L - 16 - q) / (L - q)) for q in range(k))))
    line_bytes = S * lines * 128 + S * k * 8 + (S + 1) * 8
    traffic = _pmc_traffic("c3")
    hbm = {"bound": "hbm", "achieved": round(line_bytes / t / 1e9, 1), "peak": HBM, "unit": "GB/s",
           "frac": round(line_bytes / t / 1e9 / HBM, 4), "traffic": traffic,
           "kernel": "k2_segmented",
           "bytes_per_launch": round(line_bytes), "lines_per_stream": round(lines, 2),
           "note": "algorithmic bytes = the winners' distinct 128-B lines (the fetch granule of a random 8-B "
                   "load) + the k-key output rows + offsets; traffic = HBM bytes per launch from PMC "
                   "(profiles/r05: 128 B x TCC_EA0_RDREQ + WRITE_SIZE)"}
    return {"config": "C3 segmented 2^20 x 4096, k=64", "elements": n, "seconds": t,
            "Gelem_s": n / t / 1e9,
            "roofline": hbm,
            "roofline_valu": R.valu_roofline(l0, l1, t, "k2_segmented",
                                             note="launch time = median of 5 (HIP events); VALU: the Philox draws "
                                                  "alone (hidden under the line gather: see roofline)"),
            "gather_floor": {"seconds": t_g, "frac": t_g / t,
                             "what": "torch.gather of 64 random positions per 4096-key row (2^26 random "
                                     "8-B loads, ~57 distinct 128-B lines per row): the memory work K2 "
                                     "cannot avoid; frac = floor / K2 launch"},
            "winner_gather_bytes": S * k * 8}


def _pmc_traffic(name):
    """HBM bytes per launch of a kernel from the committed PMC summary (profiles/r05, else r04), or None."""
    for r in ("r05", "r04"):
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", r, "pmc_summary.json")))
            v = d.get(name, {}).get("hbm_bytes_per_launch")
            if v:
                return v
        except (OSError, ValueError):
            pass
    return None


def c3_large_k(dev):
    """K2 past the LDS winner table: k = 8192 (per-wave tables in global memory, the GT form) beside
    k = 4096 (LDS tables) on the same 4096 streams x 2^17 keys; VALU model of the Philox draws each
    needs, and the winner gather's floor (k random 8-B loads per stream)."""
    from reservoir_amd import batch

    S, L = 4096, 1 << 17
    n = S * L
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 3)
    offs = torch.arange(0, n + 1, L, dtype=torch.int64, device=dev)
    out = []
    for k in (4096, 8192):
        t = timed(lambda: batch.sample_segmented(keys, offs, k, seed=1), reps=7)
        l0, l1 = R.k2_calls(S, L, k)
        g = torch.Generator(device=dev)
        g.manual_seed(k)
        idx = torch.randint(0, L, (S, k), device=dev, generator=g)
        rows = keys.view(S, L)
        t_g = timed(lambda: torch.gather(rows, 1, idx), reps=5)
        del idx
        out.append({"config": f"K2 {S} streams x {L} keys, k={k} ({'global' if k > 4416 else 'LDS'} winner tables)",
                    "elements": n, "seconds": t, "Gelem_s": n / t / 1e9,
                    "roofline": R.valu_roofline(l0, l1, t, "k2_segmented",
                                                note="launch time = median of 7 (HIP events); VALU: the Philox "
                                                     "draws alone"),
                    "gather_floor": {"seconds": t_g, "frac": t_g / t}})
    return out


def c4(dev, hash_kind="identity", order="auto", twins=False, seed=7):
    from reservoir_amd import Sampler, _native

    n, k = 500_000_000, 65536
    vals = c4_data(n, dev)
    if twins:
        vals = hash_twins(vals, 26)
    torch.cuda.synchronize()
    L = _native.load()
    times, kern = [], []

    def one():
        mk = Sampler.distinct(k, seed=seed, order=order)
        d = mk(hash=hash_kind) if hash_kind != "default" else mk()
        d.sample_all(vals)
        d.result()
        d.close()

    if not twins:
        ramp(one, 0.2)
    # reps 1..9 timed end to end with the filter timer off (its events add marker packets and host
    # calls to the batch); one more rep with it on, for the filter launches and their time
    for rep in range(11):
        prof = rep == 10
        mk = Sampler.distinct(k, seed=seed, order=order)
        d = mk(hash=hash_kind) if hash_kind != "default" else mk()
        d.set_stream(torch.cuda.current_stream().cuda_stream)
        if prof:
            _native.check(L.rsv_profile_enable(d.handle, 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.sample_all(vals)
        r = d.result()
        t1 = time.perf_counter()
        if prof:
            ms, cnt = C.c_double(), C.c_int64()
            _native.check(L.rsv_profile_read(d.handle, C.byref(ms), C.byref(cnt)))
            kern.append((ms.value / 1e3, cnt.value))
        elif rep:
            times.append(t1 - t0)
        assert r.size == k
        d.close()
    t = sorted(times)[len(times) // 2]
    kt, passes = kern[0]
    ordered = order == "ordered" or (order == "auto" and hash_kind == "default")
    read = n * 8 if ordered else n * 8 * passes  # ordered: one chunked pass; set: every pass reads all
    name = "hash twins (~5 distinct keys per Long.hashCode: the boundary bucket is oversubscribed, the host " \
           "replay of the logged candidates runs)" if twins else "30% dup"
    return {"config": f"C4 (one GPU's share) distinct 5e8 keys {name}, k=65536, hash={hash_kind}, order={order}",
            "elements": n, "seconds_end_to_end": t, "Gelem_s": n / t / 1e9,
            "filter_launches": passes, "filter_seconds_total": kt,
            "filter_achieved_GBs": read / kt / 1e9, "hbm_frac_filter": read / kt / 1e9 / HBM}


def c4_wide(dev, mode="set"):
    """C4's share (5e8 keys, 30 % duplicates, k = 65536) as 16-byte UUIDs: mode "set" (precomputed
    64-bit hash tensor, set mode), "uuid" (default UUID.hashCode, ordered), "twins" (UUID hash twins,
    ordered: the host replay).  Filter bytes per element: 8 (hashes) or 16 (rows)."""
    import workloads as W

    from reservoir_amd import Sampler, _native

    n, k = 500_000_000, 65536
    vals = c4_data(n, dev)
    rows = W.uuid_rows(vals, 26 if mode == "twins" else None)
    hs = W.smix(vals ^ 0x5A5A) if mode == "set" else None
    del vals
    torch.cuda.synchronize()
    L = _native.load()
    times, kern = [], []

    def make():
        if mode == "set":
            return Sampler.distinct(k, key_type="bytes16", seed=7, order="set")(hash=lambda b: 0)
        return Sampler.distinct(k, key_type="bytes16", seed=7)()

    def feed(d):
        if hs is not None:
            d.sample_all(rows, hashes=hs)
        else:
            d.sample_all(rows)

    for rep in range(7 if mode != "twins" else 4):
        prof = rep == (6 if mode != "twins" else 3)
        d = make()
        d.set_stream(torch.cuda.current_stream().cuda_stream)
        if prof:
            _native.check(L.rsv_profile_enable(d.handle, 1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        feed(d)
        r = d.result()
        t1 = time.perf_counter()
        if prof:
            ms, cnt = C.c_double(), C.c_int64()
            _native.check(L.rsv_profile_read(d.handle, C.byref(ms), C.byref(cnt)))
            kern.append((ms.value / 1e3, cnt.value))
        elif rep:
            times.append(t1 - t0)
        assert r.shape == (k, 16)
        d.close()
    t = sorted(times)[len(times) // 2]
    kt, passes = kern[0]
    per = 8 if mode == "set" else 16
    read = n * per  # the filter chunks cover all but the first ~4k + 4096 elements
    del rows, hs
    torch.cuda.empty_cache()
    what = {"set": "precomputed 64-bit hash, set mode (filter reads the 8-B hashes)",
            "uuid": "default UUID.hashCode, ordered mode (filter reads the 16-B rows)",
            "twins": "UUID hash twins (~5 keys per hashCode), ordered: the host replay runs"}[mode]
    return {"config": f"C4 (one GPU's share) distinct 5e8 16-byte UUID keys 30% dup, k=65536, {what}",
            "elements": n, "seconds_end_to_end": t, "Gelem_s": n / t / 1e9,
            "filter_launches": passes, "filter_seconds_total": kt, "filter_bytes_per_element": per,
            "filter_achieved_GBs": read / kt / 1e9, "hbm_frac_filter": read / kt / 1e9 / HBM}


def c4_replay(dev):
    """C4's share with hash twins: the ordered mode's host-replay branch, as its own line."""
    return c4(dev, "default", twins=True, seed=11)


def c2l(dev):
    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys, 0x5EED0000)
    torch.cuda.synchronize()
    ts = []
    for rep in range(4):
        s = Sampler(k, engine="java_l", seed=0)()
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.sample_all(keys)
        s.result()
        ts.append(time.perf_counter() - t0)
        s.close()
    t = sorted(ts[1:])[1]
    return {"config": "C2 on engine java_l (reference Algorithm L, events replayed on GPU)",
            "elements": n, "seconds": t, "Gelem_s": n / t / 1e9}


def c2_host(dev):
    """C2 from a 1e9-key HOST buffer through rsv_sample_batch(RSV_MEM_HOST) (what the JVM bindings
    call with keys extracted into a host batch): the batch is sampled by index and only the <= k
    winners' keys leave host memory (round 6; before it every key crossed PCIe, ~0.5 s per 8 GB).
    Both engines; a step = create, sampleAll(host keys), result(), close; wall clock, median."""
    import numpy as np

    from reservoir_amd import Sampler, _native as N

    L = N.load()
    n, k = 1_000_000_000, 1024
    keys_d = torch.empty(n, dtype=torch.int64, device=dev)
    splitmix_fill(keys_d, 0x5EED0000)
    keys = keys_d.cpu().numpy()  # pageable host memory, as a JVM-side batch would be
    del keys_d
    torch.cuda.empty_cache()
    ptr = keys.ctypes.data_as(C.c_void_p)
    out = []
    for engine in ("philox_r", "java_l"):
        ts = []
        res = None
        for rep in range(14):
            s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A, engine=engine)()
            t0 = time.perf_counter()
            N.check(L.rsv_sample_batch(s.handle, ptr, n, N.MEM_HOST, None))
            res = s.result()
            ts.append(time.perf_counter() - t0)
            s.close()
        t = sorted(ts[4:])[len(ts[4:]) // 2]
        out.append({"config": f"C2 from a 1e9-key host buffer via rsv_sample_batch(RSV_MEM_HOST), engine={engine}: "
                              "winners-only (index-only batch + host gather of the <= k winning keys)",
                    "elements": n, "seconds": t, "Gelem_s": n / t / 1e9, "result_n": int(res.size),
                    "what": "wall clock of create + sampleAll + result() + close, median of 10 after 4 warm-up"})
    del keys
    return out


def c2_indexed(dev):
    """sampleAll over a 1e9-element IndexedSeq through the C ABI (the FFM/JNI bindings' override):
    K1 over the indices, k x 8 B of slot offsets back, the winners' keys forward -- no key buffer."""
    from reservoir_amd import Sampler

    n, k = 1_000_000_000, 1024
    seq = range(n)
    ts = []
    for rep in range(12):
        s = Sampler(k, seed=0xC0FFEE, stream_id=0x5A5A)()
        t0 = time.perf_counter()
        s.sample_all(seq)
        s.result()
        ts.append(time.perf_counter() - t0)
        s.close()
    t = sorted(ts[2:])[len(ts[2:]) // 2]
    return {"config": "C2 as sampleAll(IndexedSeq) through the ABI (rsv_sample_indexed + rsv_fill_slots): "
                      "1e9-element host sequence, no key buffer, map on the winners only",
            "elements": n, "seconds": t, "Gelem_s": n / t / 1e9}


def c4_merge(dev, parts=8, k=65536, per_shard=20_000_000):
    """The C4 combine's merge on one GPU: `parts` shard sets (k = 65536 each, from consecutive
    slices of C4-distributed keys) merged into a fresh sampler by distributed.merge_local -- the
    rows and the device merge of distributed.combine without the all-gather.  Time per merge
    (HIP events on the caller stream, and host wall clock including the result publication)."""
    from reservoir_amd import Sampler
    from reservoir_amd import distributed as D

    data = c4_data(parts * per_shard, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = []
    for hash_kind in ("identity", "default"):
        mk = Sampler.distinct(k, seed=7, retain_log=hash_kind == "default")
        make = (lambda: mk(hash="identity")) if hash_kind == "identity" else (lambda: mk())
        shards = []
        for r in range(parts):
            s = make()
            s.set_stream(stream)
            s.sample_all(data[r * per_shard:(r + 1) * per_shard])
            shards.append(s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        gpu, wall = [], []
        for rep in range(25):
            t = make()
            t.set_stream(stream)
            torch.cuda.synchronize()
            w0 = time.perf_counter()
            e0.record()
            D.merge_local(t, shards, total_count=parts * per_shard)
            e1.record()
            t.result()
            wall.append(time.perf_counter() - w0)
            e1.synchronize()
            gpu.append(e0.elapsed_time(e1) / 1e3)
            t.close()
        gpu, wall = sorted(gpu[5:]), sorted(wall[5:])
        out.append({"config": f"C4 combine: {parts} shard sets of k={k} merged (merge_local = {parts} x "
                              f"export_packed + device merge_packed), hash={hash_kind}",
                    "rows": parts, "k": k, "merge_gpu_seconds": gpu[len(gpu) // 2],
                    "merge_wall_seconds_incl_result": wall[len(wall) // 2]})
        for s in shards:
            s.close()
    del data
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c3,c4,c2l")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    todo = args.only.split(",")
    if "c3" in todo:
        print(json.dumps(c3(dev)), flush=True)
        torch.cuda.empty_cache()
    if "c4" in todo:
        print(json.dumps(c4(dev, "identity")), flush=True)
        print(json.dumps(c4(dev, "default", "set")), flush=True)
        print(json.dumps(c4(dev, "default")), flush=True)  # auto -> ordered (exact ties)
        torch.cuda.empty_cache()
    if "c4o" in todo:  # default hash, auto -> ordered only (for traces)
        print(json.dumps(c4(dev, "default")), flush=True)
    if "c4r" in todo:  # the ordered replay branch
        print(json.dumps(c4_replay(dev)), flush=True)
    if "c4i" in todo:  # identity hash only (for traces)
        print(json.dumps(c4(dev, "identity")), flush=True)
    if "c2l" in todo:
        print(json.dumps(c2l(dev)), flush=True)
    if "c2i" in todo:
        print(json.dumps(c2_indexed(dev)), flush=True)
    if "c2h" in todo:
        for r in c2_host(dev):
            print(json.dumps(r), flush=True)
    if "c3k" in todo:
        for r in c3_large_k(dev):
            print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()
    if "c4w" in todo:
        for mode in ("set", "uuid", "twins"):
            print(json.dumps(c4_wide(dev, mode)), flush=True)
            torch.cuda.empty_cache()
    if "c4ws" in todo:  # UUID keys, set mode only (for traces)
        print(json.dumps(c4_wide(dev, "set")), flush=True)
    if "c4wu" in todo:  # UUID keys, UUID.hashCode ordered mode only (for traces)
        print(json.dumps(c4_wide(dev, "uuid")), flush=True)
    if "c4m" in todo:
        for r in c4_merge(dev):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
