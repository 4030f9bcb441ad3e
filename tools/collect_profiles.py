"""Summarise a scripts/gpu_r02_prof.sh run (gpurun_out/<dir>) into profiles/<round>/.

  python3 tools/collect_profiles.py gpurun_out/r02h profiles/r02

Copies the rocprofv3 kernel-stats CSVs and writes, per profiled kernel, the per-launch PMC figures:
  SQ_INSTS_VALU          wave-instructions (all XCDs)
  duration x 2.4 GHz     GPU cycles at the peak clock (GRBM_GUI_ACTIVE / 8 reads high on < 0.3 ms
                         dispatches, MI355X_MICROARCH.md: kept as a diagnostic only)
  FETCH_SIZE, WRITE_SIZE KiB; on gfx950 FETCH_SIZE reads half the bytes of a coalesced read and
                         WRITE_SIZE reads them exactly (MI355X_MICROARCH.md HBM section)
                         -> hbm_bytes_per_launch = FETCH_SIZE x 2 KiB + WRITE_SIZE KiB (other access
                         widths, e.g. K2's 8-B gathers, are uncalibrated: an estimate)
and the VALU cycles/instruction those imply (cycles x 1024 SIMDs / SQ_INSTS_VALU).
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import statistics
import sys

# C2 runs K1 unfused (rsv_runtime.hip); "gather" = tools/micro_gather's plain winner-key gather (the
# C3 memory floor); "c4" = the ordered-distinct scheduled pass (kernel stats only)
KERNELS = {"k1": "k1_last_writer", "c3": "k2_segmented", "gather": "gather<0>", "c4": "sched_filter"}


def pmc(dirpath: str, kernel: str) -> dict:
    """Median per-dispatch counter values for dispatches whose kernel name contains `kernel`."""
    if not os.path.isdir(dirpath):
        return {}
    per = collections.defaultdict(dict)
    durs = {}
    for f in os.listdir(dirpath):
        p = os.path.join(dirpath, f)
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(p)):
                if kernel in r["Kernel_Name"]:
                    d = per[r["Dispatch_Id"]]
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        elif f.endswith("kernel_trace.csv"):
            for r in csv.DictReader(open(p)):
                if kernel in r["Kernel_Name"]:
                    durs[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    if per:
        names = set().union(*per.values())
        for c in sorted(names):
            out[c] = statistics.median(v[c] for v in per.values() if c in v)
        out["dispatches"] = len(per)
    if durs:
        out["dur_us_median"] = statistics.median(durs.values()) * 1e6
    return out


def in_kernel_clock(*dirs: str):
    """The median in-kernel clock over the K1 launches of a k1_in_kernel_clock.jsonl, or None."""
    for p in (os.path.join(d, f) for d in dirs for f in ("k1_clock.log", "k1_in_kernel_clock.jsonl")):
        if not os.path.exists(p):
            continue
        rows = [json.loads(line) for line in open(p) if '"k1_in_kernel_clock"' in line]
        if rows:
            return {"clock_GHz_median": round(statistics.median(r["clock_GHz_median"] for r in rows), 3), "file": p}
    return None


def main(src: str, dst: str) -> None:
    os.makedirs(dst, exist_ok=True)
    # merged into an existing summary (other runs' kernels, e.g. the C3 line-request pass, stay)
    out_path = os.path.join(dst, "pmc_summary.json")
    summary = json.load(open(out_path)) if os.path.exists(out_path) else {}
    summary["source_run"] = os.path.basename(src.rstrip("/"))
    for tag, kern in KERNELS.items():
        stats = os.path.join(src, tag, f"{tag}_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
        sq = pmc(os.path.join(src, f"{tag}_sq"), kern)
        fe = pmc(os.path.join(src, f"{tag}_fetch"), kern)
        wr = pmc(os.path.join(src, f"{tag}_write"), kern)
        if not (sq or fe or wr):
            continue
        d = {"kernel": kern, "sq_pass": sq, "fetch_pass": fe, "write_pass": wr,
             "pmc_source_run": summary["source_run"]}
        if "SQ_INSTS_VALU" in sq and "dur_us_median" in sq:
            # GPU cycles per launch = the launch's duration x 2.4 GHz, the peak shader clock (so an
            # upper bound on the cycles the launch had: no clock above the peak is implied).
            # GRBM_GUI_ACTIVE / 8 / duration is kept only as a diagnostic: MI355X_MICROARCH.md ("DVFS
            # give-back") notes that quotient reads high on dispatches shorter than ~0.3 ms (K1's 84 us
            # launch read 2.53 GHz).  The in-kernel clock (s_memtime / s_memrealtime, tools/micro_k1o
            # c) is reported beside it when a run of it is at hand.
            cyc = sq["dur_us_median"] * 1e-6 * 2.4e9
            d["valu_instrs_per_launch"] = sq["SQ_INSTS_VALU"]
            d["gpu_cycles_per_launch"] = round(cyc, 1)
            d["clock_GHz"] = 2.4
            d["clock_source"] = "peak shader clock x launch duration (upper bound on cycles)"
            d["cycles_per_valu_instr_per_simd"] = round(cyc * 1024 / sq["SQ_INSTS_VALU"], 3)
            clk = in_kernel_clock(src, dst)
            if clk:
                d["in_kernel_clock_GHz_median"] = clk["clock_GHz_median"]
                d["in_kernel_clock_file"] = clk["file"]
            if "GRBM_GUI_ACTIVE" in sq:
                d["grbm_quotient_GHz_diagnostic"] = round(sq["GRBM_GUI_ACTIVE"] / 8 / (sq["dur_us_median"] * 1e-6) / 1e9, 3)
        if "FETCH_SIZE" in fe and "WRITE_SIZE" in wr:
            d["hbm_bytes_per_launch"] = int((2 * fe["FETCH_SIZE"] + wr["WRITE_SIZE"]) * 1024)
            d["hbm_bytes_rule"] = "(2 x FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE correction)"
        summary[tag] = {**summary.get(tag, {}), **d}
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        for line in open(bench):
            if line.startswith("{") and '"metric"' in line:
                summary["bench_line"] = json.loads(line)
                with open(os.path.join(dst, "bench.json"), "w") as f:
                    f.write(line)
    k1 = summary.get("k1", {})
    if "hbm_bytes_per_launch" in k1:
        n = summary.get("bench_line", {}).get("config", {}).get("keys_per_gpu")
        with open(os.path.join(dst, "pmc_k1.json"), "w") as f:
            json.dump({"n": n, "hbm_bytes_per_launch": k1["hbm_bytes_per_launch"], "kernel": k1["kernel"],
                       "source_run": summary["source_run"]}, f, indent=1)
    with open(out_path, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({t: {k: v for k, v in d.items() if not k.endswith("_pass")} for t, d in summary.items()
                      if isinstance(d, dict) and t != "bench_line"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
