"""Per-phase kernel durations from a rocprofv3 kernel trace (development aid).

  python3 tools/trace_phases.py <kernel_trace.csv> <kernel-name-substring> [marker-substring]

Phases are split at kernels whose name contains the marker substring (default: "fill").
"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
name, marker = sys.argv[2], (sys.argv[3] if len(sys.argv) > 3 else "fill")
phase, cur = [], []
for r in rows:
    if marker in r["Kernel_Name"]:
        phase.append(cur)
        cur = []
    elif name in r["Kernel_Name"]:
        cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
phase.append(cur)
for i, p in enumerate(phase):
    if p:
        print(f"phase {i}: n={len(p)} median={statistics.median(p):.2f} us min={min(p):.2f} max={max(p):.2f}")
