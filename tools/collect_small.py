"""Copy the small rocprofv3 outputs (kernel stats and counter CSVs) from a scratch directory into
gpurun_out/ (the .db files and full traces stay behind: gpurun_out/ travels back only under 64 MiB).
    python3 tools/collect_small.py <src-dir> <dst-dir>"""
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
n = 0
for root, _, files in os.walk(src):
    for f in files:
        p = os.path.join(root, f)
        if f.endswith(".csv") and ("stats" in f or "counter_collection" in f) and os.path.getsize(p) < 20 << 20:
            rel = os.path.relpath(root, src).replace(os.sep, "_")
            shutil.copy(p, os.path.join(dst, f"{rel}_{f}"))
            n += 1
print(f"copied {n} files")
