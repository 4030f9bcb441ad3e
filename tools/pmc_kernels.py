"""Median per-dispatch rocprofv3 counters per kernel (dev helper): summarise a --pmc run's
counter_collection.csv into a small JSON (the CSV itself is large).

    python3 tools/pmc_kernels.py <dir-with-counter_collection.csv> <out.json> [name-substring ...]"""
import collections
import csv
import json
import os
import statistics
import sys


def main(src, out, keep):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in os.listdir(src):
        if not f.endswith("counter_collection.csv"):
            continue
        for r in csv.DictReader(open(os.path.join(src, f))):
            n = r["Kernel_Name"]
            short = n.split("(anonymous namespace)::", 1)[-1].split("(")[0]
            if keep and not any(k in short for k in keep):
                continue
            per[(short, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(list)
    for (short, _), d in per.items():
        agg[short].append(d)
    res = {}
    for short, lst in agg.items():
        keys = sorted(set().union(*lst))
        med = {k: statistics.median(x[k] for x in lst if k in x) for k in keys}
        w = med.get("SQ_WAVES") or 1
        med["dispatches"] = len(lst)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if k in med:
                med[k + "_per_wave"] = round(med[k] / w, 1)
        res[short] = med
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
