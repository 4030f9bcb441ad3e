"""One ordered-distinct sampleAll from a rocprofv3 kernel trace, as a timeline (profiles/r04/):

    python3 tools/timeline.py gpurun_out/<run>/c4/c4_kernel_trace.csv > profiles/r04/c4_ordered_timeline.txt

Picks the second-to-last scheduled pass (sched_filter) of the trace and lists the kernels from the
batch's first filter launch to the set publication: start (us, from the first kernel), duration,
gap to the previous kernel's end, name."""
import csv
import sys


def main(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sched_filter" in r["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit("no scheduled pass in the trace")
    i = idx[-2]
    j = i
    # the heap-filling chunk's filter: k3_filter, or hash_all when it has no bound (round 4)
    while j > 0 and "k3_filter" not in rows[j]["Kernel_Name"] and "hash_all" not in rows[j]["Kernel_Name"]:
        j -= 1
    end = i
    while end + 1 < len(rows) and "publish" not in rows[end]["Kernel_Name"]:
        end += 1
    j = max(0, j - 3)  # what precedes the batch's first filter (the previous batch's tail, fills)
    t0 = int(rows[j]["Start_Timestamp"])
    prev = None
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kernel")
    for r in rows[j:end + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(anonymous namespace)::", 1)[-1].split("(")[0]
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {gap:7.2f}  {name}")
        prev = e
    print(f"first kernel start -> last kernel end: {(prev - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
