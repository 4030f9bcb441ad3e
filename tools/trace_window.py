"""Timeline of the engine's own dispatches from a rocprofv3 kernel_trace.csv (dev helper): the last
`reps` windows that start with a kernel matching `first` -- each dispatch's start offset from the
window start, duration and the idle gap before it, so host round trips show as gaps.

  python3 tools/trace_window.py <kernel_trace.csv> <first-kernel-substring> [reps] > out.txt
"""
import csv
import sys


def main(path: str, first: str, reps: int = 2) -> None:
    rows = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "rsv::" in n or "rocprim" in n or "rocclr" in n:
            short = n.split("(anonymous namespace)::")[-1].split("(")[0]
            if "rocprim" in n:
                short = "rocprim:" + ("radix" if "radix" in n else "merge" if "merge" in n else "scan" if "scan" in n
                                      else "other")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    sel = starts[-reps:]
    for w, i0 in enumerate(sel):
        i1 = starts[starts.index(i0) + 1] if starts.index(i0) + 1 < len(starts) else len(rows)
        t0 = rows[i0][0]
        prev_end = t0
        print(f"# window {w}")
        for s, e, name in rows[i0:i1]:
            print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f}  {name}")
            prev_end = max(prev_end, e)
        print(f"# window end {(prev_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
