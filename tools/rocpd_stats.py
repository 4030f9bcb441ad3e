"""Kernel statistics from a rocprofv3 rocpd database (its default output on this image): one CSV row
per kernel -- name, calls, total / average / min / max duration (us), share -- like --stats' csv.

  python tools/rocpd_stats.py gpurun_out/<run>/prof/<name>_results.db [> profiles/rNN/<name>.csv]
"""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
    for name, n, tot, avg, lo, hi in rows:
        w.writerow([name, n, round(tot / 1e3, 3), round(avg / 1e3, 3), round(lo / 1e3, 3), round(hi / 1e3, 3),
                    round(100.0 * tot / total, 2)])


if __name__ == "__main__":
    main(sys.argv[1])
