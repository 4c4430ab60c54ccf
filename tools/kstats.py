#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 results database: calls, average/total time, launch gaps.

usage: python tools/kstats.py gpurun_out/<dir>/run_results.db
"""
import sqlite3
import statistics
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels "
                     "group by name order by 4 desc").fetchall()
    for name, n, avg_us, tot_ms in rows:
        print(f"{name[:70]:70s} {n:6d} {avg_us:10.1f} us {tot_ms:10.2f} ms")
    ks = c.execute("select start, end from kernels order by start").fetchall()
    gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
    if gaps:
        print(f"launches {len(ks)}  span {(ks[-1][1] - ks[0][0]) / 1e6:.2f} ms  "
              f"idle {sum(g for g in gaps if g > 0) / 1e6:.2f} ms  median gap {statistics.median(gaps) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
