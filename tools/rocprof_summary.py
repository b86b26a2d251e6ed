#!/usr/bin/env python3
"""Per-kernel dispatch statistics from a rocprofv3 --kernel-trace --stats run
(the rocpd SQLite database rocprofv3 writes by default), grouped by kernel AND
grid size, so that launches of one kernel for different workloads in the same
bench command (e.g. k_ed25519_verify<strict> for config 2's 1M signatures and
for config 3's 100k header signatures) are reported separately.  Also copies
the tool's own whole-kernel summary (top_kernels).

Usage: python tools/rocprof_summary.py <run_results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, grid_x, workgroup_x, vgpr_count, scratch_size, count(*), avg(duration), min(duration),"
        " max(duration), sum(duration) from kernels group by name, grid_x, workgroup_x order by sum(duration) desc")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "GridX", "WorkgroupX", "VGPR", "ScratchBytes", "Calls", "AverageNs", "MinNs", "MaxNs",
                    "TotalNs"])
        for r in rows:
            w.writerow([r[0][:160]] + list(r[1:]))
        w.writerow([])
        w.writerow(["# rocprofv3 top_kernels (all grids merged)"])
        w.writerow(["Name", "Calls", "TotalDuration", "Average", "Percentage"])
        for r in c.execute("select * from top_kernels"):
            w.writerow([r[0][:160]] + list(r[1:]))
    print(open(out).read()[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
