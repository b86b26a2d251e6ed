"""Timeline of the last config-3 shard steps in a rocprofv3 kernel trace (rocpd
SQLite .db): every dispatch from `before` dispatches ahead of the last key-cache
launch on, with start / end relative to the trace start, duration, queue and
stream -- how the two pipeline streams' launches and the side streams'
digests interleave.
Usage: python tools/trace_segment.py <run_results.db> [before=40]"""
import sqlite3
import sys


def main(db, before=40):
    c = sqlite3.connect(db)
    rows = c.execute("select name, queue_id, stream_id, start, end, grid_x from kernels order by start").fetchall()
    t0 = rows[0][3]
    short = lambda n: n.split("(")[0].replace("void ", "").replace("nt::", "")[:48]
    last = max(i for i, r in enumerate(rows) if "keyset" in r[0])
    print("%10s %10s %9s  %-4s %-4s %8s  %s" % ("start_us", "end_us", "dur_us", "q", "s", "grid", "kernel"))
    for n, q, st, s, e, g in rows[max(0, last - before):last + 4]:
        print("%10.1f %10.1f %9.1f  q%-3d s%-3d %8d  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, st, g,
                                                            short(n)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
