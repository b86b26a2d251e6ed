"""Timeline of a rocprofv3 kernel trace (rocpd SQLite .db): per dispatch the
queue, start / end relative to the first dispatch, and for the key-cache
launches how much of each one overlaps the previous key-cache launch.
Usage: python tools/trace_overlap.py <run_results.db> [name-substring ...]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    rows = c.execute("select name, queue_id, stream_id, start, end, grid_x from kernels order by start").fetchall()
    t0 = rows[0][3]
    short = lambda n: n.split("(")[0].replace("void ", "").replace("nt::", "")[:48]
    prev = None
    for name, q, st, s, e, gx in rows:
        if "keyset" in name:
            ov = 0.0
            if prev is not None:
                ov = max(0, min(e, prev[1]) - max(s, prev[0])) / 1e3
            gap = (s - prev[1]) / 1e3 if prev is not None else 0.0
            print("%10.1f %8.1f us q%d s%d grid %7d %-48s overlap-prev %7.1f us  start-after-prev-end %8.1f us"
                  % ((s - t0) / 1e3, (e - s) / 1e3, q, st, gx, short(name), ov, gap))
            prev = (s, e)
        elif len(sys.argv) > 2 and any(k in name for k in sys.argv[2:]):
            print("%10.1f %8.1f us q%d s%d grid %7d %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, st, gx, short(name)))


if __name__ == "__main__":
    main()
