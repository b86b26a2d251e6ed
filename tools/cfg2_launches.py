"""The config-2 verify launches of a `rocprofv3 --kernel-trace --stats` run of
the driver's bench command (rocpd SQLite database) against the bench line's own
per-launch time (roofline.kernel_ms, HIP events around each one-stream launch):
the first launches of k_ed25519_verify at the config-2 grid are the one-stream
region's warm-up + timed launches, in order.
Usage: python tools/cfg2_launches.py <run_results.db> <bench log (JSON line)> [warmup=5] [steps=20]"""
import json
import sqlite3
import sys
from collections import Counter


def main(db, log, warm=5, steps=20):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, start, end from kernels where name like '%k_ed25519_verify<%' "
                     "order by start").fetchall()
    # config 2's 1M launches: the grid with the longest launches among those launched at least warm + steps times
    cnt, tot = Counter(), Counter()
    for n, g, s, e in rows:
        cnt[g] += 1
        tot[g] += e - s
    grid = max((g for g in cnt if cnt[g] >= warm + steps), key=lambda g: tot[g] / cnt[g])
    ms = [(e - s) / 1e6 for n, g, s, e in rows if g == grid]
    d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
    kname = d["roofline"].get("kernel", "k_ed25519_verify")
    timed = ms[warm:warm + steps]
    mean = sum(timed) / len(timed)
    print("config-2 verify launches (%s, grid %d) under rocprofv3 --kernel-trace --stats:" % (kname, grid))
    print("launches in order (ms): " + " ".join("%.3f" % x for x in ms[:50]))
    print("the %d timed one-stream launches (after %d warm-up): mean %.3f ms, min %.3f, max %.3f"
          % (len(timed), warm, mean, min(timed), max(timed)))
    km = d["roofline"]["kernel_ms"]
    print("bench line of the same run: roofline.kernel_ms %.3f (HIP events around each one-stream launch on its stream)"
          % km)
    print("agreement: %+.2f %%" % (100.0 * (mean - km) / km))


if __name__ == "__main__":
    a = sys.argv
    main(a[1], a[2], int(a[3]) if len(a) > 3 else 5, int(a[4]) if len(a) > 4 else 20)
