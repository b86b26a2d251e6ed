"""The config-3 8-GPU shard steps in a rocprofv3 --kernel-trace CSV
(run_kernel_trace.csv of `bench.py ... --sigs 65536` with NT_BENCH_HOST_CERTS=0,
so the run's last key-cache launches are the 8-GPU shard's): the last K
key-cache launches' mean duration, start-to-start interval and overlap with the
previous launch; the mean duration of every other kernel dispatched between
them (a short kernel that waits behind the other stream's key-cache launch shows
as a long duration here); and the timeline of the last `show` launches.
Usage: python tools/shard_steps.py <run_kernel_trace.csv> [K=20] [show=6]"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.replace("void ", "").split("(")[0].replace("nt::", "")[:48]


def main(path, k=20, show=6):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"],
                     r["Stream_Id"], int(r["Grid_Size_X"])))
    rows.sort()
    ks = [i for i, r in enumerate(rows) if "keyset" in r[2]]
    sel = ks[-k:]
    durs = [(rows[i][1] - rows[i][0]) / 1e3 for i in sel]
    s2s = [(rows[b][0] - rows[a][0]) / 1e3 for a, b in zip(sel, sel[1:])]
    ovl = [max(0, min(rows[a][1], rows[b][1]) - rows[b][0]) / 1e3 for a, b in zip(sel, sel[1:])]
    print("last %d key-cache launches: duration avg %.1f us, start-to-start avg %.1f us, overlap with the previous "
          "launch avg %.1f us" % (len(sel), sum(durs) / len(durs), sum(s2s) / len(s2s), sum(ovl) / len(ovl)))
    lo, hi = rows[sel[0]][0], rows[sel[-1]][1]
    aux = defaultdict(list)
    for s, e, n, q, st, g in rows:
        if lo <= s <= hi and "keyset" not in n:
            aux[short(n)].append((e - s) / 1e3)
    print("other kernels dispatched among them (count, mean / max duration us):")
    for n, v in sorted(aux.items(), key=lambda x: -sum(x[1])):
        print("  %-48s %4d  %8.1f  %8.1f" % (n, len(v), sum(v) / len(v), max(v)))
    t0 = rows[sel[-1]][0]
    first = sel[-show] if len(sel) >= show else sel[0]
    start = rows[first][0] - 400_000  # the aux kernels ahead of that launch
    print("%10s %10s %9s  %-4s %-4s %8s  %s" % ("start_us", "end_us", "dur_us", "q", "s", "grid", "kernel"))
    for s, e, n, q, st, g in rows:
        if start <= s <= rows[sel[-1]][1]:
            print("%10.1f %10.1f %9.1f  q%-3s s%-3s %8d  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, q, st, g,
                                                                short(n)))


if __name__ == "__main__":
    a = sys.argv
    main(a[1], int(a[2]) if len(a) > 2 else 20, int(a[3]) if len(a) > 3 else 6)
