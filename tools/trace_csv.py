"""Timeline of a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): per
dispatch the queue, stream, start relative to the first dispatch, duration,
scratch and grid; filtered by name substrings.  With --keyset: the key-cache
launches only, with their gap to the previous one and their overlap with it.
Usage: python tools/trace_csv.py <run_kernel_trace.csv> [--keyset] [substr ...]"""
import csv
import sys


def short(n):
    n = n.replace("void ", "")
    return n.split("(")[0].replace("nt::", "")[:60]


def main():
    path = sys.argv[1]
    ks = "--keyset" in sys.argv
    subs = [a for a in sys.argv[2:] if not a.startswith("--")]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    prev = None
    for r in rows:
        name = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if ks:
            if "keyset" not in name:
                continue
            ov = max(0, min(e, prev[1]) - max(s, prev[0])) / 1e3 if prev else 0.0
            gap = (s - prev[1]) / 1e3 if prev else 0.0
            print("%12.1f %9.1f us q%-3s s%-3s scr %4s grid %8s %-40s ovl %8.1f gap %8.1f"
                  % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Stream_Id"], r["Scratch_Size"], r["Grid_Size_X"],
                     short(name), ov, gap))
            prev = (s, e)
        elif not subs or any(k in name for k in subs):
            print("%12.1f %9.1f us q%-3s s%-3s scr %4s grid %8s %s"
                  % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Stream_Id"], r["Scratch_Size"], r["Grid_Size_X"],
                     short(name)))


if __name__ == "__main__":
    main()
