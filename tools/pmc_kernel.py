"""Per-dispatch counter values of one kernel in a rocprofv3 --pmc CSV
(run_counter_collection.csv): every dispatch whose name holds `substr`, with
its grid size, duration and each counter (summed over the rows rocprofv3 writes
per dispatch), largest grids first.
Usage: python tools/pmc_kernel.py <run_counter_collection.csv> <substr> [max_rows=6]"""
import csv
import sys
from collections import defaultdict


def main(path, sub, rows=6):
    disp = {}
    vals = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        disp[d] = (int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for v in vals.values() for c in v})
    print("%10s %10s  %s" % ("grid", "dur_us", "  ".join("%22s" % n for n in names)))
    for d in sorted(disp, key=lambda d: -disp[d][0])[:rows]:
        g, t = disp[d]
        print("%10d %10.1f  %s" % (g, t, "  ".join("%22.4g" % vals[d][n] for n in names)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 6)
