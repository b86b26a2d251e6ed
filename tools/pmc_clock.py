"""Clock / traffic experiment of VERDICT r03 item 2: per variant
(base = the product build; xatab / xcomb = timing-only builds whose [j]A/[j]R
table lookups / comb lines are forced to one cached entry, so HBM traffic drops
while the instruction stream stays the same) and per key-cache / verify launch:
duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration of the pass that
counted it), VALU issue share, HBM bytes (FETCH_SIZE x 2 per the gfx950
correction + WRITE_SIZE) and, for base, the dynamic VALU classes.
Usage: python tools/pmc_clock.py profiles/r04/pmc_clock"""
import collections
import csv
import glob
import os
import sys


def load(vdir):
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(lambda: collections.defaultdict(set))
    dur = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(vdir, "pass*_run_counter_collection.csv"))):
        p = os.path.basename(f).split("_")[0]
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], int(r["Grid_Size"]))
            # a counter collected in two passes (SQ_INSTS_VALU in pass 1 and 4) counts once: pass 1
            if r["Counter_Name"] == "SQ_INSTS_VALU" and p != "pass1":
                continue
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[k][(p, r["Counter_Name"])].add(r["Dispatch_Id"])
    for f in sorted(glob.glob(os.path.join(vdir, "pass*_run_kernel_trace.csv"))):
        p = os.path.basename(f).split("_")[0]
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"], int(r["Grid_Size_X"]))
            dur[k][p].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, c in cnt.items():
        per = {}
        for name, v in c.items():
            n = max(len(s) for (p, nm), s in nd[k].items() if nm == name)
            per[name] = v / n
        d1 = dur[k].get("pass1") or [0]
        out[k] = (per, sum(d1) / len(d1))
    return out


def main(root):
    print(__doc__.split("Usage")[0].strip())
    print()
    for v in ("base", "xatab", "xcomb"):
        res = load(os.path.join(root, v))
        for (name, grid), (c, ns) in sorted(res.items()):
            if "ed25519_verify" not in name:
                continue
            s = "%-6s %-50s grid %7d  %8.1f us" % (v, name.replace("nt::", ""), grid, ns / 1e3)
            if "GRBM_GUI_ACTIVE" in c and ns:
                s += "  clock %.3f GHz" % (c["GRBM_GUI_ACTIVE"] / 8 / ns)
                if "SQ_INSTS_VALU" in c:
                    s += "  issue %.3f" % (c["SQ_INSTS_VALU"] * 4 / (1024 * c["GRBM_GUI_ACTIVE"] / 8))
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                s += "  HBM %.2f GB (read %.2f)" % ((c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024 / 1e9,
                                                  c["FETCH_SIZE"] * 2048 / 1e9)
            if "SQ_INSTS_VALU" in c:
                s += "  VALU %.4g" % c["SQ_INSTS_VALU"]
            for q in ("INT64", "INT32", "CVT", "FMA_F64", "ADD_F64", "MUL_F64", "TRANS_F64"):
                if "SQ_INSTS_VALU_" + q in c:
                    s += "  %s %.4g" % (q, c["SQ_INSTS_VALU_" + q])
            print(s)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r04/pmc_clock")
