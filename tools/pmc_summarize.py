#!/usr/bin/env python3
"""Summarize tools/pmc_collect.sh output into a per-launch JSON for profiles/.

Per (kernel, grid size): counters summed over its dispatches and divided by
the dispatch count (per launch).  HBM traffic per launch = FETCH_SIZE*1024*2 (gfx950 reports
half the bytes of wide 16-B/lane streaming reads; MI355X_MICROARCH.md §HBM) +
WRITE_SIZE*1024; the uncorrected read figure is kept beside it.
VALU issue share = SQ_INSTS_VALU * 4 cycles / (SIMDs * GRBM_GUI_ACTIVE/8).
Effective clock (MI355X_MICROARCH.md, "DVFS give-back") = GRBM_GUI_ACTIVE / 8
(rocprofv3 sums the 8 XCDs) / the same dispatches' average duration from the
kernel trace of the pass that collected GRBM_GUI_ACTIVE.
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {"k_ed25519_verify_keyset": "verify_keyset", "k_ed25519_verify<": "verify", "k_sha512": "sha512",
           "k_ed25519_sign": "sign", "k_group_and": "group_and", "k_clock_probe": "clock_probe"}


def kname(k):
    for pat, name in KERNELS.items():
        if pat in k:
            return name
    return None


def _derive(c, nd):
    per = {k: v / nd for k, v in c.items()}
    d = {"dispatches_per_pass": nd, "per_launch": per}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        d["hbm_bytes_per_launch"] = per["FETCH_SIZE"] * 1024 * 2 + per["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch_uncorrected"] = (per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
    if "SQ_INSTS_VALU" in per and "GRBM_GUI_ACTIVE" in per:
        cyc = per["GRBM_GUI_ACTIVE"] / 8
        d["valu_issue_share_4cyc"] = per["SQ_INSTS_VALU"] * 4 / (1024 * cyc)
    return d


def main(indir, out, tag):
    """Counters per (kernel, grid size): one bench command launches a kernel for
    several workloads (e.g. the verify kernel for config 2's 1M signatures and in
    chunks for the host entry points).  "kernels" reports each kernel's
    LARGEST-grid launches (the config's resident-data launch); "by_grid" all."""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in sorted(glob.glob(os.path.join(indir, "pass*", "*counter_collection.csv"))):
        pdir = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            n = kname(r["Kernel_Name"])
            if not n:
                continue
            key = (n, int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[key][pdir].add(r["Dispatch_Id"])
    # per (kernel, grid): average dispatch duration (ns) in each pass's kernel trace
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(indir, "pass*", "*kernel_trace.csv"))):
        pdir = os.path.basename(os.path.dirname(f))
        acc_d = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            n = kname(r.get("Kernel_Name", ""))
            if not n:
                continue
            try:
                g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                acc_d[(n, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            except (KeyError, ValueError):
                continue
        for key, v in acc_d.items():
            dur[key][pdir] = sum(v) / len(v)
    # the pass that holds GRBM_GUI_ACTIVE, per (kernel, grid)
    grbm_pass = {}
    for f in sorted(glob.glob(os.path.join(indir, "pass*", "*counter_collection.csv"))):
        pdir = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            n = kname(r["Kernel_Name"])
            if n and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                grbm_pass[(n, int(r["Grid_Size"]))] = pdir
    res = {"tag": tag, "source": indir, "kernels": {}, "by_grid": {}}
    for (n, g), c in sorted(acc.items()):
        nd = max(len(v) for v in disp[(n, g)].values())
        d = _derive(c, nd)
        d["grid"] = g
        pp = grbm_pass.get((n, g))
        if pp and pp in dur.get((n, g), {}) and "GRBM_GUI_ACTIVE" in d["per_launch"]:
            ns = dur[(n, g)][pp]
            d["duration_ns_grbm_pass"] = ns
            d["effective_clock_ghz"] = d["per_launch"]["GRBM_GUI_ACTIVE"] / 8 / ns
        res["by_grid"]["%s@%d" % (n, g)] = d
        if n not in res["kernels"] or g > res["kernels"][n]["grid"]:
            res["kernels"][n] = d
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["kernels"], indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
