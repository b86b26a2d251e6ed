"""Config-3 rows of an ab_env.sh run: per log the key-cache certificates/s and,
per shard size, its certificates/s and ratio to the 1-GPU rate.
Usage: python tools/ab_summary.py <dir with v*_r*.log>"""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/v*_r*.log")):
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])["certificates"]
    sh = {k: (round(v["certs_per_s"] / 1e6, 3), v["per_gpu_vs_1gpu"]) for k, v in d.get("shard_of", {}).items() if isinstance(v, dict)}
    print(f.split("/")[-1], round(d["keyset"]["certs_per_s"] / 1e6, 3), sh)
