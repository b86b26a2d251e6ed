"""PCIe-inclusive throughput of the host entry points (caller buffers in host
memory): cfg2 verify_strict, cfg3-shaped verify_batch_groups through the key
cache, and SHA-512 over cfg2's messages.  Prints one JSON line.

    python tools/host_api_bench.py [--sigs 1000000] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sigs", type=int, default=1_000_000)
    ap.add_argument("--certs", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import ntcrypto
    be = ntcrypto.Backend(devices=[0])
    rng = np.random.default_rng(3)
    n, L = a.sigs, 512
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    data = rng.integers(0, 256, n * L, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, np.uint64)
    pk, sig = be.sign_batch(seeds, data, off, ln)
    out = {}
    t, r = timed(lambda: be.verify_strict(pk, sig, data, off, ln), a.reps)
    assert r.all()
    out["verify_strict"] = {"n": n, "ms": round(t * 1e3, 2), "per_s": round(n / t, 1)}
    t, _ = timed(lambda: be.sha512_trunc32(data, off, ln), a.reps)
    out["sha512_512B"] = {"n": n, "ms": round(t * 1e3, 2), "GB_per_s": round(n * L / t / 1e9, 2)}
    # cfg3 shape: 100 keys, 67 votes per certificate over one 32-B digest each
    C, V = a.certs, 67
    kseeds = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    msg32 = rng.integers(0, 256, (C, 32), dtype=np.uint8)
    kidx = np.stack([rng.choice(100, V, replace=False) for _ in range(C)]).astype(np.uint32).ravel()
    gseeds = kseeds[kidx]
    gmsg = np.repeat(msg32, V, axis=0).ravel()
    goff = np.arange(C * V, dtype=np.uint64) * 32
    gln = np.full(C * V, 32, np.uint64)
    gpk, gsig = be.sign_batch(gseeds, gmsg, goff, gln)
    kpk = be.sign_batch(kseeds)
    ks = be.keyset(kpk)
    first = np.arange(C, dtype=np.uint64) * V
    cnt = np.full(C, V, np.uint32)
    t, r = timed(lambda: ks.verify_batch_groups(kidx, gsig, first, cnt, msg32), a.reps)
    assert r.all()
    out["batch_groups_keyset"] = {"groups": C, "sigs": C * V, "ms": round(t * 1e3, 2),
                                  "certs_per_s": round(C / t, 1), "sigs_per_s": round(C * V / t, 1)}
    ks.close()
    be.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
