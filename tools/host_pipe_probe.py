"""The host entry point's copy/kernel pipeline on config 2 (VERDICT r04 item
6): nt_ed25519_verify_strict on 1M 512-B verifies from nt_host_alloc (pinned)
buffers, timed per call; run it under `rocprofv3 --kernel-trace
--memory-copy-trace` to see the chunk timeline.  Prints one JSON line.

    python tools/host_pipe_probe.py [--sigs 1000000] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sigs", type=int, default=1_000_000)
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
    pk_p, sig_p, msg_p = be.pinned(pk.shape), be.pinned(sig.shape), be.pinned(data.shape)
    pk_p[...] = pk
    sig_p[...] = sig
    msg_p[...] = data
    out = {"n": n}
    for name, args in (("pinned", (pk_p, sig_p, msg_p)), ("pageable", (pk, sig, data))):
        be.verify_strict(args[0], args[1], args[2], off, ln)
        ts = []
        for _ in range(a.reps):
            print("[probe] %s call" % name, file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            r = be.verify_strict(args[0], args[1], args[2], off, ln)
            ts.append(time.perf_counter() - t0)
        assert r.all()
        t = float(np.median(ts))
        out[name] = {"ms": round(t * 1e3, 3), "per_s": round(n / t, 1), "all_ms": [round(x * 1e3, 2) for x in ts]}
    print(json.dumps(out), flush=True)
    be.close()


if __name__ == "__main__":
    main()
