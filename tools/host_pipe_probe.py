"""The host entry points' copy/kernel pipeline: config 2
= nt_ed25519_verify_strict on 1M 512-B verifies, config 3 (--cfg3) =
nt_ed25519_verify_batch_groups_keyset on 100k certificates x 67 votes of a
100-key committee, from nt_host_alloc (pinned) and pageable buffers, timed per
call; run it under `rocprofv3 --kernel-trace --memory-copy-trace` or with
NT_PIPE_TRACE=1 to see the chunk timeline.  Prints one JSON line.

    python tools/host_pipe_probe.py [--sigs 1000000] [--reps 5] [--cfg3]
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
    ap.add_argument("--cfg3", action="store_true")
    a = ap.parse_args()
    if a.cfg3:
        return cfg3(a)
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


def cfg3(a, C=100_000, V=67, nk=100):
    import ntcrypto
    be = ntcrypto.Backend(devices=[0])
    rng = np.random.default_rng(4)
    kseeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    msg32 = rng.integers(0, 256, (C, 32), dtype=np.uint8)
    kidx = np.stack([rng.choice(nk, V, replace=False) for _ in range(C)]).astype(np.uint32).ravel()
    gmsg = np.repeat(msg32, V, axis=0).ravel()
    _, gsig = be.sign_batch(kseeds[kidx], gmsg, np.arange(C * V, dtype=np.uint64) * 32, np.full(C * V, 32, np.uint64))
    ks = be.keyset(be.sign_batch(kseeds))
    first = np.arange(C, dtype=np.uint64) * V
    cnt = np.full(C, V, np.uint32)
    key_p, sig_p = be.pinned((C * V,), np.uint32), be.pinned((C * V, 64))
    key_p[...] = kidx
    sig_p[...] = gsig
    out = {"certificates": C, "votes": V, "comb_bits": ks.info()[0]}
    for name, args in (("pinned", (key_p, sig_p)), ("pageable", (kidx, gsig))):
        ks.verify_batch_groups(args[0], args[1], first, cnt, msg32)
        ts = []
        for _ in range(a.reps):
            print("[probe] %s call" % name, file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            r = ks.verify_batch_groups(args[0], args[1], first, cnt, msg32)
            ts.append(time.perf_counter() - t0)
        assert r.all()
        t = float(np.median(ts))
        out[name] = {"ms": round(t * 1e3, 3), "certs_per_s": round(C / t, 1), "all_ms": [round(x * 1e3, 2) for x in ts]}
    print(json.dumps(out), flush=True)
    ks.close()
    be.close()


if __name__ == "__main__":
    main()
