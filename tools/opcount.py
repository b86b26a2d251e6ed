#!/usr/bin/env python3
"""Count field multiplies per operation in the exact device code (host build,
tests/cpp/nt_host_harness.cpp) and write profiles/opcount.json -- the
algorithmic numerator of bench.py's roofline.

A fe_mul is 100 partial products and a fe_sq 55, each ONE v_mad_u64_u32
(32x32->64 multiply-accumulate) on gfx950; "mads" = 100 mul + 55 sq.
SHA-512 (k = H(R||A||M)) is not included in the mad count; its compression
count is reported separately.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _hostarith as H  # noqa: E402


def _per_verify(fn):
    """field ops per signature of the two-per-lane kernel path (pair count / 2)"""
    H.counts_reset()
    assert fn() == (True, True)
    mul, sq = H.counts()
    return mul / 2, sq / 2


def measure():
    seed = bytes(range(32))
    msg = bytes(512)
    pk, sig = H.sign(seed, msg)
    pk2, sig2 = H.sign(bytes(range(1, 33)), msg)
    out = {}
    for mode, name in ((0, "verify_strict"), (1, "verify_cofactorless")):
        mul, sq = _per_verify(lambda: H.verify_pair(mode, pk, sig, msg, pk2, sig2, msg))
        out[name + "_fe_mul"] = mul
        out[name + "_fe_sq"] = sq
        out[name + "_mads"] = 100 * mul + 55 * sq
        mul, sq = _per_verify(lambda: H.verify_pair(mode, pk, sig, msg, pk2, sig2, msg, cached=True))
        out[name + "_keyset_fe_mul"] = mul
        out[name + "_keyset_fe_sq"] = sq
        out[name + "_keyset_mads"] = 100 * mul + 55 * sq
    H.counts_reset()
    H.sign(seed, msg)
    mul, sq = H.counts()
    out["sign_fe_mul"], out["sign_fe_sq"], out["sign_mads"] = mul, sq, 100 * mul + 55 * sq
    out["verify_sha512_blocks_512B_msg"] = (64 + 512 + 17 + 127) // 128
    out["note"] = ("host-compiled device code, two signatures per lane as the kernels run them "
                   "(per-signature = pair / 2); fe_mul = 100 v_mad_u64_u32, fe_sq = 55; "
                   "table builds (wide combs) excluded")
    return out


if __name__ == "__main__":
    d = measure()
    path = os.path.join(ROOT, "profiles", "opcount.json")
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))
