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


NPAIRS = 32  # the half-size ladder's window count depends on the signature: average it
KEY_BITS = 21  # the committee key combs the key cache builds when they fit (kKeyCombReduced)


def _per_verify(fn):
    """field ops per signature of the two-per-lane kernel path, averaged over
    NPAIRS deterministic signature pairs (each lane's own window count, i.e. the
    algorithmic work; the wave-uniform maximum the GPU runs is ~1 window more)"""
    H.counts_reset()
    for i in range(NPAIRS):
        assert fn(i) == (True, True)
    mul, sq = H.counts()
    return mul / (2 * NPAIRS), sq / (2 * NPAIRS)


def measure():
    msg = bytes(512)
    sigs = [H.sign(bytes([(7 * i + j) & 255 for j in range(32)]), msg) for i in range(2 * NPAIRS)]
    out = {}
    for mode, name in ((0, "verify_strict"), (1, "verify_cofactorless")):
        mul, sq = _per_verify(lambda i: H.verify_pair(mode, sigs[2 * i][0], sigs[2 * i][1], msg,
                                                      sigs[2 * i + 1][0], sigs[2 * i + 1][1], msg))
        out[name + "_fe_mul"] = mul
        out[name + "_fe_sq"] = sq
        out[name + "_mads"] = round(100 * mul + 55 * sq, 1)
        # key-cache kernel: 8 signatures per lane (keyset_per_lane()), one inversion
        H.counts_reset()
        for i in range(NPAIRS // 4):
            q = [(sigs[8 * i + k][0], sigs[8 * i + k][1], msg) for k in range(8)]
            assert H.verify_cached_n(mode, q, bits=KEY_BITS) == (True,) * 8
        mul, sq = H.counts()
        mul, sq = mul / (2 * NPAIRS), sq / (2 * NPAIRS)
        out[name + "_keyset_fe_mul"] = mul
        out[name + "_keyset_fe_sq"] = sq
        out[name + "_keyset_mads"] = round(100 * mul + 55 * sq, 1)
    seed = bytes(range(32))
    H.counts_reset()
    H.sign(seed, msg)
    mul, sq = H.counts()
    out["sign_fe_mul"], out["sign_fe_sq"], out["sign_mads"] = mul, sq, 100 * mul + 55 * sq
    out["verify_sha512_blocks_512B_msg"] = (64 + 512 + 17 + 127) // 128
    out["note"] = ("host-compiled device code as the kernels run it (verify: two signatures per lane, "
                   "averaged over %d pairs, per-signature = pair / 2; key cache: 8 per lane sharing one "
                   "variable-time binary-GCD inversion, whose <= 17 x 72 v_mad_i64_i32 + 1 fe_mul per batch are "
                   "not field multiplies and are not counted beyond that fe_mul); B comb %d bits, key combs %d bits; fe_mul = 100 v_mad_u64_u32, fe_sq = 55; "
                   "table builds (wide combs) excluded" % (NPAIRS, H.bcomb_bits(), KEY_BITS))
    return out


if __name__ == "__main__":
    d = measure()
    path = os.path.join(ROOT, "profiles", "opcount.json")
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))
