"""Dynamic ISA class breakdown of ONE config-2 verification.

Static instruction classes of every loop of k_ed25519_verify<strict, 2 waves,
24-bit comb of B> (tools/isa/isa_classes.py loop tree of `hipcc -g
--save-temps` assembly), each weighted by its trip count per verify:

  loop (source)                           trip count per verify
  per-verify body (k_verify.inc verify_n)  1 (straight-line: scalars, decompression outside the
                                           exponentiation loops, table starts, ladder top window,
                                           comb start, final test; one SHA-512 compression)
  grid-stride body                         1/2 (two signatures per lane per iteration)
  fe_sqn loops (fe_pow22523, 2 x 9)        sum(n - 1) over n in {2,5,10,20,10,50,100,50,2} = 240 per
                                           decompression, x 2 (A and R)
  ptab_build doubling loop (2 tables)      3 each
  ladder window loop                       W - 1 = 32 (W = 33: the wave maximum of the lanes' window
                                           counts for |u|, v < 2^128.5 -- DESIGN.md 5.1)
  ladder doubling loop                     3 per window = 96
  comb of B loop                           11 (24-bit digits)
  SHA-512 full / tail block loops          3 / 1 (576 B = 64-B prefix + 512-B message: 5 blocks), plus
                                           4 more compressions of 3,455 VALU (the compression the
                                           per-verify body holds once; the one-lane-per-message
                                           kernel's per-block count)
  lattice reduction: Lehmer batch loop     6, its inner Euclid loop 69, the one-step loop 3.6
                                           (sc_halfsize)

Usage: python tools/isa/verify_model.py <kernel .s with -g> [pmc VALU per verify]"""
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import isa_classes as I  # noqa: E402

CLASSES = ("mad64", "shift64", "add64", "mul32", "alu32", "mov", "fp64")
SHA_BLOCK = {"mad64": 0, "shift64": 0, "add64": 640, "mul32": 0, "alu32": 2640, "mov": 175, "fp64": 0}  # 3,455


def main():
    path = sys.argv[1]
    pmc = float(sys.argv[2]) if len(sys.argv) > 2 else None
    loops = I.loop_tree(open(path).read(), "ILi0ELi2ELi24")

    def src_of(d, prefix):
        return sum(v for k, v in d["src"].items() if k.startswith(prefix))

    rows = []   # (label, weight, classes)
    sqn = [h for h, d in loops.items() if sum(d["c"].values()) and d["c"]["mad64"] == 56 and d["depth"] == 3]
    for h, d in loops.items():
        c = d["c"]
        valu = sum(c[k] for k in CLASSES)
        if h == "-":
            continue
        if d["depth"] == 1:
            rows.append(("grid-stride loop body", 0.5, c, h))
        elif d["depth"] == 2:
            rows.append(("per-verify straight-line body (incl. one SHA-512 compression)", 1.0, c, h))
        elif h in sqn:
            rows.append(("fe_sqn squaring loops (%d loops)" % len(sqn), 480.0 / len(sqn), c, h))
        elif src_of(d, "sha512.hpp") and valu < 100:
            rows.append(("SHA-512 full-block load loop", 3.0, c, h))
        elif src_of(d, "sha512.hpp"):
            rows.append(("SHA-512 tail-block loop", 1.0, c, h))
        elif src_of(d, "sc25519.hpp") and d["depth"] == 4:
            rows.append(("lattice: Lehmer inner Euclid steps", 69.0, c, h))
        elif src_of(d, "sc25519.hpp") and c["mad64"] > 40:
            rows.append(("lattice: Lehmer batch", 6.0, c, h))
        elif src_of(d, "sc25519.hpp"):
            rows.append(("lattice: one-step Euclid", 3.6, c, h))
        elif d["depth"] == 4:
            rows.append(("ladder: doubling (ge_dbl_p2)", 96.0, c, h))
        elif 3000 < valu < 4500:
            rows.append(("ladder: window (3M + dbl + 2 cached additions)", 32.0, c, h))
        elif 2000 < valu < 3000:
            rows.append(("ptab_build doubling loop (2 tables)", 3.0, c, h))
        elif 1000 < valu < 1500:
            rows.append(("comb of B: mixed addition", 11.0, c, h))
        else:
            rows.append(("other loop %s" % h, 1.0, c, h))
    rows.append(("SHA-512: 4 further compressions", 4.0, Counter(SHA_BLOCK), "-"))
    # aggregate rows that share a label
    agg = {}
    for label, w, c, h in rows:
        a = agg.setdefault(label, Counter())
        for k in CLASSES:
            a[k] += w * c[k]
    total = Counter()
    for a in agg.values():
        total.update(a)
    tv = sum(total[k] for k in CLASSES)
    out = ["Dynamic VALU instructions per config-2 verification (k_ed25519_verify<strict, 2, 24>, 512-B messages)",
           "by region and class: static ISA counts of each loop x its trip count per verify (tools/isa/verify_model.py)",
           "", "%-66s %8s %7s %7s %7s %6s %7s %5s %5s" % ("region", "VALU", "share", "mad64", "carry64", "mul32",
                                                         "alu32", "mov", "fp")]
    for label, a in sorted(agg.items(), key=lambda kv: -sum(kv[1][k] for k in CLASSES)):
        v = sum(a[k] for k in CLASSES)
        out.append("%-66s %8.0f %6.1f%% %7.0f %7.0f %6.0f %7.0f %5.0f %5.0f"
                   % (label, v, 100 * v / tv, a["mad64"], a["shift64"] + a["add64"], a["mul32"], a["alu32"],
                      a["mov"], a["fp64"]))
    out.append("%-66s %8.0f %6.1f%% %7.0f %7.0f %6.0f %7.0f %5.0f %5.0f"
               % ("TOTAL (model)", tv, 100.0, total["mad64"], total["shift64"] + total["add64"], total["mul32"],
                  total["alu32"], total["mov"], total["fp64"]))
    if pmc:
        out.append("%-66s %8.0f  (model / measured = %.3f)" % ("measured: PMC SQ_INSTS_VALU x 64 / verifies", pmc,
                                                                  tv / pmc))
    print("\n".join(out))


if __name__ == "__main__":
    main()
