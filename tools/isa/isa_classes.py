"""Instruction-class breakdown of gfx950 assembly (hipcc --save-temps .s).

  python tools/isa/isa_classes.py loops <file.s>      innermost loop bodies of every kernel, by class
  python tools/isa/isa_classes.py kernel <file.s> <substring>   the whole kernel (static), by class

Classes (what each costs on the SIMD: profiles/r01_alu_rate_v2.txt):
  mad64     v_mad_u64_u32 (32x32 -> 64 multiply-accumulate, 4.8 cyc)
  shift64   64-bit shifts (carry extraction)
  add64     v_lshl_add_u64 / v_add_co+addc pairs (carry propagation, 64-bit sums)
  mul32     32-bit multiplies (pre-scaling by 19 / 38)
  alu32     32-bit integer add/sub/logic/shift/select/bitop3/alignbit
  mov       register moves
  fp64      fp64 / conversions (the lattice reduction's quotients)
  vmem      global / buffer / scratch memory instructions
  lds       ds_* instructions
  salu      scalar ALU, branches, waits, nops (not VALU issue)
"""
import re
import sys
from collections import Counter

VALU = ("mad64", "shift64", "add64", "mul32", "alu32", "mov", "fp64", "valu_other")


def klass(op):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "mad64"
    if re.match(r"v_(lshrrev|lshlrev|ashrrev)_b64|v_lshr_b64|v_lshl_b64", op):
        return "shift64"
    if op.startswith("v_lshl_add_u64") or op.startswith("v_add_co_u32") or op.startswith("v_addc_co_u32") \
            or op.startswith("v_sub_co_u32") or op.startswith("v_subb_co_u32") or op.startswith("v_add_u64") \
            or op.startswith("v_subrev_co_u32") or op.startswith("v_subbrev_co_u32"):
        return "add64"
    if re.match(r"v_mul_(lo|hi)_u32|v_mul_u32_u24|v_mul_hi_u32_u24|v_mad_u32_u24|v_mul_i32_i24|v_mad_i32_i24", op):
        return "mul32"
    if op.startswith("v_mov_b32") or op.startswith("v_mov_b64") or op.startswith("v_pk_mov_b32") \
            or op.startswith("v_accvgpr") or op.startswith("v_readfirstlane") or op.startswith("v_readlane") \
            or op.startswith("v_writelane"):
        return "mov"
    if re.search(r"_f64|_f32|cvt", op):
        return "fp64"
    if op.startswith("v_"):
        return "alu32"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "salu"


def instructions(lines):
    for ln in lines:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        yield t.split()[0]


def kernels(text):
    """(name, [lines]) of every kernel in the file"""
    out = []
    for m in re.finditer(r"^(_Z\w+):\s*;\s*@", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        out.append((m.group(1), text[start:end].splitlines()))
    return out


def inner_loops(lines):
    """innermost loops: from a line annotated 'Inner Loop Header' back to the
    block label preceding it, until the branch back to that label"""
    res = []
    for i, ln in enumerate(lines):
        if "Inner Loop Header" not in ln:
            continue
        j = i
        while not re.match(r"^\.LBB\w+:", lines[j]):
            j -= 1
        label = lines[j].split(":")[0]
        k = i + 1
        while k < len(lines) and not re.search(r"s_cbranch_\w+\s+" + re.escape(label) + r"\b", lines[k]) \
                and not re.search(r"s_branch\s+" + re.escape(label) + r"\b", lines[k]):
            k += 1
        res.append((label, lines[j:k + 1]))
    return res


def table(c, title):
    v = sum(c[k] for k in VALU)
    rows = ["%s: %d VALU (%s)" % (title, v, ", ".join("%s %d" % (k, c[k]) for k in VALU if c[k]))]
    other = {k: c[k] for k in ("vmem", "lds", "salu") if c[k]}
    if other:
        rows.append("    non-VALU: " + ", ".join("%s %d" % kv for kv in other.items()))
    return "\n".join(rows)


def main():
    mode, path = sys.argv[1], sys.argv[2]
    text = open(path).read()
    for name, lines in kernels(text):
        if mode == "kernel":
            if sys.argv[3] not in name:
                continue
            c = Counter(klass(op) for op in instructions(lines))
            print(table(c, name))
            ops = Counter(op.split("_e32")[0].split("_e64")[0] for op in instructions(lines))
            print("    top opcodes: " + ", ".join("%s %d" % kv for kv in ops.most_common(25)))
        else:
            for label, body in inner_loops(lines):
                c = Counter(klass(op) for op in instructions(body))
                print(table(c, "%s loop %s" % (name[:48], label)))


if __name__ == "__main__" and sys.argv[1] != "tree":
    main()


# ---- loop tree (uses LLVM's loop comments; with -g, the .loc source lines) --
def loop_tree(text, kernel_sub):
    """Per loop of the kernel: depth, parent, exclusive instruction classes (the
    blocks whose innermost loop it is) and the source lines those came from."""
    files = {m.group(1): m.group(3) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', text, re.M)}
    for name, lines in kernels(text):
        if kernel_sub not in name:
            continue
        loops = {}           # header -> dict(depth, parent, classes, src)
        cur = None           # innermost loop header of the current block
        src = None
        block_hdr = []
        for ln in lines:
            t = ln.strip()
            m = re.match(r"^(\.LBB\w+|;\s*%bb\.\d+):?(.*)$", t)
            if m and (t.startswith(".LBB") or t.startswith("; %bb.")):
                label = m.group(1).replace(".LBB", "BB") if t.startswith(".LBB") else None
                block_hdr = [t]
                cur = None
                info = t
                if "Loop Header" in t and label:
                    cur = label
                mm = re.search(r"in Loop: Header=(BB\w+) Depth=(\d+)", t)
                if mm:
                    cur = mm.group(1)
                pm = re.findall(r"Parent Loop (BB\w+) Depth=(\d+)", t)
                if label and label not in loops and ("Loop Header" in t):
                    loops[label] = {"depth": 1, "parent": None, "c": Counter(), "src": Counter()}
                continue
            if t.startswith(";") and block_hdr:
                # continuation comment lines of the block label
                if "Loop Header" in t:
                    lab = block_hdr[0].split(":")[0].replace(".LBB", "BB")
                    dm = re.search(r"Depth=(\d+)", t)
                    par = [p for p in re.findall(r"Parent Loop (BB\w+) Depth=(\d+)", " ".join(block_hdr))]
                    loops[lab] = {"depth": int(dm.group(1)) if dm else 1,
                                  "parent": max(par, key=lambda x: int(x[1]))[0] if par else None,
                                  "c": Counter(), "src": Counter()}
                    cur = lab
                mm = re.search(r"in Loop: Header=(BB\w+) Depth=(\d+)", t)
                if mm:
                    cur = mm.group(1)
                block_hdr.append(t)
                continue
            if t.startswith(".loc"):
                f = t.split()
                src = "%s:%s" % (files.get(f[1], f[1]), f[2])
                continue
            if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
                continue
            block_hdr = []
            op = t.split()[0]
            key = cur or "-"
            if key not in loops:
                loops[key] = {"depth": 0 if key == "-" else 1, "parent": None, "c": Counter(), "src": Counter()}
            loops[key]["c"][klass(op)] += 1
            if src:
                loops[key]["src"][src] += 1
        return loops
    return {}


def print_tree(loops):
    for h, d in sorted(loops.items(), key=lambda kv: (kv[0] != "-", kv[0])):
        c = d["c"]
        v = sum(c[k] for k in VALU)
        top = ", ".join("%s %d" % kv for kv in d["src"].most_common(4))
        print("%-9s depth %d parent %-8s VALU %6d (mad64 %d, 64-bit carry %d, mul32 %d, alu32 %d, mov %d, fp %d) vmem %d | %s"
              % (h, d["depth"], d["parent"], v, c["mad64"], c["shift64"] + c["add64"], c["mul32"], c["alu32"],
                 c["mov"], c["fp64"], c["vmem"], top))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "tree":
    print_tree(loop_tree(open(sys.argv[2]).read(), sys.argv[3]))
