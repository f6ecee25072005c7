"""Static instruction census of the MPPI rollout step (the hot loop of mppi_plan_kernel).

Compiles csrc/mppi.hip for gfx950 with -DMPJ_COUNT_HOT_PATH (the wave-uniform slow paths
of the branch-free libm compiled out, so the loop body is the hot straight-line path) and
counts the instructions of the largest loop of the kernel by class.

  python tools/isa_count.py [--kernel mppi_plan_kernel] [--extra -DFOO]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op):
    if re.match(r"v_(add|sub)_f64|v_add_f64", op):
        return "f64 add"
    if op.startswith("v_mul_f64"):
        return "f64 mul"
    if op.startswith(("v_fma_f64", "v_fmac_f64")):
        return "f64 fma"
    if op.startswith(("v_div_", "v_rcp_f64", "v_rsq_f64", "v_sqrt_f64")):
        return "f64 div/rcp/sqrt"
    if op.startswith("v_cndmask"):
        return "v_cndmask"
    if op.startswith(("v_mov", "v_accvgpr")):
        return "v_mov"
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "v_read/writelane"
    if op.startswith("v_cmp"):
        return "v_cmp"
    if op.startswith(("v_ldexp", "v_frexp", "v_rndne", "v_trunc", "v_floor", "v_fract", "v_cvt")):
        return "f64 misc"
    if op.startswith("v_"):
        return "other VALU"
    if op.startswith(("ds_",)):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "s_waitcnt/nop"
    if op.startswith("s_"):
        return "SALU/branch"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="mppi_plan_kernel")
    ap.add_argument("--src", default=os.path.join(ROOT, "motionplanning_amd", "csrc", "mppi.hip"))
    ap.add_argument("--extra", action="append", default=[])
    ap.add_argument("--top", type=int, default=0)
    ap.add_argument("--inst", default="ILi512E", help="substring selecting the template instance")
    ap.add_argument("--funcs", action="store_true", help="group the loop's VALU instructions by enclosing "
                                                          "source function (-g)")
    ap.add_argument("--lines", type=int, default=0, help="attribute the loop's VALU instructions to source lines "
                                                         "(-g .loc directives) and print the top N")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "--cuda-device-only", "-S", "-DMPJ_COUNT_HOT_PATH", *(["-g"] if (a.lines or a.funcs) else []), "-I" + os.path.join(ROOT, "include"),
                        *a.extra, "-o", asm, a.src], check=True, capture_output=True)
        lines = open(asm).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))
    # kernels: every symbol containing the name; take the one with the biggest body
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + a.kernel + r"\S*:", l) and a.inst in l]
    best = None
    for s0 in starts:
        e0 = next(i for i in range(s0, len(lines)) if lines[i].startswith(".Lfunc_end"))
        body = lines[s0:e0]
        heads = [i for i, l in enumerate(body) if "Loop Header: Depth=1" in l and l.startswith(".LBB")]
        for h in heads:
            lab = body[h].split(":")[0]  # .LBBk_n
            tag = lab[2:]  # BBk_n as in the "in Loop: Header=BBk_n" / "Parent Loop BBk_n" block notes
            # every basic block of the loop nest: the header and each block the assembler notes as in it
            ins, locs, inside, loc = [], [], False, None
            for l in body:
                if l.startswith(".LBB") or l.startswith("; %bb."):
                    inside = l.startswith(lab + ":") or ("Header=" + tag + " ") in l or ("Parent Loop " + tag + " ") in l
                    continue
                t = l.strip()
                if t.startswith(".loc"):
                    f = t.split()
                    loc = (files.get(f[1], f[1]), int(f[2]))
                    continue
                if inside and t and not t.startswith((";", ".")):
                    ins.append(t.split()[0])
                    locs.append(loc)
            if best is None or len(ins) > len(best[1]):
                best = (lines[s0].split(":")[0], ins, locs)
    name, ins, locs = best
    c = collections.Counter(classify(op) for op in ins)
    valu = sum(v for k, v in c.items() if k.startswith(("f64", "v_", "other VALU")))
    nbr = sum(1 for op in ins if op.startswith("s_cbranch"))
    print(f"{name[:60]}: largest loop body {len(ins)} instructions, VALU {valu}, conditional branches {nbr}")
    for k, v in c.most_common():
        print(f"  {k:20s} {v:6d}")
    if a.funcs:
        srcs = {}

        def func_of(lc):
            if not lc or not lc[0]:
                return "?"
            if lc[0] not in srcs:
                txt = None
                for d in (os.path.join(ROOT, "include"), os.path.join(ROOT, "motionplanning_amd", "csrc")):
                    fp = os.path.join(d, lc[0])
                    if os.path.exists(fp):
                        txt = open(fp).read().split("\n")
                srcs[lc[0]] = txt
            txt = srcs[lc[0]]
            if txt is None:
                return lc[0]
            for i in range(min(lc[1] - 1, len(txt) - 1), -1, -1):
                m = re.search(r"(?:MPJ_FN|__device__)[^(]*?\b(\w+)\s*\(", txt[i])
                if m:
                    return f"{lc[0]}:{m.group(1)}"
            return lc[0]
        byf = collections.Counter()
        for op, lc in zip(ins, locs):
            if classify(op).startswith(("f64", "v_", "other VALU")):
                byf[func_of(lc)] += 1
        for f, v in byf.most_common():
            print(f"    {v:5d}  {f}")
    if a.lines:
        byline = collections.Counter()
        for op, lc in zip(ins, locs):
            if classify(op).startswith(("f64", "v_", "other VALU")):
                byline[lc] += 1
        for lc, v in byline.most_common(a.lines):
            src = ""
            if lc and lc[0]:
                for d in (os.path.join(ROOT, "include"), os.path.join(ROOT, "motionplanning_amd", "csrc")):
                    fp = os.path.join(d, lc[0])
                    if os.path.exists(fp):
                        src = open(fp).read().split("\n")[lc[1] - 1].strip()[:90]
            print(f"    {v:5d}  {lc[0] if lc else '?'}:{lc[1] if lc else 0}  {src}")
    if a.top:
        for op, v in collections.Counter(ins).most_common(a.top):
            print(f"    {op:28s} {v}")


if __name__ == "__main__":
    main()
