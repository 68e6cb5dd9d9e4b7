"""Static instruction counts of a kernel's loop blocks (device assembly from hipcc -S).

usage: python scripts/isa_loop.py [KERNEL_REGEX] [--hist] [-D MACRO ...]
       python scripts/isa_loop.py --groups [KERNEL_REGEX] [-D MACRO ...]
Default kernel: the fp32 trace-mode single-site expansion (expand_kernel<float, OUT_TRACE3, false>).
Prints VGPR count and, per backward-branch loop, VALU / SALU / memory instruction counts.

--groups: an analysis build (-DTMH_ISA_MARKS) whose comment markers delimit the expansion's
four-second group bodies (the meter's Philox block, the noise's, four daylight seconds, four
night seconds); prints, per marked region of the fault-free loop, the opcodes by class with
their issue cycles (profiles/r03_isa_rate.txt weights) and the totals per second.  Out-of-line
rare paths (the noise quantile's far tails) sit outside the markers; both sides of DISC's
divergent kt split are inside (a wave with chains on both sides runs both).
"""
from __future__ import annotations

import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def asm(defines=()):
    out = "/tmp/isa_engine.s"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", out,
           os.path.join(ROOT, "tmhpvsim_amd", "csrc", "tmh_engine.hip")] + [f"-D{d}" for d in defines]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read().split("\n")


# issue cycles per wave64 instruction per SIMD (profiles/r03_isa_rate.txt, every SIMD full,
# operands in distinct registers), by opcode prefix; the rest of the VALU at the compare /
# select rate
W_FAST = ("v_fma_f32", "v_fmac_f32", "v_fmaak_f32", "v_fmamk_f32", "v_mul_f32", "v_add_f32", "v_sub_f32",
          "v_subrev_f32", "v_mov_b32", "v_bitop3_b32", "v_xor_b32", "v_and_b32", "v_or_b32", "v_lshrrev_b32",
          "v_lshlrev_b32", "v_ashrrev_i32", "v_add_u32", "v_sub_u32", "v_lshl_add_u32", "v_lshl_or_b32",
          "v_and_or_b32", "v_add3_u32", "v_bfe_u32", "v_bfi_b32", "v_not_b32")
W_TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32")


def weight(op):
    op = re.sub(r"_e(32|64)$", "", op)
    if op in W_TRANS:
        return 8.4
    if op in ("v_rcp_f64", "v_sqrt_f64", "v_rsq_f64"):
        return 16.2
    if op in W_FAST:
        return 2.3
    return 4.2


def groups(kre, defines=()):
    lines = asm(["TMH_ISA_MARKS", *defines])
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kre + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    marks = [(i, m.group(1), m.group(2)) for i, l in enumerate(body) if (m := re.search(r"TMH_MARK (\w+) (begin|end)", l))]
    seen = collections.Counter()
    per = {"meter": 4, "noise": 4, "day4": 4, "night4": 4}
    for (i, name, kind), (j, name2, kind2) in zip(marks, marks[1:]):
        if kind != "begin" or kind2 != "end" or name2 != name:
            continue
        seen[name] += 1
        ins = [l.split()[0] for l in body[i:j] if l.startswith("\t") and not l.strip().startswith(";")
               and not l.strip().startswith(".")]
        v = [x for x in ins if x.startswith("v_")]
        cyc = sum(weight(x) for x in v)
        sal = sum(1 for x in ins if x.startswith("s_") and x != "s_nop")
        nan = sum(1 for l in body[i:j] if "v_cndmask" in l and "0x7fc00000" in l) + \
            sum(1 for l in body[i:j] if re.search(r"v_cmp_(lt|ge)_i32", l))
        tag = f"{name}#{seen[name]}" + (" (fault-free loop)" if not nan else " (general loop: NaN selects)")
        print(f"{tag:34s}\n        VALU {len(v):4d} ({len(v) / per[name]:6.1f}/s)  cycles {cyc:7.1f} ({cyc / per[name]:6.1f}/s)  "
              f"SALU {sal:4d} ({sal / per[name]:5.1f}/s)  mem {sum(1 for x in ins if x[:2] not in ('v_', 's_'))}")
        hist = collections.Counter(re.sub(r"_e(32|64)$", "", x) for x in v)
        print("         " + "  ".join(f"{k}:{n}" for k, n in hist.most_common(24)))
        shist = collections.Counter(x for x in ins if x.startswith("s_") and x != "s_nop")
        if shist:
            print("   SALU  " + "  ".join(f"{k}:{n}" for k, n in shist.most_common(12)))


def main():
    args = sys.argv[1:]
    defines = [args[i + 1] for i, a in enumerate(args) if a == "-D"]
    if "--groups" in args:
        pos = [a for i, a in enumerate(args) if not a.startswith("-") and (i == 0 or args[i - 1] != "-D")]
        groups(pos[0] if pos else r"expand_kernelIfLi1ELb0E", defines)
        return
    hist = "--hist" in args
    pos = [a for i, a in enumerate(args) if not a.startswith("-") and (i == 0 or args[i - 1] != "-D")]
    kre = pos[0] if pos else r"expand_kernelIfLi1ELb0E"
    lines = asm(defines)
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kre + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    name = lines[start].split(":")[0]
    body = lines[start:end]
    vg = [l for l in lines if f"{name}.num_vgpr," in l]
    print(name[:80], vg[0].split(",")[-1].strip() if vg else "?", "VGPRs")
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and labels.get(m.group(1), 1 << 30) < i:
            loops.append((labels[m.group(1)], i))
    for a, b in sorted(set(loops)):
        ins = [l.split()[0] for l in body[a:b + 1] if l.startswith("\t") and not l.strip().startswith(";")
               and not l.strip().startswith(".")]
        c = collections.Counter("valu" if x.startswith("v_") else "salu" if x.startswith("s_") else "mem"
                                for x in ins)
        print(f"loop {a}-{b}: {len(ins)} instr  VALU {c['valu']}  SALU {c['salu']}  mem {c['mem']}")
        if hist and b - a > 200:
            for k, v in collections.Counter(re.sub(r"_e(32|64)$", "", x) for x in ins).most_common(40):
                print(f"   {v:4d} {k}")


if __name__ == "__main__":
    main()
