"""Static instruction counts of a kernel's loop blocks (device assembly from hipcc -S).

usage: python scripts/isa_loop.py [KERNEL_REGEX] [--hist] [-D MACRO ...]
Default kernel: the fp32 trace-mode single-site expansion (expand_kernel<float, OUT_TRACE3, false>).
Prints VGPR count and, per backward-branch loop, VALU / SALU / memory instruction counts.
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


def main():
    args = sys.argv[1:]
    hist = "--hist" in args
    defines = [args[i + 1] for i, a in enumerate(args) if a == "-D"]
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
