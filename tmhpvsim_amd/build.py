"""In-tree build of libtmhpvsim.so for gfx950 (hipcc, no JIT cache)."""
from __future__ import annotations

import os
import re
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "tmh_engine.hip")]
DEPS = SRC + [os.path.join(HERE, "csrc", "tmh_math.h"), os.path.join(HERE, "csrc", "tmh_model.h"),
        os.path.join(ROOT, "include", "tmhpvsim.h")]
LIB = os.path.join(HERE, "libtmhpvsim.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def hipcc():
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


# -ffp-contract=off: no silent FMA contraction, so fp64 state arithmetic rounds
# exactly like the reference's numpy/Python scalar operations.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off"]


def _code_only(text):
    """C / C++ source without comments and blank-line / trailing-space differences: what
    the compiler sees (a comment-only edit does not change the stamp)."""
    out, i, n = [], 0, len(text)
    pat = re.compile(r'//[^\n]*|/\*.*?\*/|"(?:\\.|[^"\\])*"|\'(?:\\.|[^\'\\])*\'', re.S)
    for m in pat.finditer(text):
        out.append(text[i:m.start()])
        tok = m.group(0)
        out.append(tok if tok[0] in "\"'" else " ")
        i = m.end()
    out.append(text[i:])
    lines = (ln.rstrip() for ln in "".join(out).splitlines())
    return "\n".join(ln for ln in lines if ln)


def build_stamp():
    """Hash of the library's sources (code only, comments stripped) and compile flags:
    measurement records taken with another build (profiles/pmc_kernels.json) are
    recognised as stale."""
    import hashlib
    h = hashlib.sha256(" ".join([ARCH] + FLAGS).encode())
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        h.update(_code_only(open(d, encoding="utf-8", errors="replace").read()).encode())
    return h.hexdigest()[:16]


def lib_stamp(path=LIB):
    """The build stamp compiled into a built library (tmh_build_stamp's string, read from
    the file's bytes without loading it), or None for an unstamped or missing library."""
    if not os.path.exists(path):
        return None
    m = re.search(rb"TMHSTAMP:([0-9a-f]{16})", open(path, "rb").read())
    return m.group(1).decode() if m else None


def build_lib(force=False, verbose=False):
    """Compile libtmhpvsim.so unless the in-tree library already carries the stamp of
    the current sources (a library built from other sources -- an older pushed binary,
    an A/B build copied over it -- is rebuilt, whatever its mtime)."""
    stamp = build_stamp()
    if not force and lib_stamp() == stamp:
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}"] + FLAGS + [f'-DTMH_BUILD_STAMP="TMHSTAMP:{stamp}"',
                                                          "-I", os.path.join(ROOT, "include"), "-o", LIB + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_lib(force=True, verbose=True))
