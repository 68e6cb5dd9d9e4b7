#!/bin/bash
# Build the library of a git revision for a same-box A/B: build_rev.sh REV NAME -> tmhpvsim_amd/libtmh_NAME.so
set -eu
cd "$(dirname "$0")/.."
rev=$1 name=$2
d=$(mktemp -d)
mkdir -p "$d/include" "$d/csrc"
git show "$rev:include/tmhpvsim.h" > "$d/include/tmhpvsim.h"
for f in tmh_engine.hip tmh_math.h tmh_model.h; do git show "$rev:tmhpvsim_amd/csrc/$f" > "$d/csrc/$f"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I "$d/include" \
  -o "tmhpvsim_amd/libtmh_$name.so" "$d/csrc/tmh_engine.hip"
rm -rf "$d"
