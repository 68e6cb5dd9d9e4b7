#!/bin/bash
# Build an A/B variant of the working-tree library with sed edits applied to its sources:
#   build_variant.sh NAME 'sed-expr' ['sed-expr' ...] -> tmhpvsim_amd/libtmh_NAME.so
# (each expression runs over tmh_engine.hip, tmh_model.h and tmh_math.h; the build fails
# if an expression changes nothing, so a stale pattern cannot pass as a variant)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
d=$(mktemp -d)
cp -r include "$d/include"; mkdir -p "$d/csrc"
cp tmhpvsim_amd/csrc/tmh_engine.hip tmhpvsim_amd/csrc/tmh_model.h tmhpvsim_amd/csrc/tmh_math.h "$d/csrc/"
for e in "$@"; do
  before=$(cat "$d"/csrc/* | md5sum)
  sed -i "$e" "$d"/csrc/tmh_engine.hip "$d"/csrc/tmh_model.h "$d"/csrc/tmh_math.h
  [ "$before" != "$(cat "$d"/csrc/* | md5sum)" ] || { echo "no change: $e" >&2; exit 1; }
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off ${EXTRA:-} -I "$d/include" \
  -o "tmhpvsim_amd/libtmh_$name.so" "$d/csrc/tmh_engine.hip"
rm -rf "$d"
