#!/bin/bash
# Build an A/B variant of the library: build_variant.sh NAME -DFLAG=... -> tmhpvsim_amd/libtmh_NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -I include "$@" \
  -o tmhpvsim_amd/libtmh_$name.so tmhpvsim_amd/csrc/tmh_engine.hip
