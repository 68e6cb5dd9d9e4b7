#!/bin/bash
# A/B timing of library variants (debug helper): bench + per-kernel stats for each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  echo "== variant $v"
  TMHPVSIM_LIB=$PWD/tmhpvsim_amd/libtmh_$v.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bv_$v.json || exit $?
  cat gpurun_out/bv_$v.json
done
