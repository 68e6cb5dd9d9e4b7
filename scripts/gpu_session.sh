#!/bin/bash
# One GPU session: smoke, the -m gpu suite, the default bench line and the
# two-rank launcher rehearsal (bench.py --gpus 2 spawning its own ranks, both on
# device 0 over gloo).  Every GPU step has its own time limit; the first failure ends it.
# Usage (GPU box): bash scripts/gpu_session.sh TAG [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-s}"
K="${2:-}"
step() {   # step NAME SECONDS CMD...: run under its own limit, stop the session on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
}
step smoke 300 python __graft_entry__.py smoke
step pytest 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --durations=20 --timeout 400 \
    --timeout-method thread ${K:+-k "$K"}
step bench 300 python bench.py --steps 20 --warmup 5
step dist2 300 env TMH_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 6 --warmup 2
exit 0
