#!/bin/bash
# Quick GPU iteration: GPU tests, pipelined / unpipelined bench, kernel stats (unpipelined).
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
export TMPDIR=/tmp
TAG="${1:-q}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
bash scripts/bench_matrix.sh $TAG || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run -- \
    python "$ROOT/bench.py" --steps 4 --warmup 1 --pipeline 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
python3 "$ROOT/scripts/kstats.py" "$ROOT/gpurun_out/prof_$TAG/run_kernel_stats.csv" | head -5
