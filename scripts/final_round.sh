#!/bin/bash
# Round deliverables on the GPU box: GPU tests, the PMC record of the compacted C5
# expansion (its kernel changed), bench lines of every workload (+ fp64 C2), and the
# rocprofv3 kernel-trace statistics of the default bench command.
# Usage: bash scripts/final_round.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02f}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 45; do echo "[tick $(date +%T)]"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bash scripts/gpu_tests.sh $TAG || exit $?
if [ -z "${SKIP_PMC:-}" ]; then
  bash scripts/pmc_workload.sh ${TAG}_c5c c5 65536 86400 fp32 stats markov compact=1 -- --workload c5 --steps 1 --warmup 1 || exit $?
  cp gpurun_out/pmc_kernels.json profiles/pmc_kernels.json
fi
SKIP_TESTS=1 bash scripts/gpu_round.sh $TAG c2 c3 c4 c5 || exit $?
timeout -k 10 300 python -u bench.py --precision fp64 > gpurun_out/bench_${TAG}_c2_fp64.json 2> gpurun_out/bench_${TAG}_c2_fp64.err || exit $?
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" \
    -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.json" 2>&1 ) || exit $?
python3 scripts/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv | head -14
