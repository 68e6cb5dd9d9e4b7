#!/bin/bash
# Stats workloads after a stats-kernel change: bench lines + PMC records of C3, C4, C5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02g}
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 45; do echo "[tick $(date +%T)]"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bash scripts/pmc_workload.sh ${TAG}_c3 c3 1048576 86400 fp32 stats faithful -- --workload c3 --steps 1 --warmup 1 --pipeline 1 || exit 1
PMC_PASS_TIMEOUT=240 bash scripts/pmc_workload.sh ${TAG}_c4 c4 16384 86400 fp32 stats faithful -- --workload c4 --steps 1 --warmup 1 || exit 1
bash scripts/pmc_workload.sh ${TAG}_c5 c5 65536 86400 fp32 stats markov compact=1 -- --workload c5 --steps 1 --warmup 1 || exit 1
SKIP_TESTS=1 bash scripts/gpu_round.sh $TAG c3 c4 c5 || exit 1
