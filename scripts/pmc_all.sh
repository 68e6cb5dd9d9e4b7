#!/bin/bash
# Round PMC records for every bench workload (profiles/pmc_kernels.json) + the fp64 C2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}
mkdir -p gpurun_out
( while sleep 45; do echo "[tick $(date +%T)]"; done ) &
TICK=$!
trap "kill $TICK" EXIT
bash scripts/pmc_workload.sh ${TAG}_c2 c2 4096 86400 fp32 trace faithful -- --steps 1 --warmup 1 --pipeline 1 || exit 1
bash scripts/pmc_workload.sh ${TAG}_c3 c3 1048576 86400 fp32 stats faithful -- --workload c3 --steps 1 --warmup 1 || exit 1
bash scripts/pmc_workload.sh ${TAG}_c5 c5 65536 86400 fp32 stats markov -- --workload c5 --steps 1 --warmup 1 || exit 1
PMC_PASS_TIMEOUT=240 bash scripts/pmc_workload.sh ${TAG}_c4 c4 16384 86400 fp32 stats faithful -- --workload c4 --steps 1 --warmup 1 || exit 1
