#!/bin/bash
# The measurements committed under profiles/ for a round: the default bench line,
# the rocprofv3 kernel statistics of the same command, and the PMC passes
# (scripts/pmc.sh) whose FETCH_SIZE / WRITE_SIZE give the bench's `traffic`.
# Usage (GPU box): bash scripts/profile_round.sh r01
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-r01}"
cd "$ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" \
    -o run -- python "$ROOT/bench.py" --no-cpu-baseline > "$ROOT/gpurun_out/prof_$TAG.json" 2>&1 ) || exit $?
python3 scripts/kstats.py gpurun_out/prof_$TAG/run_kernel_stats.csv | head -12
bash scripts/pmc.sh "$TAG" --steps 1 --warmup 1 --pipeline 1 --no-cpu-baseline || exit $?
python3 -c "
import sys; sys.path.insert(0, 'scripts')
import pmc_summary
print(pmc_summary.write_traffic('gpurun_out/pmc_$TAG', 4096, 86400, out='gpurun_out/pmc_traffic_$TAG.json'))
" > gpurun_out/pmc_summary_$TAG.txt || exit $?
tail -3 gpurun_out/pmc_summary_$TAG.txt
