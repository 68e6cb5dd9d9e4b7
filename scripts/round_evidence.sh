#!/bin/bash
# The measurements committed under profiles/ for a round.  Usage (GPU box):
#   round_evidence.sh TAG c2      default bench line (with cpu_baseline), rocprofv3 kernel statistics of
#                                 the same command, the C2 PMC record (traffic / VALU of this build)
#   round_evidence.sh TAG stats   PMC records of C3 / C5 / C4, then their bench lines and the fp64 C2 line
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1 WHAT=${2:-c2}
cd "$ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 45; do echo "[tick $(date +%T)]"; done ) &
TICK=$!
trap "kill $TICK" EXIT
if [ "$WHAT" = c2 ]; then
  bash scripts/pmc_workload.sh ${TAG}_c2 c2 4096 86400 fp32 trace faithful -- --steps 1 --warmup 1 --pipeline 1 || exit 1
  bash scripts/pmc_workload.sh ${TAG}_c2f64 c2 4096 86400 fp64 trace faithful -- --precision fp64 --steps 1 --warmup 1 --pipeline 1 || exit 1
  cp gpurun_out/pmc_kernels.json profiles/pmc_kernels.json
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_c2.json 2> gpurun_out/bench_${TAG}_c2.err || exit 1
  cat gpurun_out/bench_${TAG}_c2.json
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" \
      -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$ROOT/gpurun_out/prof_$TAG.json" 2>&1 ) || exit 1
  f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/kstats_$TAG.csv
  python3 scripts/kstats.py gpurun_out/kstats_$TAG.csv 14 | tee gpurun_out/kstats_$TAG.txt
  t=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
  python3 scripts/kstats_launches.py "$t" expand_kernel | tee -a gpurun_out/kstats_$TAG.txt
  rm -rf gpurun_out/prof_$TAG
else
  bash scripts/pmc_workload.sh ${TAG}_c3 c3 1048576 86400 fp32 stats faithful -- --workload c3 --steps 1 --warmup 1 || exit 1
  bash scripts/pmc_workload.sh ${TAG}_c5 c5 65536 86400 fp32 stats markov compact=1 -- --workload c5 --steps 1 --warmup 1 || exit 1
  C4WIN=$(python3 -c "from tmhpvsim_amd.pipeline import pipeline_defaults as d; print(d('c4').window)")
  PMC_PASS_TIMEOUT=240 bash scripts/pmc_workload.sh ${TAG}_c4 c4 16384 $C4WIN fp32 stats faithful -- --workload c4 --steps 1 --warmup 1 || exit 1
  cp gpurun_out/pmc_kernels.json profiles/pmc_kernels.json
  for wl in "c3 --steps 4 --warmup 1" "c4 --steps 6 --warmup 1" "c5 --steps 5 --warmup 1"; do
    set -- $wl
    timeout -k 10 600 python -u bench.py --workload $wl > gpurun_out/bench_${TAG}_$1.json 2> gpurun_out/bench_${TAG}_$1.err || exit 1
    cat gpurun_out/bench_${TAG}_$1.json
  done
  timeout -k 10 300 python -u bench.py --precision fp64 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_c2_fp64.json 2> gpurun_out/bench_${TAG}_c2_fp64.err || exit 1
  cat gpurun_out/bench_${TAG}_c2_fp64.json
fi
