#!/bin/bash
# One GPU session: smoke + -m gpu suite, then the bench lines of every workload.
# Usage (GPU box): bash scripts/gpu_round.sh TAG [workloads...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}
shift || true
WLS="${*:-c2 c3 c4 c5}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  bash scripts/gpu_tests.sh $TAG || exit $?
fi
for w in $WLS; do
  timeout -k 10 420 python -u bench.py --workload $w ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}_$w.json 2> gpurun_out/bench_${TAG}_$w.err || { echo "bench $w rc=$?"; tail -5 gpurun_out/bench_${TAG}_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'frac', r.get('frac'), 'kernel_ms', r.get('kernel_ms'))" gpurun_out/bench_${TAG}_$w.json $w
done
