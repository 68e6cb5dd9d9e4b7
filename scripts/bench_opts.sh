#!/bin/bash
# Same-box A/B of bench option sets: bench_opts.sh TAG "opts1" "opts2" ... (two rounds)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
for rep in 1 2; do
i=0
for opts in "$@"; do  # BENCH_STEPS overrides steps/warmup
  i=$((i+1))
  timeout -k 10 200 python bench.py ${BENCH_SW:---steps 10 --warmup 3} --no-cpu-baseline $opts > gpurun_out/bo_${TAG}_$i.json 2> gpurun_out/bo_${TAG}_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/bo_${TAG}_$i.json').read()); r=d['roofline']
print('[$opts] value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms']), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
done
done
