#!/bin/bash
# A/B of bench variants: each extra argument is one quoted option string (one bench run each).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
i=0
for opts in "$@"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $opts > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_$i.json').read()); r=d['roofline']
print('[$opts] value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms']), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
  i=$((i+1))
done
