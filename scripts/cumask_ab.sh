#!/bin/bash
# Same-box A/B of bench.py schedule options (one bench per variant, two passes).
# Usage: cumask_ab.sh TAG "opts A" "opts B" ...   (each an argument string for bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
for rep in ${REPS:-1 2}; do
i=0
for o in "$@"; do
  i=$((i + 1))
  timeout -k 10 180 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $o > gpurun_out/cab_${TAG}_$i.json 2> gpurun_out/cab_${TAG}_$i.err || { tail -5 gpurun_out/cab_${TAG}_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cab_${TAG}_$i.json').read()); r=d['roofline']
print('[$o] value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms']), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
done
done
