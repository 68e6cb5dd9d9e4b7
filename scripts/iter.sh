#!/bin/bash
# One build -> measure iteration on the GPU box: GPU tests, default bench, expansion alone.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-it}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/b_${TAG}.json 2> gpurun_out/b_${TAG}.err || exit $?
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --pipeline 1 --no-cpu-baseline > gpurun_out/b_${TAG}_p1.json 2> gpurun_out/b_${TAG}_p1.err || exit $?
for f in gpurun_out/b_${TAG}.json gpurun_out/b_${TAG}_p1.json; do python3 -c "
import json; d=json.loads(open('$f').read()); r=d['roofline']
print('$f value %.4g ms/step %.3f expand %.3f alone %.3f frac %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms'], r['frac']), d.get('phases_ms'))"; done
