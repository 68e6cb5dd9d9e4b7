#!/bin/bash
# Expansion time vs chains per batch (workgroup-round / tail effects): alone + pipelined
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="$1"; shift
for n in "$@"; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --chains $n > gpurun_out/cs_${TAG}_$n.json 2> gpurun_out/cs_${TAG}_$n.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/cs_${TAG}_$n.json').read()); r=d['roofline']
print('chains $n value %.4g ms/step %.3f expand %.3f alone %.3f  alone ns/chain-day %.1f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms'], r['alone']['kernel_ms'] * 1e6 / $n))"
done
