#!/bin/bash
# pipeline-depth sweep of the C2 bench (each run under its own time limit)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for d in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 4 --pipeline $d --no-cpu-baseline > gpurun_out/bd_$d.json 2> gpurun_out/bd_$d.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/bd_$d.json').read()); print('depth $d', '%.4g' % d['value'], '%.3f ms' % d['ms_per_step'], d['phases_ms'])"
done
