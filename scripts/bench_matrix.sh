#!/bin/bash
# A few bench variants in one GPU session (each with its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-m}"
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --pipeline 1 --no-cpu-baseline > gpurun_out/bm_${TAG}_p1.json 2> gpurun_out/bm_${TAG}_p1.err || exit $?
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --pipeline 2 --no-cpu-baseline > gpurun_out/bm_${TAG}_p2.json 2> gpurun_out/bm_${TAG}_p2.err || exit $?
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --pipeline 2 --mode stats --no-cpu-baseline > gpurun_out/bm_${TAG}_stats.json 2> gpurun_out/bm_${TAG}_stats.err || exit $?
for f in gpurun_out/bm_${TAG}_*.json; do echo "$f"; python3 -c "
import json,sys; d=json.loads(open('$f').read()); print(' value %.4g ms/step %.3f phases %s' % (d['value'], d['ms_per_step'], d.get('phases_ms')))"; done
