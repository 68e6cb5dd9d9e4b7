#!/bin/bash
# Walk lanes per chain (tmh_set_walk_lanes) A/B: the invariance test, a few parity tests,
# then the default C2 bench with 16 / 8 / 4 lanes per chain.  Usage: walk_lanes_ab.sh TAG [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-wl}; shift
[ -n "${NOTEST:-}" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "walk_lanes or walk_chains or keyed_vs_oracle or segment_overflow or pipelined" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
[ -n "${NOTEST:-}" ] || grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_$TAG.log | tail -8
[ -n "${NOTEST:-}" ] || [ $rc -eq 0 ] || exit $rc
for G in ${GS:-16 8 4}; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --walk-lanes $G "$@" > gpurun_out/bm_${TAG}_g$G.json 2> gpurun_out/bm_${TAG}_g$G.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/bm_${TAG}_g$G.json').read())
print('G=$G value %.4g ms/step %.3f phases %s alone %.3f' % (d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['phases_ms'].items() if v}, d['roofline']['alone']['kernel_ms']))"
done
