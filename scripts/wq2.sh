#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="walk or time_parallel or segment or pipelined" bash scripts/gpu_tests.sh wq2 || exit $?
bash scripts/varab.sh wq2 'old|old|' 'cur|cur|' 'w2c2|cur|--walks 2 --walk-cpr 2' 'w2c2p5|cur|--walks 2 --walk-cpr 2 --pipeline 5' || exit $?
bash scripts/trace_c2.sh w2 --walks 2 --walk-cpr 2 || exit $?
python3 scripts/walkgaps.py gpurun_out/tr_w2/kernel_trace.csv > gpurun_out/tr_w2/walkgaps.txt
python3 scripts/timeline.py gpurun_out/tr_w2/kernel_trace.csv > gpurun_out/tr_w2/timeline.txt
tail -8 gpurun_out/tr_w2/timeline.txt
