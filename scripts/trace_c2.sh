#!/bin/bash
# Kernel trace of the pipelined C2 bench (rocprofv3 --kernel-trace --stats): trace_c2.sh TAG [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG="$1"; shift
mkdir -p gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/tr_$TAG/bench.json 2> gpurun_out/tr_$TAG/bench.err || exit $?
f=$(find gpurun_out/tr_$TAG -name '*kernel_trace.csv' | head -1)
cp "$f" gpurun_out/tr_$TAG/kernel_trace.csv
python3 scripts/timeline.py gpurun_out/tr_$TAG/kernel_trace.csv > gpurun_out/tr_$TAG/timeline.txt; rm -rf gpurun_out/tr_$TAG/*/; cat gpurun_out/tr_$TAG/timeline.txt
