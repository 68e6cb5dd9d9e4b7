#!/bin/bash
# Kernel traces of the pipelined C2 bench for a few option sets: trace_ab.sh TAG "opts1" "opts2" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG="$1"; shift
i=0
for opts in "$@"; do
  d=gpurun_out/tr_${TAG}_$i; mkdir -p $d
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $opts > $d/bench.json 2> $d/bench.err || exit $?
  f=$(find $d -name '*kernel_trace.csv' | head -1); mv "$f" $d/kernel_trace.csv
  find $d -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null
  echo "== [$opts]"; python3 -c "import json; d=json.loads(open('$d/bench.json').read()); print('value %.4g ms/step %.3f' % (d['value'], d['ms_per_step']))"
  python3 scripts/busy.py $d/kernel_trace.csv | tee $d/busy.txt
  i=$((i+1))
done
