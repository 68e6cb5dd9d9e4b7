#!/bin/bash
# One-GPU proxies of the strong-scaled workloads' N-GPU shards (bench.py --proxy-world N: rank 0's
# shard timed alone; projected_node_value = N x value; not a scaling measurement).
# Usage (GPU box): bash scripts/proxies.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
for spec in "c3 8 --steps 4 --warmup 1" "c4 2 --steps 6 --warmup 1" "c4 4 --steps 6 --warmup 1" "c4 8 --steps 6 --warmup 1" \
            "c5 8 --steps 5 --warmup 1"; do
  set -- $spec
  wl=$1 n=$2; shift 2
  out=gpurun_out/proxy_${TAG}_${wl}_n$n
  timeout -k 10 400 python bench.py --workload $wl --proxy-world $n --secondary none --no-cpu-baseline "$@" > $out.json 2> $out.err || { echo "failed: $spec"; tail -5 $out.err; exit 1; }
  python3 - $out.json $wl $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "N =", sys.argv[3], "shard value %.4g" % d["value"], "projected %.4g" % d["projected_node_value"], "ms/step %.2f" % d["ms_per_step"])
PY
done
