#!/bin/bash
# PMC passes over the segment walk alone for walk lanes G in $GS: walk_pmc.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
export TMPDIR=/tmp
cd /tmp
for G in ${GS:-16 8 4}; do
  timeout -k 10 60 python3 $ROOT/scripts/walk_only.py --walk-lanes $G || exit $?
  i=0
  for counters in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY" \
                  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"; do
    i=$((i+1))
    d=$ROOT/gpurun_out/wpmc_${TAG}_g${G}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d $d -o run -- python3 $ROOT/scripts/walk_only.py --walk-lanes $G > $d.log 2>&1 || { echo "pass $i G=$G failed"; tail -3 $d.log; continue; }
    f=$(find $d -name '*counter_collection.csv' | head -1)
    python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(float); n = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    if "segments_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print({k: "%.3g" % (v / max(1, n[k]) * 1) for k, v in acc.items()}, "dispatch-counter rows", dict(n))
PY
    find $d -mindepth 1 -type d -exec rm -rf {} + 2>/dev/null
  done
done
