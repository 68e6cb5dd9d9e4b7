#!/bin/bash
# PMC passes over one bench workload (one rocprofv3 run per counter group; gfx950
# slot limits: 8 SQ, 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2), 2 GRBM), then the
# dominant expand kernel's per-launch means into profiles/pmc_kernels.json.
# Usage (GPU box): bash scripts/pmc_workload.sh TAG WORKLOAD CHAINS LAUNCH_SECONDS PRECISION MODE CC -- BENCH ARGS
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1 WL=$2 CH=$3 LS=$4 PREC=$5 MODE=$6 CC=$7
shift 7
EXTRA=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do EXTRA="$EXTRA $1"; shift; done   # extra record keys k=v
[ "${1:-}" = "--" ] && shift
ARGS="$*"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp
i=0
for counters in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
    "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
    "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
    "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL ${PMC_PASS_TIMEOUT:-150} rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
python3 scripts/pmc_summary.py "$OUT" --record workload=$WL chains=$CH launch_seconds=$LS precision=$PREC mode=$MODE cc=$CC $EXTRA \
    > "$OUT/record.json" || exit 1
cp profiles/pmc_kernels.json gpurun_out/pmc_kernels.json
rm -rf "$OUT"/p[0-9]*/   # the per-dispatch CSVs (tens of MB for C4); summary.txt and record.json stay
cat "$OUT/record.json"
