#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter group; gfx950 slot
# limits: 8 SQ, 4 TCC, 2 TA, 2 GRBM).  Output gpurun_out/pmc_<tag>/p<i>/run_counter_collection.csv
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-x}"
shift || true
ARGS="${*:---steps 2 --warmup 1 --pipeline 1 --no-cpu-baseline}"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp
i=0
for counters in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
    "SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES" \
    "TCC_EA0_WRREQ TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_BUSY" \
    "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- \
      python "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1 || true
grep -A3 "expand_kernel" "$OUT/summary.txt" | head -12
