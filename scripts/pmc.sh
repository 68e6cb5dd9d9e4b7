#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, gfx950 slot limits respected)
# over a short bench run.  Output: gpurun_out/pmc_<tag>/<pass>/...counter_collection.csv
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
TAG="${1:-r01}"
shift || true
ARGS="${*:---steps 1 --warmup 1 --no-cpu-baseline}"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
    "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pass $i: $counters"
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- \
      python "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo done
