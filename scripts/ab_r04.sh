#!/bin/bash
# Round-4 A/B runs on one box (each a bench line; one rep unless REPS is set):
#   c5 with the current library vs the 3-waves-per-SIMD C5 expansion (libtmh_c5w3.so);
#   the C4 one-GPU proxies at N = 8 with day windows vs 7-day windows, 32 vs 16 hardware queues;
#   C3 / C4 persistent statistics expansion vs one tile per workgroup (libtmh_nopersist.so).
# The variant libraries were built from the sources of their day (scripts/build_variant.sh,
# or -D flags: TMH_EXP_WAVES_F64, TMH_EXP_WG_STATS); the results are in DESIGN.md's round-4
# section, and the code they compared has since moved on, so this script records the runs
# rather than reproducing them on the current tree (scripts/ab_runs.sh runs new A/B lists).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-ab}"
run() {   # run NAME LIB ARGS...
  local name=$1 lib=$2; shift 2
  local l=$PWD/tmhpvsim_amd/libtmhpvsim.so; [ "$lib" = cur ] || l=$PWD/tmhpvsim_amd/libtmh_$lib.so
  TMHPVSIM_LIB=$l timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none "$@" \
      > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err || { echo "$name failed rc=$?"; tail -3 gpurun_out/ab_${TAG}_$name.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', 'value %.4g ms/step %.2f kernel %.3f alone %s' % (d['value'], d['ms_per_step'], r.get('kernel_ms') or 0, (r.get('alone') or {}).get('kernel_ms')), d.get('projected_node_value'))"
}
for rep in $(seq 1 ${REPS:-1}); do
  run c3_cur cur --workload c3 --steps 3 --warmup 1
  run c3_nop nopersist --workload c3 --steps 3 --warmup 1
  run c4_cur cur --workload c4 --steps 6 --warmup 1
  run c4_nop nopersist --workload c4 --steps 6 --warmup 1
  run c4p8_q16 cur --workload c4 --proxy-world 8 --steps 8 --warmup 1 --hw-queues 16
  run c5_cur cur --workload c5 --steps 2 --warmup 1
  run c5_w3 c5w3 --workload c5 --steps 2 --warmup 1
  run c5_loop c5loop --workload c5 --steps 2 --warmup 1
  run c5_loopw3 c5loopw3 --workload c5 --steps 2 --warmup 1
  run c4p8_d1 cur --workload c4 --proxy-world 8 --steps 8 --warmup 1
  run c4p8_d7 cur --workload c4 --proxy-world 8 --steps 8 --warmup 1 --window 604800
done
