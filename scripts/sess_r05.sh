#!/bin/bash
# Round-5 GPU session: smoke, then the -m gpu suite (optionally a -k subset), then A/B lines.
#   bash scripts/sess_r05.sh TAG [pytest -k expr | -] ['name|lib|bench args' ...]
# lib: cur = tmhpvsim_amd/libtmhpvsim.so, else tmhpvsim_amd/libtmh_<lib>.so.  Every GPU step runs
# under its own time limit and the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; K=${2:--}; shift 2 || shift $#
( while sleep 50; do echo "[tick $(date +%T)]" >> gpurun_out/tick_$TAG.log; done ) &
TICK=$!
trap "kill $TICK" EXIT
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
}
if [ "$K" != "skip" ]; then
  step smoke 300 python __graft_entry__.py smoke
  if [ "$K" = "-" ]; then
    step pytest 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --durations=30 --timeout 600 --timeout-method thread
  else
    step pytest 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --durations=30 --timeout 600 --timeout-method thread -k "$K"
  fi
fi
for spec in "$@"; do
  IFS='|' read -r name lib args <<< "$spec"
  l=$PWD/tmhpvsim_amd/libtmhpvsim.so; [ "$lib" = cur ] || l=$PWD/tmhpvsim_amd/libtmh_$lib.so
  out=gpurun_out/ab_${TAG}_$name
  TMHPVSIM_LIB=$l timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none $args > $out.json 2> $out.err \
    || { echo "$name failed rc=$?"; tail -3 $out.err; exit 1; }
  python3 - $out.json $name <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d.get("roofline") or {}
al = (r.get("alone") or {}).get("kernel_ms")
print("%-10s value %.4g ms/step %.3f expand %.3f alone %s" % (sys.argv[2], d["value"], d["ms_per_step"], r.get("kernel_ms") or 0, al),
      {k: round(v, 3) for k, v in (d.get("phases_ms") or {}).items() if v})
EOF
done
exit 0
