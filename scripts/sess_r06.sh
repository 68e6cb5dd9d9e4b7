#!/bin/bash
# Round-6 GPU session steps (each under its own time limit; a failure ends the script).
# usage: bash scripts/sess_r06.sh TAG STEP...   steps: smoke | tests:<pytest -k expr> | alltests |
#        bench:<n reps>[:extra bench args] | prof | pmc:<workload>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for step in "$@"; do
  case "$step" in
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed rc=$?"; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    tests:*)
      K="${step#tests:}"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rf --durations=10 --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pyt_$TAG.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pyt_$TAG.log | tail -25
      [ $rc -eq 0 ] || exit $rc ;;
    alltests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rf --durations=15 --timeout 300 --timeout-method thread > gpurun_out/pytest_all_$TAG.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_all_$TAG.log | tail -15
      [ $rc -eq 0 ] || exit $rc ;;
    bench:*)
      rest="${step#bench:}"; reps="${rest%%:*}"; extra=""; [ "$rest" != "$reps" ] && extra="${rest#*:}"
      for i in $(seq 1 $reps); do
        timeout -k 10 400 python bench.py --secondary none --no-cpu-baseline $extra > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}_$i.err; exit 1; }
        python - "gpurun_out/bench_${TAG}_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.4g ms/step %.4f kernel %.4f alone %s frac %.3f stamp %s" % (d["value"], d["ms_per_step"], r.get("kernel_ms") or 0,
      r.get("alone", {}).get("kernel_ms"), r.get("frac") or 0, d.get("lib_stamp")))
PY
      done ;;
    ab:*)   # ab:<reps>:<VAR>: alternate bench runs with VAR=1 / VAR=0 (C2 defaults)
      rest="${step#ab:}"; reps="${rest%%:*}"; var="${rest#*:}"
      for i in $(seq 1 $reps); do
        for v in 1 0; do
          env $var=$v timeout -k 10 400 python bench.py --secondary none --no-cpu-baseline > gpurun_out/ab_${TAG}_${v}_$i.json 2> gpurun_out/ab_${TAG}_${v}_$i.err || { echo "bench failed"; tail -5 gpurun_out/ab_${TAG}_${v}_$i.err; exit 1; }
          python - "gpurun_out/ab_${TAG}_${v}_$i.json" "$var=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%s value %.4g ms/step %.4f kernel %.4f alone %.4f" % (sys.argv[2], d["value"], d["ms_per_step"], r["kernel_ms"], r["alone"]["kernel_ms"]))
PY
        done
      done ;;
    prof)
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/prof_$TAG" -o run -- \
          python3 "$OLDPWD/bench.py" --secondary none --no-cpu-baseline > "$OLDPWD/gpurun_out/prof_$TAG.log" 2>&1 ) || { echo "rocprof failed"; exit 1; }
      python3 scripts/kstats.py "$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -print -quit)" > gpurun_out/kstats_$TAG.txt 2>&1; cat gpurun_out/kstats_$TAG.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
