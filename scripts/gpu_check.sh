#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel summary.
# Every GPU step has its own time limit; a timeout / signal / crash ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-r01}"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 3; }
timeout -k 10 400 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; rc=$?
echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; tail -3 "$OUT/bench_$TAG.err"
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python "$ROOT/bench.py" --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1; rc=$?
echo "rocprof rc=$rc"; find "$OUT/prof_$TAG" -name "*stats*"
exit $rc
