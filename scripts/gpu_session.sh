#!/bin/bash
# One GPU session: smoke, the -m gpu suite, the default bench line (with its secondary
# lines), and diagnostics named in $3 (walkprof: the walk's section profile from the
# -DTMH_WALK_PROF build).  Every GPU step has its own time limit; the first failure ends it.
# Usage (GPU box): bash scripts/gpu_session.sh TAG [pytest -k expression] [diagnostics]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-s}"
K="${2:-}"
D="${3:-}"
step() {   # step NAME SECONDS CMD...: run under its own limit, stop the session on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
step smoke 300 python __graft_entry__.py smoke
step pytest 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --durations=25 --timeout 400 \
    --timeout-method thread ${K:+-k "$K"}
fi
step bench 480 python bench.py --steps 20 --warmup 5
case "$D" in *counters*)
  (cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > "$OLDPWD/gpurun_out/counters_$TAG.txt" 2>&1; echo "counters rc=$?") ;;
esac
case "$D" in *walkprof*)
  step walkprof 240 env TMHPVSIM_LIB=$PWD/tmhpvsim_amd/libtmh_wprof.so python scripts/walk_prof.py --chains 4096 2048 ;;
esac
exit 0
