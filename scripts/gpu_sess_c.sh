#!/bin/bash
# GPU session: the -m gpu suite, then same-box A/B of library builds (scripts/libab.sh) on
# C2 and on C3 / C4.  Usage: gpu_sess_c.sh TAG "C2 variants" ["C3/C4 variants"]
# (variants: "cur" = libtmhpvsim.so, else libtmh_<v>.so; the C3/C4 list defaults to the C2 one)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-c} V2=${2:-"nskip cur"}
V34=${3:-$V2}
if [ -x scripts/micro/isa_rate ]; then timeout -k 10 120 scripts/micro/isa_rate > gpurun_out/isa_rate_$TAG.txt 2>&1 || exit $?; cat gpurun_out/isa_rate_$TAG.txt; fi
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
fi
bash scripts/libab.sh ${TAG}c2 $V2 || exit $?
BARGS="--workload c3 --steps 4 --warmup 1" bash scripts/libab.sh ${TAG}c3 $V34 || exit $?
BARGS="--workload c4 --steps 3 --warmup 1" bash scripts/libab.sh ${TAG}c4 $V34 || exit $?
if [ -n "${C5:-}" ]; then BARGS="--workload c5 --steps 2 --warmup 1" bash scripts/libab.sh ${TAG}c5 $V34 || exit $?; fi
