#!/bin/bash
# GPU test session: smoke + the -m gpu suite (each under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG="${1:-t}"
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --durations=15 --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_$TAG.log | tail -15
exit $rc
