#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="${PYTEST_K:-}" bash scripts/gpu_tests.sh ${1:-wab} || exit $?
timeout -k 10 200 python scripts/diag_p1.py > gpurun_out/diag_p1_batch.txt 2>&1 || exit $?
cat gpurun_out/diag_p1_batch.txt
shift || true
bash scripts/varab.sh wab "$@"
