#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="${PYTEST_K:-}" bash scripts/gpu_tests.sh ${1:-wq} || exit $?
shift || true
bash scripts/varab.sh wq "$@"
