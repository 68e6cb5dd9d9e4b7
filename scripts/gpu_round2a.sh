set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-a}; shift
timeout -k 10 300 python -u scripts/diag_fp32.py > gpurun_out/diag_fp32.log 2>&1; rc=$?; tail -6 gpurun_out/diag_fp32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_$TAG.log; [ $rc -le 1 ] || exit $rc
bash scripts/libab.sh $TAG "$@" || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 1 --pipeline 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
python3 "$GRAFT_REPO_ROOT/scripts/kstats.py" "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/run_kernel_stats.csv" > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.txt"; head -8 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.txt"
