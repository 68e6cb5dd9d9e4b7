#!/bin/bash
# N > 1 rehearsal of bench.py on a one-GPU box: torchrun with 2 ranks sharing
# device 0 over gloo (TMH_BENCH_SHARE_GPU=1); the scaling runs use one GPU per rank
# and RCCL.  C2 (trace, no collective) and C3-sized stats (the all-reduce).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp TMH_BENCH_SHARE_GPU=1
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/dist2_c2.json 2> gpurun_out/dist2_c2.err || exit $?
cat gpurun_out/dist2_c2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --workload c3 --chains 131072 --steps 2 --warmup 1 > gpurun_out/dist2_c3.json 2> gpurun_out/dist2_c3.err || exit $?
cat gpurun_out/dist2_c3.json
# C4 (multi-window statistics schedule, 30-day windows) through bench.py's own launcher
timeout -k 10 300 python bench.py --gpus 2 --workload c4 --chains 4096 --steps 2 --warmup 1 > gpurun_out/dist2_c4.json 2> gpurun_out/dist2_c4.err || exit $?
cat gpurun_out/dist2_c4.json
