"""One rank of tests/test_gpu_dist.py: dist.simulate_stats on cuda:0 over gloo
(every rank shares the one GPU of the test box, as bench.py's TMH_BENCH_SHARE_GPU
rehearsal does) or, with a fourth argument "nccl", over RCCL (one rank: the test box has
one GPU, and RCCL takes one GPU per rank); writes the node totals to OUT_DIR/rank<r>.npz."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmhpvsim_amd.dist import simulate_stats  # noqa: E402


def main():
    n_total, n_steps, out_dir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    backend = sys.argv[4] if len(sys.argv) > 4 else "gloo"
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
    else:
        dist.init_process_group("gloo")
    try:
        tot, bad = simulate_stats(n_total, "2019-09-05 06:00:00", n_steps, tz="Europe/Berlin", device="cuda:0",
                                  window=7200)
        np.savez(os.path.join(out_dir, f"rank{dist.get_rank()}.npz"), bad=bad,
                 **{k: v.cpu().numpy() for k, v in tot.items()})
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
