"""The multi-GPU stats path on the one test GPU: two ranks (gloo, both on cuda:0) run
tmhpvsim_amd.dist.simulate_stats on their chain shards through the product path and
all-reduce; the node totals equal one unsharded run bit for bit -- histogram, peak and
energies (keyed Philox makes every chain independent of the partition, SURVEY.md §8e,
and the node energies are integer fixed-point sums, dist.chain_totals)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_simulate_stats_two_ranks_equal_one(tmp_path):
    from tmhpvsim_amd.dist import simulate_stats
    n_total, n_steps, world = 777, 6 * 3600, 2          # 3 day-windows of 7,200 s, odd shard sizes
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_gpu_worker.py"), str(n_total), str(n_steps),
                               str(tmp_path)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    one, bad1 = simulate_stats(n_total, "2019-09-05 06:00:00", n_steps, tz="Europe/Berlin", device="cuda:0",
                               window=7200)
    want = {k: v.cpu().numpy() for k, v in one.items()}
    assert want["hist"].sum() > 0 and want["energy_pv"] > 0
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npz")
        assert int(got["bad"]) == bad1
        np.testing.assert_array_equal(got["hist"], want["hist"])
        assert float(got["peak_residual"]) == float(want["peak_residual"])
        np.testing.assert_array_equal(got["energy_fx"], want["energy_fx"])   # integer energy sums: bit for bit
        for k in ("energy_pv", "energy_meter", "energy_residual"):
            assert float(got[k]) == float(want[k])


def test_simulate_stats_rccl_one_rank_equals_direct(tmp_path):
    """The RCCL all-reduce of the statistics (dist.all_reduce_stats: the int64 histogram and
    energy limbs in one SUM, the peak in a MAX) executed on the GPU: one rank over the
    `nccl` backend (RCCL; the test box has one GPU), whose node totals equal the
    unsharded run bit for bit."""
    from tmhpvsim_amd.dist import simulate_stats
    n_total, n_steps = 321, 2 * 3600
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    p = subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_gpu_worker.py"), str(n_total), str(n_steps),
                          str(tmp_path), "nccl"], env=env)
    assert p.wait(timeout=240) == 0
    one, bad1 = simulate_stats(n_total, "2019-09-05 06:00:00", n_steps, tz="Europe/Berlin", device="cuda:0",
                               window=7200)
    got = np.load(tmp_path / "rank0.npz")
    assert int(got["bad"]) == bad1
    np.testing.assert_array_equal(got["hist"], one["hist"].cpu().numpy())
    np.testing.assert_array_equal(got["energy_fx"], one["energy_fx"].cpu().numpy())
    assert float(got["peak_residual"]) == float(one["peak_residual"])
