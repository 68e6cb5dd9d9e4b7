"""Multi-process (gloo, world_size 2, CPU) tests of the sharding and the stats reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tmhpvsim_amd.dist import all_reduce_stats, shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_covers_range_once():
    for n_total in (0, 1, 7, 4096, 1_048_576, 1_000_003):
        for world in (1, 2, 3, 8):
            parts = [shard(n_total, r, world) for r in range(world)]
            ids = [c for c0, n in parts for c in range(c0, c0 + n)] if n_total < 10_000 else None
            assert sum(n for _, n in parts) == n_total
            assert parts[0][0] == 0
            for (a0, an), (b0, _) in zip(parts, parts[1:]):
                assert a0 + an == b0
            assert max(n for _, n in parts) - min(n for _, n in parts) <= 1
            if ids is not None:
                assert ids == list(range(n_total))
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _local_totals(rank, n_bins=64):
    g = np.random.default_rng(1234 + rank)
    hist = torch.as_tensor(g.integers(0, 1 << 40, n_bins), dtype=torch.int64)
    return dict(energy_pv=torch.tensor(float(g.normal() * 1e9), dtype=torch.float64),
                energy_meter=torch.tensor(float(g.normal() * 1e9), dtype=torch.float64),
                energy_residual=torch.tensor(float(g.normal() * 1e9), dtype=torch.float64),
                peak_residual=torch.tensor(float(g.normal() * 1e3), dtype=torch.float64),
                hist=hist)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = all_reduce_stats(_local_totals(rank))
        q.put((rank, {k: v.numpy().copy() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_all_reduce_stats_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    loc = [_local_totals(r) for r in range(world)]
    want_hist = sum(t["hist"] for t in loc).numpy()
    for r in range(world):
        got = res[r]
        assert np.array_equal(got["hist"], want_hist)                      # exact counts (< 2^53)
        for k in ("energy_pv", "energy_meter", "energy_residual"):
            assert got[k] == pytest.approx(float(sum(t[k] for t in loc)), rel=1e-15)
        assert got["peak_residual"] == max(float(t["peak_residual"]) for t in loc)


def test_all_reduce_stats_single_process_is_identity():
    t = _local_totals(0)
    out = all_reduce_stats(t)
    assert torch.equal(out["hist"], t["hist"])
    assert float(out["peak_residual"]) == float(t["peak_residual"])
    assert float(out["energy_pv"]) == float(t["energy_pv"])
