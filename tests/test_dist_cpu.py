"""Multi-process (gloo, world_size 2, CPU) tests of the sharding and the stats reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tmhpvsim_amd.dist import all_reduce_stats, shard, simulate_stats


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


# ---- simulate_stats end to end on CPU: each rank's shard simulated by the C oracle
# (test infrastructure standing in for the GPU runner), reduced over gloo; the node
# totals must equal one unsharded run (histogram bit for bit)
SIM = dict(start="2019-09-05 09:00:00", n_steps=7200, tz="Europe/Berlin")


def oracle_shard(chain0, n, start, n_steps, tz, params, precision, window, n_bins, lo, hi, device):
    from oracle import oracle as O
    from tmhpvsim_amd.params import ModelParams
    ref = O.run(params or ModelParams(), chain0, n, n_steps, start, tz=tz, outputs=(),
                stats=dict(n_bins=n_bins, lo=lo, hi=hi))
    ok = ref["status"] == 0
    acc = torch.as_tensor(ref["acc"])
    tot = dict(energy_pv=acc[ok, 0].sum(), energy_meter=acc[ok, 1].sum(), energy_residual=acc[ok, 2].sum(),
               peak_residual=acc[ok, 3].max(), hist=torch.as_tensor(ref["hist"].astype(np.int64).sum(0)))
    return tot, ref["status"]


def _sim_worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tot, bad = simulate_stats(n_total, runner=oracle_shard, **SIM)
        q.put((rank, {k: v.numpy().copy() for k, v in tot.items()}, bad))
    finally:
        dist.destroy_process_group()


def test_simulate_stats_sharded_equals_unsharded():
    world, n_total = 2, 101          # odd: the shards differ in size
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sim_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (t, b) for r, t, b in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one, bad1 = simulate_stats(n_total, runner=oracle_shard, **SIM)       # world 1: no process group
    assert int(one["hist"].sum()) > 0
    for r in range(world):
        got, bad = res[r]
        assert bad == bad1
        np.testing.assert_array_equal(got["hist"], one["hist"].numpy())   # bit for bit
        assert float(got["peak_residual"]) == float(one["peak_residual"])
        for k in ("energy_pv", "energy_meter", "energy_residual"):       # fp64 sums in another order
            assert float(got[k]) == pytest.approx(float(one[k]), rel=1e-12)
