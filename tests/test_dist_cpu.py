"""Multi-process (gloo, world_size 2, CPU) tests of the sharding and the stats reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tmhpvsim_amd.dist import FX_BITS, all_reduce_stats, chain_totals, energy_limbs, shard, simulate_stats


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


def _local_acc(rank, n=257):
    """synthetic per-chain accumulators [4, n]: energies of chain-years (~1e11 W s, both signs)"""
    g = np.random.default_rng(1234 + rank)
    acc = g.normal(size=(4, n)) * np.array([[1e11], [1e11], [1e11], [1e3]])
    return torch.as_tensor(acc)


def _local_totals(rank, n_bins=64):
    g = np.random.default_rng(99 + rank)
    hist = torch.as_tensor(g.integers(0, 1 << 40, n_bins), dtype=torch.int64)
    return chain_totals(_local_acc(rank), hist)


def _exact(accs):
    """sum of every chain's energy rounded to the 2^-FX_BITS grid, in Python integers, then
    one correctly rounded conversion"""
    out = []
    for k in range(3):
        s = sum(int(v) for a in accs for v in np.round(a[k].numpy() * 2.0 ** FX_BITS))
        out.append(s / (1 << FX_BITS))
    return out


def test_energy_limbs_exact_and_order_free():
    acc = _local_acc(0, n=1001)
    perm = torch.randperm(1001, generator=torch.Generator().manual_seed(5))
    a, b = chain_totals(acc), chain_totals(acc[:, perm])
    assert torch.equal(a["energy_fx"], b["energy_fx"])            # integer sums: any order
    for k, want in zip(("energy_pv", "energy_meter", "energy_residual"), _exact([acc])):
        assert float(a[k]) == want
    # a faulted chain's pre-fault seconds count; a chain faulted at construction adds nothing
    z = torch.zeros(4, 1, dtype=torch.float64)
    z[3] = -float("inf")
    c = chain_totals(torch.cat([acc, z], dim=1))
    assert torch.equal(c["energy_fx"], a["energy_fx"]) and float(c["peak_residual"]) == float(a["peak_residual"])
    with pytest.raises(OverflowError):
        energy_limbs(torch.tensor([[float("nan")], [0.0], [0.0], [0.0]]))


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
        assert np.array_equal(got["hist"], want_hist)                      # exact counts (int64)
        for k, want in zip(("energy_pv", "energy_meter", "energy_residual"), _exact([_local_acc(q) for q in range(world)])):
            assert float(got[k]) == want                                    # exact integer sums, one rounding
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
# markov cc: chains fault (the reference's AssertionError) within the run, so the
# faulted-chain rule is exercised across the shards
SIMS = {"faithful": SIM, "markov": dict(SIM, n_steps=2 * 86400)}


def _params(cc):
    from tmhpvsim_amd.params import CC_MARKOV, ModelParams
    return ModelParams(cc_mode=CC_MARKOV) if cc == "markov" else None


def oracle_shard(chain0, n, start, n_steps, tz, params, precision, window, n_bins, lo, hi, device):
    from oracle import oracle as O
    from tmhpvsim_amd.params import ModelParams
    ref = O.run(params or ModelParams(), chain0, n, n_steps, start, tz=tz, outputs=(),
                stats=dict(n_bins=n_bins, lo=lo, hi=hi))
    # the product's definition (dist.chain_totals): every chain's accumulated seconds
    tot = chain_totals(torch.as_tensor(ref["acc"]).T.contiguous(), torch.as_tensor(ref["hist"].astype(np.int64).sum(0)))
    return tot, ref["status"]


def _sim_worker(rank, world, port, n_total, cc, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tot, bad = simulate_stats(n_total, runner=oracle_shard, params=_params(cc), **SIMS[cc])
        q.put((rank, {k: v.numpy().copy() for k, v in tot.items()}, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cc", ["faithful", "markov"])
def test_simulate_stats_sharded_equals_unsharded(cc):
    """Two gloo ranks == one unsharded run, bit for bit: histogram, peak and the
    energies (integer limbs and their fp64 values).  markov: about a third of the chains
    fault within the two days (the reference's AssertionError), so the faulted-chain rule (their
    seconds before the fault count, in energies and histogram alike) spans the shards."""
    world, n_total = 2, 101          # odd: the shards differ in size
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sim_worker, args=(r, world, port, n_total, cc, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (t, b) for r, t, b in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one, bad1 = simulate_stats(n_total, runner=oracle_shard, params=_params(cc), **SIMS[cc])   # world 1
    assert int(one["hist"].sum()) > 0
    if cc == "markov":
        assert bad1 > n_total // 4, "the markov case needs chains that fault"
    for r in range(world):
        got, bad = res[r]
        assert bad == bad1
        np.testing.assert_array_equal(got["hist"], one["hist"].numpy())   # bit for bit
        assert float(got["peak_residual"]) == float(one["peak_residual"])
        assert np.array_equal(got["energy_fx"], one["energy_fx"].numpy())  # integer energy sums: bit for bit
        for k in ("energy_pv", "energy_meter", "energy_residual"):
            assert float(got[k]) == float(one[k])
