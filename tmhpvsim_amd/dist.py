"""Multi-GPU: chain sharding and the one exchange step.

Chains are independent (no cross-chain term in clearskyindexmodel.py,
cloud_cover_binary.py or pvmodel.py), so each rank simulates a contiguous range
of global chain ids and keyed Philox makes every chain's result independent of
the partition.  The only collective is the reduction of the aggregate
statistics at the end of a run: histogram and energies are summed, the peak
residual is a max.  On ROCm the "nccl" backend is RCCL (xGMI); tests use gloo.
"""
from __future__ import annotations


def shard(n_total: int, rank: int, world: int):
    """Contiguous chain range of `rank`: returns (chain0, n_local); sizes differ by at most 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(int(n_total), world)
    chain0 = rank * base + min(rank, extra)
    return chain0, base + (1 if rank < extra else 0)


def all_reduce_stats(tot: dict, group=None) -> dict:
    """Reduce BatchedSim.stats_totals() over the ranks of `group` (in place on device).

    Two collectives: one SUM over [energy_pv, energy_meter, energy_residual, hist...]
    packed as fp64 (bin counts stay exact below 2^53), one MAX over the peak.
    Returns a new dict with the node totals (every rank gets them).
    """
    import torch
    import torch.distributed as dist

    e = torch.stack([torch.as_tensor(tot[k], dtype=torch.float64)
                     for k in ("energy_pv", "energy_meter", "energy_residual")]).reshape(3)
    hist = tot.get("hist")
    dev = e.device if hist is None else hist.device
    e = e.to(dev)
    packed = e if hist is None else torch.cat([e, hist.to(torch.float64)])
    peak = torch.as_tensor(tot["peak_residual"], dtype=torch.float64, device=dev).reshape(1).clone()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(peak, op=dist.ReduceOp.MAX, group=group)
    out = dict(energy_pv=packed[0], energy_meter=packed[1], energy_residual=packed[2], peak_residual=peak[0])
    if hist is not None:
        out["hist"] = packed[3:].to(torch.int64)
    return out


def simulate_stats(n_total, start, n_steps, tz=None, params=None, precision="fp32", window=86400,
                   n_bins=4096, lo=-300.0, hi=9000.0, group=None, device=None, runner=None):
    """Node-wide stats run (C3/C4): this rank's shard of `n_total` chains, reduced over `group`.

    Returns (totals, faulted): the all-reduced totals (histogram and energies
    summed, peak a max; every rank gets them) and the node's count of faulted
    chains.  `runner(chain0, n, **spec) -> (totals, status)` simulates one shard;
    the default runs it on this rank's GPU (`BatchedSim`, stats mode, no trace).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    chain0, n = shard(n_total, rank, world)
    spec = dict(start=start, n_steps=n_steps, tz=tz, params=params, precision=precision, window=window,
                n_bins=n_bins, lo=lo, hi=hi, device=device)
    tot, status = (runner or _gpu_shard)(chain0, n, **spec)
    tot = all_reduce_stats(tot, group=group)
    bad = torch.tensor([int((status != 0).sum())], dtype=torch.int64, device=tot["energy_pv"].device)
    if world > 1:
        dist.all_reduce(bad, op=dist.ReduceOp.SUM, group=group)
    return tot, int(bad[0])


def _gpu_shard(chain0, n, start, n_steps, tz, params, precision, window, n_bins, lo, hi, device):
    from .engine import BatchedSim
    sim = BatchedSim(n, start, tz=tz, params=params, precision=precision, chain0=chain0, device=device,
                     horizon=n_steps)
    sim.enable_stats(n_bins=n_bins, lo=lo, hi=hi)
    sim.run(n_steps, trace=(), window=window)
    return sim.stats_totals(), sim.status()
