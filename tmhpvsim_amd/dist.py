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


# ------------------------------------------------------------------ exact aggregate statistics
# One definition of the aggregate statistics, used by BatchedSim.stats_totals(),
# BatchPipeline.totals() and all_reduce_stats: every chain's accumulated seconds
# count, a faulted chain's seconds before its fault included (the kernels and the
# oracle stop a chain's sums and histogram at the fault, so energies and histogram
# cover the same chain-seconds).  Node energies are integers: each chain's fp64
# energy is rounded once to the fixed-point grid 2^-FX_BITS W s (exact: a scaling by
# a power of two, then round-half-even), split into two int64 limbs (hi = fx >> 31,
# lo = fx & (2^31 - 1), so n < 2^31 chains cannot overflow either sum) and summed as
# integers -- on the GPU, then by one integer SUM all-reduce -- so the totals do not
# depend on the order of the chains or on how they are partitioned over ranks; they
# are converted to fp64 once, at the end (correctly rounded, Python int division).
FX_BITS = 20           # 2^-20 W s ~ 1e-6 W s: ~1e-15 of a chain-day's ~4e8 W s
_LIMB = 31
_FX_MAX = 2.0 ** 62    # |energy| < 2^42 W s per chain (~15 years at 9 kW)
ENERGY_KEYS = ("energy_pv", "energy_meter", "energy_residual")


def energy_limbs(acc):
    """int64 [2, 3] limbs (hi, lo) of the fixed-point sums of acc[:3] ([>=3, n] fp64
    per-chain energies: sum pv, sum meter, sum residual) over the chains."""
    import torch
    e = torch.as_tensor(acc)[:3].to(torch.float64)
    fx = torch.round(e * float(1 << FX_BITS))          # exact scaling, one rounding
    if e.numel() and not bool((fx.abs() < _FX_MAX).all()):   # also rejects NaN / inf
        raise OverflowError("per-chain energy not finite or beyond the fixed-point range (2^42 W s)")
    fx = fx.to(torch.int64)
    return torch.stack([(fx >> _LIMB).sum(dim=1), (fx & ((1 << _LIMB) - 1)).sum(dim=1)])


def limbs_to_energies(limbs):
    """The three fp64 energies (W s) of int64 limbs [2, 3]: exact integer, one rounding."""
    hi, lo = limbs.cpu().tolist()
    return [((h << _LIMB) + l) / (1 << FX_BITS) for h, l in zip(hi, lo)]


def totals_from(limbs, peak, hist, device=None):
    """The totals dict: energy limbs (the exact quantity), the fp64 energies derived from
    them, the peak residual (fp64, a max: order-free) and the histogram (int64 bins)."""
    import torch
    dev = device if device is not None else limbs.device
    out = {k: torch.tensor(v, dtype=torch.float64, device=dev) for k, v in zip(ENERGY_KEYS, limbs_to_energies(limbs))}
    out["energy_fx"] = limbs.to(dev)
    out["peak_residual"] = torch.as_tensor(peak, dtype=torch.float64, device=dev).reshape(())
    if hist is not None:
        out["hist"] = hist.to(dev)
    return out


def chain_totals(acc, hist=None):
    """Node-local totals of per-chain accumulators acc [4, n] (fp64: sum pv, sum meter,
    sum residual, max residual; BatchedSim.chain_acc) and a histogram: every chain
    counts (a faulted chain with the seconds before its fault, a chain faulted at
    construction with none: zero sums and peak -inf)."""
    import torch
    acc = torch.as_tensor(acc)
    peak = acc[3].max() if acc.shape[1] else torch.tensor(float("-inf"), dtype=torch.float64, device=acc.device)
    return totals_from(energy_limbs(acc), peak, hist, device=acc.device)


def all_reduce_stats(tot: dict, group=None) -> dict:
    """Reduce node-local totals (chain_totals: BatchedSim.stats_totals(),
    BatchPipeline.totals()) over the ranks of `group`.

    Two collectives: one integer SUM over [energy limbs (6), hist...] packed as int64
    (exact and order-free, so the node totals do not depend on the partition), one
    MAX over the peak.  Returns a new dict with the node totals (every rank gets them).
    """
    import torch
    import torch.distributed as dist

    if "energy_fx" not in tot:
        raise KeyError("all_reduce_stats needs the exact energy limbs 'energy_fx' of chain_totals(); a totals dict "
                       "of the pre-round-5 format (fp64 energies only) cannot be reduced partition-independently")
    limbs = tot["energy_fx"]
    hist = tot.get("hist")
    dev = limbs.device if hist is None else hist.device
    packed = limbs.to(dev).reshape(6) if hist is None else torch.cat([limbs.to(dev).reshape(6), hist.to(torch.int64)])
    packed = packed.clone()
    peak = torch.as_tensor(tot["peak_residual"], dtype=torch.float64, device=dev).reshape(1).clone()
    if dist.is_available() and dist.is_initialized():   # (a one-rank group too: the collective runs)
        dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(peak, op=dist.ReduceOp.MAX, group=group)
    return totals_from(packed[:6].reshape(2, 3), peak[0], packed[6:] if hist is not None else None, device=dev)


def simulate_stats(n_total, start, n_steps, tz=None, params=None, precision="fp32", window=86400,
                   n_bins=4096, lo=-300.0, hi=9000.0, group=None, device=None, runner=None):
    """Node-wide stats run (C3/C4): this rank's shard of `n_total` chains, reduced over `group`.

    Returns (totals, faulted): the all-reduced totals (histogram and energies
    summed exactly, peak a max; every rank gets them; `chain_totals` semantics) and
    the node's count of faulted chains.  `runner(chain0, n, **spec) -> (totals,
    status)` simulates one shard (totals as `chain_totals` returns them); the
    default runs it on this rank's GPU (`BatchedSim`, stats mode, no trace).
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
