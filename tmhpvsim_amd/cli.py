"""`pvsim` / `metersim` entry points with the reference's options plus a batched
offline mode that drives the MI355X engine (tmhpvsim/pvsim.py:103-121,
tmhpvsim/metersim.py:79-95).

    python -m tmhpvsim_amd.cli pvsim FILE [--amqp-url URL] [--exchange NAME] [-v]
                                          [--realtime/--no-realtime]
                                          [--batch N --start T --seconds S --seed K
                                           --precision fp64|fp32 --all-chains OUT.npz]
    python -m tmhpvsim_amd.cli metersim [--amqp-url URL] [--exchange NAME] [-v]
                                        [--realtime/--no-realtime]
                                        [--batch N --start T --seconds S --seed K --out FILE]

Without --batch the commands are the reference's AMQP pipelines (a fanout
exchange carrying one JSON float per second, pvsim.py:43-84, metersim.py:13-62):
they need aio_pika and a broker and are not rebuilt here (out of scope);
the command says so and exits non-zero.

--batch N --no-realtime is the offline mode: N chains (site x scenario) advance
on the GPU for --seconds seconds from --start in one engine run, with the meter
draw fused into the kernel.  `pvsim` writes FILE exactly like the reference's
write_file (pvsim.py:72-84: header `time,meter,pv,residual load`, one row per
second, residual = meter - pv) for chain 0, and optionally every chain's traces
to an .npz.  `metersim` writes the messages it would publish, one JSON object per
line: {"timestamp": ..., "body": <json.dumps(meter)>} (metersim.py:38-42).
There is no CPU fallback: the batch mode fails if the engine cannot run.
"""
from __future__ import annotations

import csv
import datetime as dt
import json
import logging
import os

import click

logger = logging.getLogger(__name__)


def _batch_run(n, start, seconds, seed, precision, fields):
    from .engine import BatchedSim
    from .params import ModelParams
    import torch
    if not torch.cuda.is_available():
        raise click.ClickException("--batch runs on the MI355X engine and no GPU is visible (there is no CPU path)")
    params = ModelParams(seed=int(seed))
    sim = BatchedSim(int(n), start, tz=params.site.tz, params=params, precision=precision, device="cuda:0",
                     horizon=int(seconds))
    out = sim.run(int(seconds), trace=fields)
    torch.cuda.synchronize()
    bad = int((sim.status() != 0).sum())
    if bad:
        logger.warning(f"{bad} of {n} chains faulted (reference exceptions); their values are NaN")
    return {k: v.double().cpu().numpy() if v.dtype != torch.uint8 else v.cpu().numpy() for k, v in out.items()}


def _times(start, seconds):
    t0 = dt.datetime.fromisoformat(str(start))
    return [t0 + dt.timedelta(seconds=s) for s in range(int(seconds))]


def _need_batch(realtime, batch, name):
    if batch is None:
        try:
            import aio_pika  # noqa: F401
        except ImportError:
            raise click.ClickException(
                f"{name} without --batch is the reference's AMQP pipeline (aio_pika + a broker), which is not part of "
                "this build; use --batch N --no-realtime for the offline engine mode")
        raise click.ClickException(f"{name}: the AMQP pipeline is out of scope here; use --batch N --no-realtime")
    if realtime:
        raise click.ClickException("--batch is an offline mode: combine it with --no-realtime")


_common = [
    click.option("--amqp-url", default=os.environ.get("AMQP_URL"), help="AMQP URL (defaults to 'amqp://localhost:5672/')"),
    click.option("--exchange", default=os.environ.get("TMHPVSIM_EXCHANGE", "meter"),
                 help="The name of the exchange (defaults to 'meter')"),
    click.option("-v", "--verbose", count=True, help="Increase logging level from default WARN"),
    click.option("--realtime/--no-realtime", default=True, help="Switch off rate limiting (for simulation)"),
    click.option("--batch", type=int, default=None, help="offline engine mode: number of chains (site x scenario)"),
    click.option("--start", default="2019-09-06T12:00:00", help="batch mode: local wall-clock start time"),
    click.option("--seconds", type=int, default=86400, help="batch mode: seconds to simulate"),
    click.option("--seed", type=int, default=0x5EED, help="batch mode: keyed Philox seed"),
]


def common(f):
    for opt in reversed(_common):
        f = opt(f)
    return f


@click.group()
def main():
    """tmhpvsim entry points on the MI355X engine."""


@main.command()
@click.argument("file")
@common
@click.option("--precision", type=click.Choice(["fp64", "fp32"]), default="fp64", help="batch mode arithmetic")
@click.option("--all-chains", default=None, help="batch mode: also write every chain's traces to this .npz")
def pvsim(file, amqp_url, exchange, verbose, realtime, batch, start, seconds, seed, precision, all_chains):
    """Simulated PV + meter + residual load to FILE (CSV, pvsim.py:72-84)."""
    logging.basicConfig(level=logging.WARN - 10 * verbose)
    _need_batch(realtime, batch, "pvsim")
    out = _batch_run(batch, start, seconds, seed, precision, ("meter", "pv", "residual"))
    with open(file, mode="w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["time", "meter", "pv", "residual load"])
        m, p, r = out["meter"][:, 0], out["pv"][:, 0], out["residual"][:, 0]
        for i, t in enumerate(_times(start, seconds)):
            w.writerow([t, float(m[i]), float(p[i]), float(r[i])])
    if all_chains:
        import numpy as np
        np.savez(all_chains, **out)
    click.echo(f"wrote {seconds} rows to {file}" + (f" and {batch} chains to {all_chains}" if all_chains else ""))


@main.command()
@common
@click.option("--out", "out_file", default="-", help="batch mode: JSON-lines message file ('-' = stdout)")
def metersim(amqp_url, exchange, verbose, realtime, batch, start, seconds, seed, out_file):
    """Meter values as the AMQP messages of metersim.py:38-42, one JSON object per line."""
    logging.basicConfig(level=logging.WARN - 10 * verbose)
    _need_batch(realtime, batch, "metersim")
    out = _batch_run(batch, start, seconds, seed, "fp64", ("meter",))
    m = out["meter"]
    with click.open_file(out_file, "w") as fh:
        for i, t in enumerate(_times(start, seconds)):
            for c in range(m.shape[1]):
                rec = {"timestamp": t.isoformat(), "body": json.dumps(float(m[i, c]), ensure_ascii=False)}
                if m.shape[1] > 1:
                    rec["chain"] = c
                fh.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
