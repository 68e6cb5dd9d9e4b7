"""Drop-in for the sampling half of tmhpvsim.cloud_cover_hourly
(reference: tmhpvsim/cloud_cover_hourly.py:93-106, 269-316).

Host-side helpers with the reference's names and signatures: the asymmetric
Laplace distribution, the shape table -> frozen-distribution loaders and the
hourly Markov-chain generator `get_cloud_cover`, drawing from numpy's global
RandomState through scipy exactly as the reference does.  The batched engine
runs the same hourly chain per GPU chain (`draw_cc_from`, `markov_cc_kernel`,
per-site tables via tmh_set_shape_tables).  The reference's offline fitting
half (ERA5 download, pymc3; :41-267) is replaced by
tmhpvsim_amd.params.infer_shapes.  Checked draw for draw against the reference
(tests/test_shims_cpu.py, fixture tests/golden/shims.npz).
"""
from __future__ import annotations

import numpy as np
import scipy.stats

from .params import EDGES, SHAPE_IS_T, SHAPES


class _asymmetric_laplace(scipy.stats.rv_continuous):
    """Asymmetric Laplace with asymmetry kappa (cloud_cover_hourly.py:93-106):
    density exp(-kappa x) for x >= 0 and exp(x / kappa) below, over kappa + 1/kappa."""

    def _pdf(self, x, kappa):
        rate = np.where(x >= 0, -kappa, 1 / kappa)
        return 1 / (kappa + 1 / kappa) * np.exp(rate * x)

    def _ppf(self, y, kappa):
        k2 = kappa ** 2   # mass below 0 is kappa^2 / (1 + kappa^2)
        return np.where(y < k2 / (1 + k2),
                        kappa * np.log((1 + k2) / k2 * y),
                        -1 / kappa * np.log((1 + k2) * (1 - y)))


asymmetric_laplace = _asymmetric_laplace()

_DISTS = {"al": asymmetric_laplace, "t": scipy.stats.t}


def get_fixed_distribution(dist, **params):
    """Frozen 'al' (kappa, loc, scale) or 't' (df, loc, scale) distribution (:269-276)."""
    if dist not in _DISTS:
        raise NotImplementedError(f"distribution {dist!r} is not implemented in get_distributions_from_shapes")
    return _DISTS[dist](**params)


def get_distributions_from_shapes(shapes):
    """pd.Series interval -> frozen distribution from a shape DataFrame (:278-280)."""
    import pandas as pd
    return pd.Series([get_fixed_distribution(**row.dropna()) for _, row in shapes.iterrows()], shapes.index)


def _default_shapes():
    """The packaged table (data/mc_dist_shapes.csv) as pandas loads it: the bits
    of tmhpvsim_amd.params.SHAPES."""
    import pandas as pd
    lefts = (-0.001,) + EDGES[:-1]
    rows = []
    for (loc, scale, kappa, df), t in zip(SHAPES, SHAPE_IS_T):
        rows.append(dict(loc=loc, scale=scale, kappa=np.nan if t else kappa, df=df if t else np.nan,
                         dist="t" if t else "al"))
    return pd.DataFrame(rows, index=pd.IntervalIndex.from_tuples(list(zip(lefts, EDGES))))


def get_distributions_from_shapes_file(dist_shapes_file=None):
    """Frozen distributions of a shape table in mc_dist_shapes.csv format (:282-288);
    None = the packaged table."""
    import pandas as pd
    if dist_shapes_file is None:
        return get_distributions_from_shapes(_default_shapes())
    shapes = pd.read_csv(dist_shapes_file, index_col=[0, 1])
    shapes.index = pd.IntervalIndex.from_tuples(shapes.index)
    return get_distributions_from_shapes(shapes)


def get_cloud_cover(distributions, initial_state=1.):
    """Generator of hourly cloud covers in [0, 1] (:290-316): the Markov chain whose
    step from state s is drawn from the distribution of the bin holding s (right-
    closed bins; np.searchsorted on the right edges), clipped to [0, 1]."""
    right = np.asarray(distributions.index.map(lambda iv: iv.right))
    dists = np.asarray(distributions)
    state = np.clip(initial_state, 0., 1.)
    while True:
        state = np.clip(state + dists[np.searchsorted(right, state)].rvs(), 0., 1.)
        yield state
