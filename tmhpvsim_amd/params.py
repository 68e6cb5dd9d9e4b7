"""Model parameters for the batched simulator (plain data, no compute).

Shape table
    The six hourly cloud-cover step distributions of
    tmhpvsim/data/mc_dist_shapes.csv as the reference LOADS them
    (tmhpvsim/cloud_cover_hourly.py:278-288, pandas default float parser), bit
    for bit (pinned by tests/test_oracle_golden.py against
    tests/golden/functions.npz).  Bins are right-closed with right edges
    EDGES; the draw uses the bin `searchsorted(EDGES, state)` (side='left',
    cloud_cover_hourly.py:309,314).

Site / PV system (tmhpvsim/pvmodel.py:12-30)
    Munich: latitude 48.12, longitude 11.60, altitude 34 m, tilt = latitude,
    surface azimuth 180, tz Europe/Berlin; pvlib's PVSystem default albedo
    0.25; sapm_celltemp with wind 0, air 20 C (pvmodel.py:69-70).

Module / inverter
    pvmodel.py:13-17 names the SAM entries "Hanwha_HSL60P6_PA_4_250T__2013_"
    (Sandia module DB) and "ABB__MICRO_0_25_I_OUTD_US_208_208V__CEC_2014_"
    (CEC inverter DB).  Those databases ship with pvlib, which is absent from
    this image (and unfetchable), so the numbers below are STAND-INS of the
    right class (a 60-cell 250 W mc-Si module, a 250 W micro-inverter) and are
    explicit, overridable inputs.  PV parity against pvlib is unpinned
    (DESIGN.md); parity of the kernels against the C oracle is exact to 1e-12.

Linke turbidity
    pvlib's LinkeTurbidities.h5 lookup (clearsky.lookup_linke_turbidity) is
    replaced by 12 monthly values (a central-European climatology stand-in),
    interpolated by day of year exactly as pvlib 0.6.3 interpolates them.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

EDGES = (0.1, 0.3, 0.7, 0.9, 0.99, 1.0)
# (loc, scale, kappa, df) per bin; kappa NaN for the Student-t bin, df NaN otherwise
SHAPES = (
    (-float.fromhex("0x1.e798442f368e5p-14"), float.fromhex("0x1.19aae076866b8p-5"),
     float.fromhex("0x1.351825923f16fp-1"), math.nan),
    (-float.fromhex("0x1.7743f483ff9e8p-5"), float.fromhex("0x1.bb2006b5fca1cp-4"),
     float.fromhex("0x1.497ea156fd1cep-1"), math.nan),
    (float.fromhex("0x1.fafdc82eeb650p-7"), float.fromhex("0x1.678f64b7b949dp-3"),
     math.nan, float.fromhex("0x1.64d0cc399bf28p+3")),
    (float.fromhex("0x1.3e4d683c0b176p-4"), float.fromhex("0x1.b16dba5381b9cp-4"),
     float.fromhex("0x1.ae7e9badb2252p+0"), math.nan),
    (float.fromhex("0x1.793a94312d8eap-6"), float.fromhex("0x1.55f53b6448c1bp-5"),
     float.fromhex("0x1.ef7b16a3870c2p+0"), math.nan),
    (float.fromhex("0x1.8e16c284b4885p-20"), float.fromhex("0x1.9d9a05656754dp-8"),
     float.fromhex("0x1.1e66761d9c6e4p+1"), math.nan),
)
SHAPE_IS_T = (0, 0, 1, 0, 0, 0)

# SAPM module parameter order used by the C-ABI (include/tmhpvsim.h, TMH_MOD_*)
MODULE_KEYS = ("A0", "A1", "A2", "A3", "A4", "B0", "B1", "B2", "B3", "B4", "B5", "FD",
               "Impo", "Vmpo", "Aimp", "C0", "C1", "C2", "C3", "Bvmpo", "Mbvmp", "N",
               "Cells_in_Series", "temp_a", "temp_b", "temp_deltaT")
MODULE_DEFAULT = dict(
    A0=0.9381, A1=0.05402, A2=-0.009848, A3=0.0008356, A4=-2.712e-05,
    B0=1.0, B1=-0.002438, B2=0.0003103, B3=-1.246e-05, B4=2.112e-07, B5=-1.359e-09,
    FD=1.0, Impo=8.1, Vmpo=30.6, Aimp=-0.0002, C0=1.0118, C1=-0.0118, C2=0.1, C3=-8.0,
    Bvmpo=-0.14, Mbvmp=0.0, N=1.1, Cells_in_Series=60.0,
    # sapm_celltemp 'open_rack_cell_glassback' (pvlib 0.6.3)
    temp_a=-3.47, temp_b=-0.0594, temp_deltaT=3.0,
)
INVERTER_KEYS = ("Paco", "Pdco", "Vdco", "Pso", "C0", "C1", "C2", "C3", "Pnt")
INVERTER_DEFAULT = dict(Paco=250.0, Pdco=259.522, Vdco=40.2426, Pso=1.7716, C0=-4.1e-05,
                        C1=-9.1e-05, C2=0.000494, C3=-0.013171, Pnt=0.075)
LINKE_DEFAULT = (3.2, 3.4, 3.9, 4.3, 4.6, 4.9, 5.0, 4.8, 4.3, 3.8, 3.4, 3.2)

CC_FAITHFUL = 0   # reference behaviour: fresh get_cloud_cover generator per hourly draw
CC_MARKOV = 1     # the hourly Markov chain get_cloud_cover describes (persistent state)
RNG_KEYED = 0     # counter-based Philox keyed by (chain, step, draw family)
RNG_INJECTED = 1  # per-chain uniform stream consumed in reference order


@dataclass
class Site:
    latitude: float = 48.12
    longitude: float = 11.60
    altitude: float = 34.0
    tilt: float = 48.12
    surface_azimuth: float = 180.0
    albedo: float = 0.25
    temp_air: float = 20.0
    wind_speed: float = 0.0
    tz: str = "Europe/Berlin"

    def as_array(self):
        return np.array([self.latitude, self.longitude, self.altitude, self.tilt,
                         self.surface_azimuth, self.albedo, self.temp_air, self.wind_speed])


@dataclass
class ModelParams:
    cc_mode: int = CC_FAITHFUL
    rng_mode: int = RNG_KEYED
    seed: int = 0x5EED
    with_pv: bool = True
    shapes: np.ndarray = field(default_factory=lambda: np.array(SHAPES, dtype=np.float64))
    shape_is_t: tuple = SHAPE_IS_T
    edges: tuple = EDGES
    site: Site = field(default_factory=Site)
    linke: tuple = LINKE_DEFAULT
    module: dict = field(default_factory=lambda: dict(MODULE_DEFAULT))
    inverter: dict = field(default_factory=lambda: dict(INVERTER_DEFAULT))

    def module_array(self):
        return np.array([self.module[k] for k in MODULE_KEYS], dtype=np.float64)

    def inverter_array(self):
        return np.array([self.inverter[k] for k in INVERTER_KEYS], dtype=np.float64)


def load_shapes_csv(path):
    """Load a shape table in the reference's mc_dist_shapes.csv format.

    Uses pandas' default parser exactly like cloud_cover_hourly.py:282-288 so
    the loaded bits equal the reference's.  Returns (shapes[6,4], is_t[6], edges[6]).
    """
    import pandas as pd
    df = pd.read_csv(path, index_col=[0, 1])
    shapes = np.full((len(df), 4), np.nan)
    is_t = np.zeros(len(df), dtype=np.int32)
    edges = np.array([iv[1] for iv in df.index], dtype=np.float64)
    for i, (_, row) in enumerate(df.iterrows()):
        shapes[i, 0], shapes[i, 1] = row["loc"], row["scale"]
        if row["dist"] == "t":
            is_t[i] = 1
            shapes[i, 3] = row["df"]
        elif row["dist"] == "al":
            shapes[i, 2] = row["kappa"]
        else:
            raise NotImplementedError(f"distribution {row['dist']!r} is not implemented")
    return shapes, is_t, edges


def save_shapes_csv(path, shapes, is_t, edges, lefts=None):
    """Write a shape table in the reference's mc_dist_shapes.csv format
    (cloud_cover_hourly.py:282-288 reads it: a two-level (left, right] interval
    index, then loc, scale, kappa, df, dist with 'al' / 't').  Values are written
    with Python's shortest round-trip repr; NaN cells stay empty.  `lefts`
    defaults to (-0.001, then the previous right edge)."""
    shapes = np.asarray(shapes, dtype=np.float64)
    edges = np.asarray(edges, dtype=np.float64)
    if lefts is None:
        lefts = np.concatenate([[-0.001], edges[:-1]])

    def cell(v):
        return "" if not np.isfinite(v) else repr(float(v))

    with open(path, "w") as f:
        f.write(",,loc,scale,kappa,df,dist\n")
        for i in range(len(edges)):
            t = bool(is_t[i])
            f.write(",".join([repr(float(lefts[i])), repr(float(edges[i])), cell(shapes[i, 0]), cell(shapes[i, 1]),
                              "" if t else cell(shapes[i, 2]), cell(shapes[i, 3]) if t else "",
                              "t" if t else "al"]) + "\n")


def save_site_tables(path, shapes, is_t):
    """Per-site shape tables ([n, 6, 4] fp64, [n, 6] int32) as an .npz (no pickles)."""
    np.savez(path, shapes=np.asarray(shapes, dtype=np.float64), is_t=np.asarray(is_t, dtype=np.int32))


def load_site_tables(path):
    d = np.load(path, allow_pickle=False)
    return d["shapes"], d["is_t"]


def _philox4x32_10(ctr, key):
    """Philox4x32-10 (Random123) on uint32 arrays ctr (..., 4), key (..., 2); host-side
    table generation only (the kernels' Philox is tmhpvsim_amd/csrc/tmh_math.h)."""
    M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
    c = [ctr[..., i].astype(np.uint32) for i in range(4)]
    k0, k1 = key[..., 0].astype(np.uint32), key[..., 1].astype(np.uint32)
    lo32 = np.uint64(0xFFFFFFFF)
    for r in range(10):
        p0 = c[0].astype(np.uint64) * M0
        p1 = c[2].astype(np.uint64) * M1
        c = [((p1 >> np.uint64(32)).astype(np.uint32) ^ c[1] ^ k0), (p1 & lo32).astype(np.uint32),
             ((p0 >> np.uint64(32)).astype(np.uint32) ^ c[3] ^ k1), (p0 & lo32).astype(np.uint32)]
        if r < 9:
            k0 = k0 + W0
            k1 = k1 + W1
    return np.stack(c, axis=-1)


def site_shape_tables(n_sites, site0=0, shapes=SHAPES, shape_is_t=SHAPE_IS_T, seed=0x7AB1E, spread=0.1):
    """Per-site hourly cloud-cover tables for a lat/lon sweep: every
    parameter of the mc_dist_shapes.csv table (cloud_cover_hourly.py:282-288)
    times U(1 - spread, 1 + spread), drawn per (site, entry) from Philox4x32-10
    keyed by (seed, global site id), so a site's table does not depend on how
    the sweep is partitioned.  Returns shapes [n, 6, 4] fp64 (NaN entries stay
    NaN) and is_t [n, 6] int32, ready for BatchedSim(shape_tables=...)."""
    sid = np.arange(site0, site0 + n_sites, dtype=np.uint64)
    ctr = np.zeros((n_sites, 6, 4), dtype=np.uint32)
    ctr[..., 0] = np.arange(6, dtype=np.uint32)[None, :]
    ctr[..., 1] = (sid >> np.uint64(32)).astype(np.uint32)[:, None]
    key = np.zeros((n_sites, 6, 2), dtype=np.uint32)
    key[..., 0] = np.uint32(seed & 0xFFFFFFFF)
    key[..., 1] = (sid & np.uint64(0xFFFFFFFF)).astype(np.uint32)[:, None]
    u = (_philox4x32_10(ctr, key).astype(np.float64) + 0.5) * 2.0 ** -32
    tab = np.asarray(shapes, dtype=np.float64)[None] * (1.0 - spread + 2.0 * spread * u)
    is_t = np.broadcast_to(np.asarray(shape_is_t, dtype=np.int32), (n_sites, 6)).copy()
    return np.ascontiguousarray(tab), is_t


def site_grid(n_lat=256, n_lon=256, lat=(35.0, 60.0), lon=(-10.0, 30.0), base: Site | None = None):
    """PV sites on a regular lat/lon grid (256 x 256 over 35-60 N,
    10 W-30 E), latitude-major: [n_lat * n_lon, 8] rows in tmh_params.site order.
    Every site is the reference's system (pvmodel.py:19-30) moved: tilt =
    latitude, facing south, the base site's altitude, albedo, air temperature
    and wind.  Ready for BatchedSim(sites=...) (slice rows for a chain range)."""
    b = base or Site()
    la = np.linspace(lat[0], lat[1], n_lat)
    lo = np.linspace(lon[0], lon[1], n_lon)
    g = np.empty((n_lat, n_lon, 8), dtype=np.float64)
    g[..., 0] = la[:, None]
    g[..., 1] = lo[None, :]
    g[..., 2] = b.altitude
    g[..., 3] = la[:, None]
    g[..., 4] = b.surface_azimuth
    g[..., 5] = b.albedo
    g[..., 6] = b.temp_air
    g[..., 7] = b.wind_speed
    return g.reshape(-1, 8)


def infer_shapes(cc, edges=EDGES, dists=("al", "al", "t", "al", "al", "al"), lag=1):
    """Fit a 6-bin shape table to an hourly total-cloud-cover series: the
    replacement for the reference's offline fitting (cloud_cover_hourly.py:110-190,
    pymc3 posterior means on ERA-5 data; pymc3 and the data are not available).
    Steps cc[t + lag] - cc[t] are grouped by the bin of cc[t] exactly as
    get_cloud_cover selects a bin (np.searchsorted(edges, state), :309-314) and
    fitted by maximum likelihood: the asymmetric Laplace of :93-104 is scipy's
    laplace_asymmetric (same density in kappa), Student-t is scipy's t.
    Returns (shapes [6, 4] (loc, scale, kappa, df), is_t [6]) for
    save_shapes_csv / ModelParams / site tables."""
    import scipy.stats

    cc = np.asarray(cc, dtype=np.float64)
    state, step = cc[:-lag], cc[lag:] - cc[:-lag]
    ok = np.isfinite(state) & np.isfinite(step)
    state, step = state[ok], step[ok]
    b = np.searchsorted(np.asarray(edges, dtype=np.float64), state, side="left")
    shapes = np.full((len(edges), 4), np.nan)
    is_t = np.zeros(len(edges), dtype=np.int32)
    for i, dist in enumerate(dists):
        x = step[b == i]
        if len(x) < 10:
            raise ValueError(f"bin {i} has {len(x)} steps: too few to fit")
        if dist == "al":
            kappa, loc, scale = scipy.stats.laplace_asymmetric.fit(x)
            shapes[i, :3] = loc, scale, kappa
        elif dist == "t":
            df, loc, scale = scipy.stats.t.fit(x)
            shapes[i, 0], shapes[i, 1], shapes[i, 3] = loc, scale, df
            is_t[i] = 1
        else:
            raise NotImplementedError(f"distribution {dist!r} is not implemented")
    return shapes, is_t
