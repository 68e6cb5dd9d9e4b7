"""TEST INFRASTRUCTURE ONLY — injected-uniform harness around the imported reference.

Runs only in the build container, where the read-only reference checkout lives
at /root/reference (it never travels to the GPU box).  It generates the golden
fixtures committed under tests/golden/ (driver: tests/golden/make_golden.py).

Recipe:
1. Stub the offline-fitting-only modules imported at
   tmhpvsim/cloud_cover_hourly.py:25-32 (pymc3, theano, xarray, seaborn,
   cdsapi); nothing on the sampling path uses them.
2. Replace every random source the hot path touches by one object `R` that
   maps ONE injected uniform to ONE variate by inverse CDF:
     uniform / random           -> u
     standard_normal            -> scipy.special.ndtri(u)
     standard_gamma(a)          -> scipy.special.gammaincinv(a, u)
     standard_t(df)             -> scipy.special.stdtrit(df, u)
     np.random.gamma(k, theta)  -> theta * gammaincinv(k, u)
   Sources patched: np.random.random / np.random.gamma (cloud_cover_binary.py:23,40),
   scipy.stats.norm / gamma module instances (clearskyindexmodel.py:65,71,82,88,147)
   and every frozen distribution returned by get_distributions_from_shapes_file
   (cloud_cover_hourly.py:278-288, drawn at :315).
3. Drive ClearskyindexModel(t0) then .next(t) for consecutive seconds and log
   per-step CSI, covered bit, stream position, every next_cloud call and every
   sampler push.

Nothing here is imported by the product package.
"""
from __future__ import annotations

import sys
import types
from dataclasses import dataclass, field

import numpy as np

REFERENCE_PATH = "/root/reference"
_STUBS = ["pymc3", "theano", "theano.tensor", "xarray", "seaborn", "cdsapi"]


def import_reference():
    """Import the reference package with the offline-only modules stubbed."""
    sys.dont_write_bytecode = True
    for name in _STUBS:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["theano"].tensor = sys.modules["theano.tensor"]
    if REFERENCE_PATH not in sys.path:
        sys.path.insert(0, REFERENCE_PATH)
    import tmhpvsim.clearskyindexmodel as csm  # noqa: F401
    import tmhpvsim.cloud_cover_binary as ccb  # noqa: F401
    import tmhpvsim.cloud_cover_hourly as cch  # noqa: F401
    return csm, ccb, cch


class StreamExhausted(Exception):
    pass


class InjectedRandomState:
    """One injected uniform -> one variate (inverse CDF)."""

    def __init__(self, u):
        from scipy import special
        self._sp = special
        self.u = np.asarray(u, dtype=np.float64)
        self.pos = 0
        self.kinds: list[str] = []

    def _take(self, kind):
        if self.pos >= self.u.size:
            raise StreamExhausted(kind)
        v = self.u[self.pos]
        self.pos += 1
        self.kinds.append(kind)
        return v

    @staticmethod
    def _shape(v, size):
        if size is None:
            return float(v)
        if size == ():
            return np.array(v)
        return np.full(size, v)

    def _draw(self, size, kind, fn):
        n = 1 if size in (None, ()) else int(np.prod(size))
        if n != 1:
            vals = np.array([fn(self._take(kind)) for _ in range(n)]).reshape(size)
            return vals
        return self._shape(fn(self._take(kind)), size)

    # numpy.random.RandomState surface used by scipy's _rvs implementations
    def uniform(self, low=0.0, high=1.0, size=None):
        assert low == 0.0 and high == 1.0
        return self._draw(size, "uniform", lambda u: u)

    def random_sample(self, size=None):
        return self._draw(size, "random", lambda u: u)

    random = random_sample

    def standard_normal(self, size=None):
        return self._draw(size, "normal", lambda u: self._sp.ndtri(u))

    def standard_gamma(self, shape, size=None):
        return self._draw(size, "gamma", lambda u: self._sp.gammaincinv(shape, u))

    def standard_t(self, df, size=None):
        return self._draw(size, "t", lambda u: self._sp.stdtrit(df, u))

    def gamma(self, shape, scale=1.0, size=None):
        return self._draw(size, "np.gamma", lambda u: scale * self._sp.gammaincinv(shape, u))


@dataclass
class ChainLog:
    csi: list = field(default_factory=list)
    covered: list = field(default_factory=list)
    sec: list = field(default_factory=list)
    pos: list = field(default_factory=list)
    calls: list = field(default_factory=list)      # next_cloud outer calls
    pushes: list = field(default_factory=list)     # (step, sampler id, after value)
    init: dict = field(default_factory=dict)
    error: str = ""
    error_step: int = -2


SAMPLERS = ["cloudcover_hour", "clearskyindex_clear_day", "clearskyindex_cloudy_hour",
            "clearskyindex_cloudy_noise_min", "clearskyindex_clear_noise_min", "windspeed_day"]


class Harness:
    """Patches the imported reference once; `run_chain` drives one chain."""

    def __init__(self):
        self.csm, self.ccb, self.cch = import_reference()
        import scipy.stats
        self._stats = scipy.stats
        self._orig_get_dists = self.cch.get_distributions_from_shapes_file
        self._orig_get_cloud_cover = self.cch.get_cloud_cover
        self._orig_next_cloud = self.ccb.CloudCoverBinary.next_cloud
        self._orig_sampler_next = self.csm.InterpolatedSampler.__next__
        self._sampler_ids: dict = {}
        self.R: InjectedRandomState | None = None
        self.log: ChainLog | None = None
        self.step = -1
        self._depth = 0
        self._persistent = None
        self.markov = False
        self._install()

    def _install(self):
        h = self
        np.random.random = lambda shape=None: h.R.random_sample(shape)
        np.random.gamma = lambda k, theta=1.0, size=None: h.R.gamma(k, theta, size)

        def get_dists(dist_shapes_file=None):
            d = h._orig_get_dists(dist_shapes_file)
            for frozen in d.values:
                frozen.dist._random_state = h.R
            return d
        self.csm.get_distributions_from_shapes_file = get_dists

        def get_cloud_cover(distributions, initial_state=1.):
            if not h.markov:
                return h._orig_get_cloud_cover(distributions, initial_state)
            if h._persistent is None:   # markov mode: ONE generator per chain
                h._persistent = h._orig_get_cloud_cover(distributions, initial_state)
            return h._persistent
        self.csm.get_cloud_cover = get_cloud_cover

        def next_cloud(obj, recurse=False):
            outer = h._depth == 0
            h._depth += 1
            pos0 = h.R.pos
            L0 = len(obj.sigma_cloud)
            hh, ws = float(obj.hourly_cloudcover), float(obj.windspeed)
            try:
                res = h._orig_next_cloud(obj, recurse)
            finally:
                h._depth -= 1
            if outer and h.log is not None:
                h.log.calls.append((h.step, pos0, h.R.pos, hh, ws, L0,
                                    float(np.asarray(obj.cloud_length).reshape(-1)[0]),
                                    float(np.asarray(obj.clear_length).reshape(-1)[0]),
                                    len(obj.sigma_cloud)))
            return res
        self.ccb.CloudCoverBinary.next_cloud = next_cloud

        def sampler_next(obj):
            r = h._orig_sampler_next(obj)
            k = h._sampler_ids.get(id(obj))
            if k is not None and h.log is not None:
                h.log.pushes.append((h.step, k, float(obj.after)))
            return r
        self.csm.InterpolatedSampler.__next__ = sampler_next

    def _bind(self, u, markov):
        self.R = InjectedRandomState(u)
        self._stats.norm._random_state = self.R
        self._stats.gamma._random_state = self.R
        self._stats.t._random_state = self.R
        self.markov = markov
        self._persistent = None

    def run_chain(self, times, u, markov=False) -> ChainLog:
        self._bind(u, markov)
        log = ChainLog()
        self.log = log
        self.step = -1
        try:
            model = self.csm.ClearskyindexModel(times[0])
        except (NameError, AssertionError, StreamExhausted) as e:
            log.error, log.error_step = type(e).__name__, -1
            log.pos.append(self.R.pos)
            return log
        b = model.cloudcover_binary
        log.init = {
            "samplers": np.array([[getattr(model, s).before, getattr(model, s).after]
                                  for s in SAMPLERS], dtype=np.float64),
            "sec": int(b.sec),
            "cloud_length": float(np.asarray(b.cloud_length).reshape(-1)[0]),
            "clear_length": float(np.asarray(b.clear_length).reshape(-1)[0]),
            "sigma_cloud": np.asarray(b.sigma_cloud, dtype=np.float64).copy(),
            "sigma_clear": np.asarray(b.sigma_clear, dtype=np.float64).copy(),
            "pos": self.R.pos,
        }
        self._sampler_ids = {id(getattr(model, s)): k for k, s in enumerate(SAMPLERS)}
        for i, t in enumerate(times):
            self.step = i
            try:
                csi = model.next(t)
            except (NameError, AssertionError, StreamExhausted) as e:
                log.error, log.error_step = type(e).__name__, i
                break
            log.csi.append(float(csi))
            log.covered.append(int(b.sec < np.asarray(b.cloud_length).reshape(-1)[0]))
            log.sec.append(int(b.sec))
            log.pos.append(self.R.pos)
        self.log = None
        self._sampler_ids = {}
        return log

    # -- function-level references -------------------------------------------------
    def distributions(self):
        """Loaded shape table: (6, 5) = loc, scale, kappa|nan, df|nan, is_t."""
        d = self._orig_get_dists()
        rows = []
        for frozen in d.values:
            kw = frozen.kwds
            is_t = frozen.dist.name == "t"
            rows.append([kw["loc"], kw["scale"], np.nan if is_t else kw["kappa"],
                         kw["df"] if is_t else np.nan, float(is_t)])
        edges = np.array([iv.right for iv in d.index], dtype=np.float64)
        return np.array(rows, dtype=np.float64), edges

    def al_ppf(self, u, kappa):
        return self.cch.asymmetric_laplace._ppf(np.asarray(u, dtype=np.float64), kappa)

    def cloudlength(self, ws, u):
        self._bind(np.asarray(u, dtype=np.float64), False)
        return np.array([self.ccb.random_cloudlength_in_s(w)[0] for w in ws])

    def cloud_cover_chain(self, u, n_hours):
        """Standalone hourly Markov chain get_cloud_cover (cloud_cover_hourly.py:290-316)."""
        self._bind(u, False)
        d = self.csm.get_distributions_from_shapes_file()
        gen = self._orig_get_cloud_cover(d)
        out = []
        try:
            for _ in range(n_hours):
                out.append(float(next(gen)))
        except StreamExhausted:
            pass
        return np.array(out), self.R.pos
