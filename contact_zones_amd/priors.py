"""Priors of the batched sampler (host side): which prior terms are supported, their parameters for
the kernel (sbz_set_priors), and the full log prior of chain states.

Supported — every other prior type raises NotImplementedError:
  area_size   'none' (0), 'uniform' (-sum log C(N, size)), 'quadratic' (-sum log size^2)
              (ZoneSizePrior, sbayes/model.py:893-976)
  geo         'uniform' (0)                      (GeoPrior, model.py:979-1139)
  weights     'uniform' (0)                      (WeightsPrior, model.py:840-890)
  universal   'uniform' (0) or 'counts'          (PGlobalPrior, model.py:571-629)
  contact     'uniform' (0)                      (PZonesPrior, model.py:771-838)
  inheritance 'uniform' (0) or 'counts'          (PFamiliesPrior, model.py:631-769)
A 'counts' prior is a Dirichlet on each feature's applicable states with the concentrations the
reference derives from the counts files (util.counts_to_dirichlet / inheritance_counts_to_dirichlet,
util.py:547-626); they are passed scattered to [F][S] / [Fam][F][S] (0 at inapplicable states).

``log_prior`` restates Prior.__call__ (model.py:484-505) for these types, vectorised over chains,
in the reference's order of operations: the value equals the reference's for the same sample.
"""
import numpy as np
from scipy.special import betaln, gammaln, xlogy

SIZE_PRIORS = {"none": 0, "uniform": 1, "quadratic": 2}


def _type(obj):
    t = getattr(obj, "prior_type", None)
    return getattr(t, "value", t)


class PriorSpec:
    """The prior terms of the MH ratio (defaults: all zero)."""

    def __init__(self, alpha_global=None, alpha_fam=None, size_prior="none", geo_cost=None,
                 geo_scale=None):
        self.alpha_global = None if alpha_global is None else np.ascontiguousarray(alpha_global, np.float64)
        self.alpha_fam = None if alpha_fam is None else np.ascontiguousarray(alpha_fam, np.float64)
        if isinstance(size_prior, str):
            if size_prior not in SIZE_PRIORS:
                raise NotImplementedError(f"zone-size prior '{size_prior}' (supported: {list(SIZE_PRIORS)})")
            size_prior = SIZE_PRIORS[size_prior]
        if size_prior not in (0, 1, 2):
            raise ValueError(f"size_prior must be 0, 1 or 2, got {size_prior}")
        self.size_prior = int(size_prior)
        # 'cost_based' geo prior (GeoPrior, model.py:979-1139): cost matrix [N][N] and scale
        self.geo_cost = None if geo_cost is None else np.ascontiguousarray(geo_cost, np.float64)
        self.geo_scale = None if geo_cost is None else float(geo_scale)

    @property
    def is_zero(self):
        return (self.alpha_global is None and self.alpha_fam is None and self.size_prior == 0
                and self.geo_cost is None)

    @classmethod
    def from_model(cls, model, states):
        """From a reference ``Model`` (its ``prior``: Prior, model.py:455-482) or anything with the
        same attributes; a model without a ``prior`` attribute has zero priors.  ``states`` is the
        [F][S] applicable-state mask (data.states)."""
        prior = getattr(model, "prior", None)
        if prior is None:
            return cls()
        states = np.asarray(states, bool)
        F, S = states.shape
        geo = getattr(prior, "geo_prior", None)
        geo_cost = geo_scale = None
        if _type(geo) == "cost_based":
            geo_cost, geo_scale = geo.cost_matrix, geo.scale
        for name, ok in (("geo_prior", ("uniform", "cost_based")), ("prior_weights", ("uniform",)),
                         ("prior_p_zones", ("uniform",))):
            t = _type(getattr(prior, name, None))
            if t is not None and t not in ok:
                raise NotImplementedError(f"{name} of type '{t}' is not supported by the batched sampler")
        size = _type(getattr(prior, "size_prior", None)) or "none"
        ag = af = None
        pg = getattr(prior, "prior_p_global", None)
        t = _type(pg)
        if t == "counts":
            ag = np.zeros((F, S))
            for f in range(F):
                ag[f, states[f]] = pg.dirichlet[f]
        elif t not in (None, "uniform"):
            raise NotImplementedError(f"universal prior of type '{t}' is not supported")
        if getattr(model, "inheritance", False):
            pf = getattr(prior, "prior_p_families", None)
            t = _type(pf)
            if t == "counts":
                n_fam = len(pf.dirichlet)
                af = np.zeros((n_fam, F, S))
                for fam in range(n_fam):
                    for f in range(F):
                        af[fam, f, states[f]] = pf.dirichlet[fam][f]
            elif t not in (None, "uniform"):
                raise NotImplementedError(f"inheritance prior of type '{t}' is not supported")
        return cls(ag, af, size, geo_cost, geo_scale)

    def log_prior(self, zone_of_site, p_global, p_fam, states, n_zones, inheritance):
        """Log prior of B chain states: zone_of_site [B][N] (255 = none), p_global [B][F][S],
        p_fam [B][Fam][F][S] or None -> float64 [B]."""
        zos = np.asarray(zone_of_site)
        B, N = zos.shape
        states = np.asarray(states, bool)
        out = np.zeros(B)
        sizes = np.stack([np.count_nonzero(zos == z, axis=1) for z in range(n_zones)], axis=1) \
            if n_zones else np.zeros((B, 0), np.int64)
        if self.size_prior == 1:   # -np.sum(log_binom(n_sites, sizes)), util.py:1217
            out = out + (-np.sum(-betaln(1 + N - sizes, 1 + sizes) - np.log(N + 1), axis=1))
        elif self.size_prior == 2:
            out = out + (-np.sum(np.log(sizes ** 2), axis=1))
        else:
            out = out + 0.
        if self.geo_cost is not None and n_zones:
            out = out + np.array([geo_prior_distance(zos[b] == n_zones - 1, self.geo_cost, self.geo_scale)
                                  for b in range(B)])
        else:
            out = out + 0.  # geo
        out = out + 0.  # weights
        if self.alpha_global is not None:
            pg = np.asarray(p_global, np.float64).reshape(B, states.shape[0], states.shape[1])
            out = out + np.sum(_dirichlet_logpdf_rows(pg, self.alpha_global, states), axis=1)
        else:
            out = out + 0
        out = out + 0.  # p_zones
        if inheritance:
            if self.alpha_fam is not None:
                pf = np.asarray(p_fam, np.float64)
                n_fam = pf.shape[1]
                lp = np.stack([_dirichlet_logpdf_rows(pf[:, fam], self.alpha_fam[fam], states)
                               for fam in range(n_fam)], axis=1)  # [B][Fam][F]
                out = out + np.sum(lp.reshape(B, -1), axis=1)
            else:
                out = out + 0.
        return out


def _dirichlet_logpdf_rows(p, alpha, states):
    """scipy.stats.dirichlet._logpdf(p[b, f, states[f]], alpha[f, states[f]]) -> [B][F]:
    -(sum gammaln(a) - gammaln(sum a)) + sum xlogy(a - 1, x)."""
    B, F, _ = p.shape
    out = np.empty((B, F))
    for f in range(F):
        idx = np.flatnonzero(states[f])
        a = alpha[f, idx]
        lnB = np.sum(gammaln(a)) - gammaln(np.sum(a))
        out[:, f] = -lnB + np.sum(xlogy(a - 1, p[:, f, idx]), axis=1)
    return out


def geo_prior_distance(zone, cost, scale):
    """GeoPrior 'cost_based' (model.py:1096-1139) as the reference evaluates it: the log density of
    an exponential(scale) at every edge of the minimum spanning tree of the zone's cost matrix
    (scipy csgraph, zero-cost edges leave the sparse tree), averaged.  The reference's zone loop
    overwrites the value, so only the LAST zone counts; callers pass that zone's mask."""
    from scipy import stats
    from scipy.sparse.csgraph import csgraph_from_dense, minimum_spanning_tree
    zone = np.asarray(zone, bool)
    cz = np.asarray(cost)[zone][:, zone]
    if cz.shape[0] <= 1:
        raise ValueError("Too few locations to compute distance.")
    mst = minimum_spanning_tree(csgraph_from_dense(cz, null_value=np.inf))
    distances = mst.tocsr()[mst.nonzero()] if mst.nnz > 0 else 0
    return float(np.mean(stats.expon.logpdf(distances, loc=0, scale=scale)))
