"""cquantile(Poisson(lambda), p) as used by smart_forward_moves!
(src/model.jl:661).

Distributions 0.19.2 -> StatsFuns 0.8.0 -> Rmath 0.5.0
`qpois(p, lambda, lower_tail=false, log_p=false)` (R's nmath/qpois.c): a
Cornish-Fisher start followed by a unit-step search for the smallest integer
y with ppois(y, lambda) >= (1 - p) * (1 - 64 * DBL_EPSILON).  ppois is the
regularised upper incomplete gamma Q(y + 1, lambda) (scipy.special.pdtr);
scipy's and Rmath's last bits may differ, which can only matter when
ppois(y) lies within ~1e-15 of the target (documented as weakly pinned).
"""
from __future__ import annotations

import math
import sys

from scipy.special import ndtri, pdtr

DBL_EPSILON = sys.float_info.epsilon


def _ppois(y: float, lam: float) -> float:
    return float(pdtr(y, lam))


def cquantile_poisson(lam: float, p: float) -> float:
    if not math.isfinite(lam) or lam < 0:
        return math.nan
    if lam == 0:
        return 0.0
    target = 0.5 - p + 0.5                       # R_DT_qIv(p), upper tail
    if target == 0.0:
        return 0.0
    if target == 1.0:
        return math.inf
    if target + 1.01 * DBL_EPSILON >= 1.0:
        return math.inf
    mu, sigma = lam, math.sqrt(lam)
    gamma = 1.0 / sigma
    z = float(ndtri(target))
    y = float(round(mu + sigma * (z + gamma * (z * z - 1) / 6)))   # R_forceint (nearbyint)
    y = max(y, 0.0)
    zz = _ppois(y, lam)
    pp = target * (1 - 64 * DBL_EPSILON)
    if zz >= pp:                                 # search to the left
        while True:
            if y == 0:
                return y
            zz = _ppois(y - 1, lam)
            if zz < pp:
                return y
            y = max(0.0, y - 1)
    while True:                                  # search to the right
        y = y + 1
        if _ppois(y, lam) >= pp:
            return y


def cquantile_poisson_many(lams, p: float):
    """cquantile_poisson over an array of lambdas: the same Cornish-Fisher
    start and unit-step search, element by element with the same FP64
    operations (numpy / scipy ufuncs evaluate each element exactly as the
    scalar calls do), so every threshold equals cquantile_poisson(lam, p)."""
    import numpy as np
    lams = np.asarray(lams, np.float64)
    target = 0.5 - p + 0.5
    ok = np.isfinite(lams) & (lams > 0)
    if target in (0.0, 1.0) or target + 1.01 * DBL_EPSILON >= 1.0 or not ok.all():
        return np.array([cquantile_poisson(float(x), p) for x in lams])
    mu, sigma = lams, np.sqrt(lams)
    gamma = 1.0 / sigma
    z = float(ndtri(target))
    y = np.maximum(np.rint(mu + sigma * (z + gamma * (z * z - 1) / 6)), 0.0)
    pp = target * (1 - 64 * DBL_EPSILON)
    zz = pdtr(y, lams)
    out = np.empty_like(y)
    left = zz >= pp
    # search to the left: the smallest y with ppois(y) >= pp
    idx = np.nonzero(left)[0]
    yl = y[idx]
    while idx.size:
        at0 = yl == 0
        out[idx[at0]] = 0.0
        idx, yl = idx[~at0], yl[~at0]
        if not idx.size:
            break
        zl = pdtr(yl - 1, lams[idx])
        done = zl < pp
        out[idx[done]] = yl[done]
        idx, yl = idx[~done], np.maximum(0.0, yl[~done] - 1)
    # search to the right
    idx = np.nonzero(~left)[0]
    yr = y[idx]
    while idx.size:
        yr = yr + 1
        done = pdtr(yr, lams[idx]) >= pp
        out[idx[done]] = yr[done]
        idx, yr = idx[~done], yr[~done]
    return out
