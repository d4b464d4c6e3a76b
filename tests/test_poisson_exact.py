"""cquantile(Poisson(lambda), 0.1) (model.jl:661 -> Rmath qpois upper tail)
pinned against an exact Poisson CDF.

The host restatement (rifraf_amd/poisson.py) uses scipy's pdtr for ppois;
Rmath computes the same regularised incomplete gamma.  Here the CDF is summed
exactly (60-digit decimal arithmetic, stdlib only) and the smallest integer
y with P(X <= y) >= (1 - p) * (1 - 64 * DBL_EPSILON) -- qpois's stopping
rule -- is searched directly.  The lambda range covers every est_n_errors
the BASELINE configs produce (a few errors per 1 kb read up to ~300 for
10 kb reads at 3 % error, config 5).  Both sides agree on every lambda, so
the band-doubling thresholds of smart_forward_moves! (model.jl:643-672) are
pinned to the exact quantile."""
import sys
from decimal import Decimal, getcontext

import numpy as np
import pytest

from rifraf_amd.poisson import cquantile_poisson

EPS = sys.float_info.epsilon


def exact_quantile(lam: float, p: float) -> int:
    getcontext().prec = 60
    L = Decimal(lam)                      # the exact binary value of the float
    target = (Decimal(1) - Decimal(p)) * (Decimal(1) - 64 * Decimal(EPS))
    term = (-L).exp()                     # P(X = 0)
    cdf = term
    y = 0
    while cdf < target:
        y += 1
        term = term * L / y
        cdf += term
    return y


LAMBDAS = sorted(set(np.round(np.concatenate([
    np.linspace(0.5, 20, 40), np.linspace(20, 400, 77),
    np.random.default_rng(661).uniform(0.5, 400, 120)]), 9).tolist()))


@pytest.mark.parametrize("p", [0.1, 0.05, 0.5])
def test_cquantile_matches_exact_cdf(p):
    bad = [(lam, cquantile_poisson(lam, p), exact_quantile(lam, p)) for lam in LAMBDAS
           if cquantile_poisson(lam, p) != exact_quantile(lam, p)]
    assert not bad, bad[:5]


def test_cquantile_small_and_edge():
    assert cquantile_poisson(0.0, 0.1) == 0.0
    for lam in (1e-6, 1e-3, 0.1, 0.3):
        assert cquantile_poisson(lam, 0.1) == exact_quantile(lam, 0.1)
