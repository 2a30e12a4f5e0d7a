"""Scalar DP math of the hot path, restated for the oracle (TEST INFRASTRUCTURE).

Pinned by the reference's own known-answer tests:
  * analytic-Gaussian sigma: tests/dp_computations_test.py:62-67, 371-405,
    485-545 (114.375, 37.53742639189524, 18.662109375, 88.06640625,
    17.1826171875, 16.9125, 277.34375)  -- restates PyDP
    GaussianMechanism(eps, delta, l2).std used at dp_computations.py:107-117;
  * truncated-geometric keep probability: analysis/tests/
    per_partition_combiners_test.py:200-238 (0.12818308050524607,
    0.3321336253750503) -- restates PyDP NearTruncatedGeometric
    partition selection used at partition_selection.py:29-44.
Unpinned (no reference test): the l0 > 1 delta adjustment and the
Laplace / Gaussian thresholding thresholds (restated from the un-vendored
Google DP C++ library, python-dp==1.1.4).
"""
import math

SIGMA_ACCURACY = 1e-3


def _phi(x):
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def gaussian_delta(sigma, eps, l2):
    a = l2 / (2.0 * sigma)
    b = eps * sigma / l2
    return _phi(a - b) - math.exp(eps) * _phi(-a - b)


def gaussian_sigma(eps, delta, l2):
    """Smallest sigma (to 1e-3 relative) with gaussian_delta <= delta."""
    lo, hi = 0.0, float(l2)
    while gaussian_delta(hi, eps, l2) > delta:
        lo, hi = hi, hi * 2.0
    while hi - lo > SIGMA_ACCURACY * lo:
        mid = lo * 0.5 + hi * 0.5
        if gaussian_delta(mid, eps, l2) > delta:
            lo = mid
        else:
            hi = mid
    return hi


def adjusted_delta(delta, l0):
    return -math.expm1(math.log1p(-delta) / l0)


def truncated_geometric_table(eps, delta, l0, max_len=1 << 22):
    """pi(n) for n = 0.. until pi reaches 1 (the recursion of the optimal
    partition-selection mechanism)."""
    e = eps / l0
    d = adjusted_delta(delta, l0)
    ee, eme = math.exp(e), math.exp(-e)
    p = [0.0]
    while p[-1] < 1.0 and len(p) < max_len:
        q = p[-1]
        p.append(min(ee * q + d, 1.0 + eme * (q + d - 1.0), 1.0))
    return p


def laplace_threshold(eps, delta, l0):
    d = adjusted_delta(delta, l0)
    b = l0 / eps
    if d > 0.5:
        return 1.0 + b * math.log(2.0 * (1.0 - d)), b
    return 1.0 - b * math.log(2.0 * d), b


def _inv_norm_cdf(p):
    from scipy.stats import norm
    return float(norm.ppf(p))


def gaussian_threshold(eps, delta, l0):
    noise_delta = delta / 2.0
    thr_delta = delta - noise_delta
    sigma = gaussian_sigma(eps, noise_delta, math.sqrt(l0))
    d = adjusted_delta(thr_delta, l0)
    return 1.0 + sigma * _inv_norm_cdf(1.0 - d), sigma
