"""Noise parity: the granular Laplace / Gaussian samplers (oracle restatement
of the kernels' samplers) against the reference's distribution tests
(tests/dp_computations_test.py:69-160, 461-483, 515-545): KS p > 1e-4 and the
1-sigma / 2-sigma probability masses, and "not all integers" (snapping)."""
import math

import numpy as np
from scipy import stats

from oracle import oracle

N = 30000


def _samples(kind, x, scale):
    return np.array([oracle.noise_sample(kind, x, scale, 12345, k, 0) for k in range(N)])


def _masses(values, mean, sigma, p1, p12):
    d = np.abs(values - mean)
    w1 = np.mean(d <= sigma)
    w12 = np.mean((d > sigma) & (d <= 2 * sigma))
    assert abs(w1 - p1) < 4 * math.sqrt(p1 * (1 - p1) / len(values))
    assert abs(w12 - p12) < 4 * math.sqrt(p12 * (1 - p12) / len(values))


def test_laplace_noise_distribution():
    b = 1.0 / 0.5  # l1 = 1, eps = 0.5
    v = _samples(1, 20.0, b)
    assert any(not float(x).is_integer() for x in v)
    assert stats.ks_1samp(v, stats.laplace(loc=20.0, scale=b).cdf).pvalue > 1e-4
    _masses(v, 20.0, math.sqrt(2) * b, 1 - math.exp(-math.sqrt(2)),
            math.exp(-math.sqrt(2)) - math.exp(-2 * math.sqrt(2)))


def test_gaussian_noise_distribution():
    sigma = 17.1826171875  # eps 2, delta 1e-15, l2 4.5 (reference golden)
    v = _samples(2, 0.0, sigma)
    assert any(not float(x).is_integer() for x in v)
    assert stats.ks_1samp(v, stats.norm(loc=0.0, scale=sigma).cdf).pvalue > 1e-4
    _masses(v, 0.0, sigma, 0.68268949213, 0.27181024396)


def test_noise_is_keyed_by_partition_and_slot():
    a = oracle.noise_sample(1, 0.0, 1.0, 7, 5, 0)
    assert a == oracle.noise_sample(1, 0.0, 1.0, 7, 5, 0)
    assert a != oracle.noise_sample(1, 0.0, 1.0, 7, 5, 1)
    assert a != oracle.noise_sample(1, 0.0, 1.0, 7, 6, 0)
    assert a != oracle.noise_sample(1, 0.0, 1.0, 8, 5, 0)


def test_philox_known_answer():
    # Random123 known-answer vector for philox4x32-10 (ctr = key = 0)
    assert oracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C,
                                                   0x9B00DBD8]
