"""Scalar DP math evaluated on the host, once per aggregation.

Restates the parts of pipeline_dp/dp_computations.py that the device path
needs as *parameters*: sensitivities (:79-104, :579-619, :719-761), the
analytic-Gaussian sigma (:107-117, PyDP GaussianMechanism.std), Laplace
diversity b = l1/eps (:431-478), the mean / variance parameter plumbing
(:64-76, :233-261, :307-366) and the mechanism descriptions used by the
explain report.  Per-partition noise itself is drawn on the GPU
(csrc/dpg_select.h), never here.
"""
import abc
import dataclasses
import math
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np

from pipelinedp_amd import aggregate_params as agg

_SIGMA_ACCURACY = 1e-3  # relative accuracy of the sigma binary search


def compute_middle(min_value: float, max_value: float) -> float:
    return min_value + (max_value - min_value) / 2


def compute_squares_interval(min_value: float, max_value: float) -> Tuple[float, float]:
    if min_value < 0 < max_value:
        return 0, max(min_value**2, max_value**2)
    return min_value**2, max_value**2


def compute_l1_sensitivity(l0: float, linf: float) -> float:
    return l0 * linf


def compute_l2_sensitivity(l0: float, linf: float) -> float:
    return math.sqrt(l0) * linf


def _std_normal_cdf(x: float) -> float:
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def _gaussian_delta(sigma: float, eps: float, l2: float) -> float:
    """delta achieved by N(0, sigma^2) noise at (eps, l2) (analytic Gaussian
    mechanism, Balle & Wang 2018)."""
    a = l2 / (2.0 * sigma)
    b = eps * sigma / l2
    if eps < 700.0:
        return _std_normal_cdf(a - b) - math.exp(eps) * _std_normal_cdf(-a - b)
    # e^eps overflows a double: evaluate e^eps * Phi(-a-b) in the log domain
    from scipy.special import log_ndtr
    return _std_normal_cdf(a - b) - math.exp(min(700.0, eps + float(log_ndtr(-a - b))))


def compute_sigma(eps: float, delta: float, l2_sensitivity: float) -> float:
    """Smallest sigma, to 1e-3 relative, whose Gaussian noise is
    (eps, delta)-DP for L2 sensitivity l2 -- the search PyDP's
    GaussianMechanism performs (upper bound by doubling from l2, then
    bisection; the upper end is returned)."""
    if delta >= 1:
        return 0.0
    lo, hi = 0.0, float(l2_sensitivity)
    while _gaussian_delta(hi, eps, l2_sensitivity) > delta:
        lo, hi = hi, 2.0 * hi
    while hi - lo > _SIGMA_ACCURACY * lo:
        mid = 0.5 * lo + 0.5 * hi
        if _gaussian_delta(mid, eps, l2_sensitivity) > delta:
            lo = mid
        else:
            hi = mid
    return hi


def equally_split_budget(eps: float, delta: float, no_mechanisms: int) -> List[Tuple[float, float]]:
    """dp_computations.py:233-261: k-1 equal shares; the last one takes what
    is left so the shares sum to exactly (eps, delta)."""
    if no_mechanisms <= 0:
        raise ValueError("The number of mechanisms must be a positive integer.")
    shares, eps_used, delta_used = [], 0, 0
    for _ in range(no_mechanisms - 1):
        shares.append((eps / no_mechanisms, delta / no_mechanisms))
        eps_used += eps / no_mechanisms
        delta_used += delta / no_mechanisms
    shares.append((eps - eps_used, delta - delta_used))
    return shares


@dataclasses.dataclass
class Sensitivities:
    """dp_computations.py:579-619."""
    l0: Optional[int] = None
    linf: Optional[float] = None
    l1: Optional[float] = None
    l2: Optional[float] = None

    def __post_init__(self):
        for name in ("l0", "linf", "l1", "l2"):
            v = getattr(self, name)
            if v is not None and v <= 0:
                raise ValueError(f"{name.upper() if name != 'linf' else 'Linf'} "
                                 f"must be positive, but {v} given.")
        if (self.l0 is None) != (self.linf is None):
            raise ValueError("l0 and linf sensitivities must be either both set"
                             " or both unset.")
        if self.l0 is not None:
            l1 = compute_l1_sensitivity(self.l0, self.linf)
            l2 = compute_l2_sensitivity(self.l0, self.linf)
            if self.l1 is None:
                self.l1 = l1
            elif abs(l1 - self.l1) > 1e-12:
                raise ValueError(f"L1={self.l1} != L0*Linf={l1}")
            if self.l2 is None:
                self.l2 = l2
            elif abs(l2 - self.l2) > 1e-12:
                raise ValueError(f"L2={self.l2} != sqrt(L0)*Linf={l2}")


def sensitivities_for_count(p: agg.AggregateParams) -> Sensitivities:
    if p.max_contributions is not None:
        return Sensitivities(l1=p.max_contributions, l2=p.max_contributions)
    return Sensitivities(l0=p.max_partitions_contributed,
                         linf=p.max_contributions_per_partition)


def sensitivities_for_privacy_id_count(p: agg.AggregateParams) -> Sensitivities:
    if p.max_contributions is not None:
        return Sensitivities(l1=p.max_contributions, l2=math.sqrt(p.max_contributions))
    return Sensitivities(l0=p.max_partitions_contributed, linf=1)


def sensitivities_for_sum(p: agg.AggregateParams) -> Sensitivities:
    if p.bounds_per_contribution_are_set:
        max_abs = max(abs(p.min_value), abs(p.max_value))
        if p.max_contributions:
            s = max_abs * p.max_contributions
            return Sensitivities(l1=s, l2=s)
        linf = max_abs * p.max_contributions_per_partition
    else:
        linf = max(abs(p.min_sum_per_partition), abs(p.max_sum_per_partition))
    return Sensitivities(l0=p.max_partitions_contributed, linf=linf)


def sensitivities_for_normalized_sum(p: agg.AggregateParams) -> Sensitivities:
    half = (p.max_value - p.min_value) / 2
    if p.max_contributions:
        s = half * p.max_contributions
        return Sensitivities(l1=s, l2=s)
    return Sensitivities(l0=p.max_partitions_contributed,
                         linf=half * p.max_contributions_per_partition)


class AdditiveMechanism:
    """Laplace or Gaussian parameters of one metric (no sampling on the host)."""

    def __init__(self, noise_kind: agg.NoiseKind, eps: float, delta: float,
                 sensitivities: Sensitivities):
        self.noise_kind = noise_kind
        self.eps = eps
        self.delta = delta
        if noise_kind == agg.NoiseKind.LAPLACE:
            if sensitivities.l1 is None:
                raise ValueError("L1 or (L0 and Linf) sensitivities must be set for"
                                 " Laplace mechanism.")
            self.sensitivity = sensitivities.l1
            self.noise_parameter = self.sensitivity / eps  # diversity b
            self.std = self.noise_parameter * math.sqrt(2)
        else:
            if sensitivities.l2 is None:
                raise ValueError("L2 or (L0 and Linf) sensitivities must be set for"
                                 " Gaussian mechanism.")
            self.sensitivity = sensitivities.l2
            self.noise_parameter = compute_sigma(eps, delta, self.sensitivity)
            self.std = self.noise_parameter

    @property
    def scale(self) -> float:
        return self.noise_parameter

    def describe(self) -> str:
        if self.noise_kind == agg.NoiseKind.LAPLACE:
            return (f"Laplace mechanism:  parameter={self.noise_parameter}  eps="
                    f"{self.eps}  l1_sensitivity={self.sensitivity}")
        return (f"Gaussian mechanism:  parameter={self.noise_parameter}  "
                f"eps={self.eps}  delta={self.delta}  "
                f"l2_sensitivity={self.sensitivity}")


def noise_scale(noise_kind: agg.NoiseKind, eps: float, delta: float, l0: float,
                linf: float) -> float:
    """Scale used by dp_computations._add_random_noise (:155-184)."""
    if noise_kind == agg.NoiseKind.LAPLACE:
        return compute_l1_sensitivity(l0, linf) / eps
    return compute_sigma(eps, delta, compute_l2_sensitivity(l0, linf))


def compute_count_noise_std(noise_kind: agg.NoiseKind, eps: float, delta: float, l0: float,
                            linf: float) -> float:
    """Noise standard deviation of a COUNT with sensitivities (l0, linf)
    (dp_computations.py:369-388: Laplace b * sqrt(2), Gaussian sigma)."""
    if noise_kind == agg.NoiseKind.LAPLACE:
        return compute_l1_sensitivity(l0, linf) / eps * math.sqrt(2)
    return compute_sigma(eps, delta, compute_l2_sensitivity(l0, linf))


class ExponentialMechanism:
    """Chooses one of a list of candidates with probability proportional to
    exp(eps * score / (sensitivity, doubled unless the score is monotonic))
    (dp_computations.py:662-716).  The scores are host work over at most a
    few thousand candidates."""

    class ScoringFunction(abc.ABC):

        @abc.abstractmethod
        def score(self, k) -> float:
            """Higher is more likely."""

        @property
        @abc.abstractmethod
        def global_sensitivity(self) -> float:
            """Global sensitivity of the score."""

        @property
        @abc.abstractmethod
        def is_monotonic(self) -> bool:
            """Whether score(D, k) moves the same way for every k between
            neighbouring datasets."""

        def scores(self, candidates: Sequence) -> np.ndarray:
            """All scores at once (override for a vectorised form)."""
            return np.array([self.score(k) for k in candidates], dtype=np.float64)

    def __init__(self, scoring_function: "ExponentialMechanism.ScoringFunction"):
        self._scoring_function = scoring_function

    def apply(self, eps: float, inputs_to_score_col: List[Any]) -> Any:
        probs = self._calculate_probabilities(eps, inputs_to_score_col)
        return np.random.default_rng().choice(inputs_to_score_col, p=probs)

    def _calculate_probabilities(self, eps: float, inputs_to_score_col: List[Any]) -> np.ndarray:
        scores = self._scoring_function.scores(inputs_to_score_col)
        denominator = self._scoring_function.global_sensitivity
        if not self._scoring_function.is_monotonic:
            denominator *= 2
        # shifted by the best score: the same distribution as the reference's
        # exp(score * eps / d) / sum, without the 0 / 0 it hits when every
        # weight underflows (very negative scores)
        z = scores * eps / denominator
        weights = np.exp(z - z.max())
        return weights / weights.sum()
