"""Differentially private choice of max_partitions_contributed (API mirror of
pipeline_dp/private_contribution_bounds.py).

The data-dependent part is the L0 contribution histogram, computed on the
device (dataset_histograms/computing_histograms.py).  Scoring the candidate
bounds against its bins and drawing from the exponential mechanism is host
work over at most a few thousand candidates x bins, done vectorised.
"""
import dataclasses
from typing import List

import numpy as np
import torch

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import dp_computations as dpc
from pipelinedp_amd.dataset_histograms import histograms as hist


def generate_possible_contribution_bounds(upper_bound: int) -> List[int]:
    """1, 2, ..., 999, 1000, 1010, ..., 9990, 10000, 10100, ... up to
    upper_bound: numbers with at most 3 non-zero leading digits, the lowers
    of the integer histogram bins (private_contribution_bounds.py:179-196)."""
    bounds = []
    cur, power = 1, 10
    while cur <= upper_bound:
        bounds.append(cur)
        if cur >= power:
            power *= 10
        cur += max(1, power // 1000)
    return bounds


class L0ScoringFunction(dpc.ExponentialMechanism.ScoringFunction):
    """score(k) = -(P * count_noise_std(k) + sum over privacy ids of
    max(min(#partitions, B) - k, 0)) / 2 (private_contribution_bounds.py
    :90-176), B = min(upper bound, P)."""

    def __init__(self, params: agg.CalculatePrivateContributionBoundsParams,
                 number_of_partitions: int, l0_histogram: hist.Histogram):
        super().__init__()
        self._params = params
        self._number_of_partitions = number_of_partitions
        self._l0_histogram = l0_histogram
        self._lowers = np.array([b.lower for b in l0_histogram.bins], dtype=np.float64)
        self._counts = np.array([b.count for b in l0_histogram.bins], dtype=np.float64)

    def _max_partitions_contributed_best_upper_bound(self) -> int:
        return min(self._params.max_partitions_contributed_upper_bound, self._number_of_partitions)

    @property
    def global_sensitivity(self) -> float:
        return self._max_partitions_contributed_best_upper_bound()

    @property
    def is_monotonic(self) -> bool:
        return True

    def _l0_impact_noise(self, k: int) -> float:
        p = self._params
        return self._number_of_partitions * dpc.compute_count_noise_std(
            p.aggregation_noise_kind, p.aggregation_eps, p.aggregation_delta, k, 1)

    def _l0_impact_dropped(self, k) -> np.ndarray:
        capped = np.minimum(self._lowers, self._max_partitions_contributed_best_upper_bound())
        k = np.asarray(k, dtype=np.float64).reshape(-1, 1)
        return (np.maximum(capped[None, :] - k, 0.0) * self._counts[None, :]).sum(axis=1)

    def score(self, k: int) -> float:
        return float(self.scores([k])[0])

    def scores(self, candidates) -> np.ndarray:
        noise = np.array([self._l0_impact_noise(int(k)) for k in candidates], dtype=np.float64)
        return -(0.5 * noise + 0.5 * self._l0_impact_dropped(candidates))


class PrivateL0Calculator:
    """Chooses max_partitions_contributed with the exponential mechanism
    (private_contribution_bounds.py:27-87)."""

    @dataclasses.dataclass
    class Inputs:
        l0_histogram: hist.Histogram
        number_of_partitions: int

    def __init__(self, params: agg.CalculatePrivateContributionBoundsParams, partitions,
                 histograms, backend) -> None:
        self._params = params
        self._backend = backend
        self._partitions = partitions
        self._histograms = histograms
        self._result = None

    def _number_of_partitions(self) -> int:
        """Distinct partition keys (the reference's len(set(...)) of
        hashable keys): tensors and arrays are counted by value, not by
        element object identity, without a device sync per element."""
        p = self._partitions
        if isinstance(p, torch.Tensor):
            return int(torch.unique(p).numel())
        if isinstance(p, np.ndarray):
            return int(np.unique(p).size)
        if isinstance(p, range):
            return len(p)
        return len(set(p))

    def _calculate_l0(self, inputs: "PrivateL0Calculator.Inputs") -> int:
        scoring = L0ScoringFunction(self._params, inputs.number_of_partitions,
                                    inputs.l0_histogram)
        candidates = generate_possible_contribution_bounds(
            scoring._max_partitions_contributed_best_upper_bound())
        return int(dpc.ExponentialMechanism(scoring).apply(self._params.calculation_eps,
                                                           candidates))

    def calculate(self):
        """1-element collection with the chosen bound."""
        if self._result is None:
            (h,) = list(self._histograms)
            self._result = [self._calculate_l0(
                PrivateL0Calculator.Inputs(h.l0_contributions_histogram,
                                           self._number_of_partitions()))]
        return self._result
