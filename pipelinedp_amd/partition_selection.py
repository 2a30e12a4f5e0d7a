"""Private partition selection, tabulated on the host for the GPU kernel.

The reference maps its enum to a PyDP strategy object created per partition
(pipeline_dp/partition_selection.py:19-44, dp_engine.py:345-348) and calls
`should_keep(n)`.  Here each strategy is reduced once per aggregation to
the handful of numbers the selection kernel (csrc/dpg_select.h) needs:

* TRUNCATED_GEOMETRIC: the keep-probability table pi(n), n = 0.. until it
  reaches 1, from the recursion of the optimal partition-selection
  mechanism (Desfontaines et al., "Differentially private partition
  selection"):  pi(0)=0,
      pi(n) = min(e^eps' pi(n-1) + delta', 1 + e^-eps' (pi(n-1) + delta' - 1), 1)
  with eps' = eps / l0 and delta' = 1 - (1 - delta)^(1/l0).  Pinned for
  l0 = 1 by analysis/tests/per_partition_combiners_test.py:200-238.
* LAPLACE_THRESHOLDING: keep iff n + Lap(l0/eps) > 1 - (l0/eps) ln(2 delta').
* GAUSSIAN_THRESHOLDING: half of delta for the noise, half for the
  threshold: sigma = sigma(eps, delta/2, sqrt(l0)) and keep iff
  n + N(0, sigma^2) > 1 + sigma * Phi^-1(1 - delta'') with delta'' the
  l0-adjusted delta/2.
The l0 > 1 adjustment and both thresholds restate the un-vendored Google DP
library behind PyDP (python-dp==1.1.4); no reference test pins them
("parity unpinned" for those strategies).
`pre_threshold`: n < pre -> drop, else evaluate at n - pre + 1 (pinned:
n = 12, pre = 3 behaves as n = 10 in the same test).
"""
import dataclasses
import functools
import math
from typing import Optional

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import dp_computations

_MAX_TABLE = 1 << 22


def adjusted_delta(delta: float, l0: int) -> float:
    """Per-partition delta such that 1 - (1 - delta')^l0 = delta."""
    return -math.expm1(math.log1p(-delta) / l0)


@functools.lru_cache(maxsize=64)
def truncated_geometric_table(eps: float, delta: float, l0: int) -> tuple:
    """pi(0..) until it reaches 1 (cached: a sweep asks for the same (eps,
    delta, l0) many times)."""
    e = eps / l0
    d = adjusted_delta(delta, l0)
    grow, shrink = math.exp(e), math.exp(-e)
    table = [0.0]
    while table[-1] < 1.0 and len(table) < _MAX_TABLE:
        q = table[-1]
        table.append(min(grow * q + d, 1.0 + shrink * (q + d - 1.0), 1.0))
    if table[-1] < 1.0:
        # the kernel keeps every partition with n >= len(table): refuse rather
        # than keep partitions near the cap with probability 1
        raise ValueError(
            f"truncated geometric partition selection: eps / l0 = {e:.3g} needs more than "
            f"{_MAX_TABLE} keep-table entries; use a larger epsilon or a smaller "
            f"max_partitions_contributed")
    return tuple(table)


def _inverse_std_normal_cdf(p: float) -> float:
    from statistics import NormalDist
    return NormalDist().inv_cdf(p)


@dataclasses.dataclass
class SelectionPlan:
    strategy: agg.PartitionSelectionStrategy
    eps: float
    delta: float
    max_partitions_contributed: int
    pre_threshold: Optional[int]
    table: Optional[list] = None
    threshold: float = 0.0
    noise_scale: float = 0.0

    @property
    def native_strategy(self) -> int:
        return {agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC: 1,
                agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING: 2,
                agg.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING: 3}[self.strategy]


def create_partition_selection_strategy(strategy: agg.PartitionSelectionStrategy,
                                        epsilon: float, delta: float,
                                        max_partitions_contributed: int,
                                        pre_threshold: Optional[int] = None
                                        ) -> SelectionPlan:
    """Counterpart of partition_selection.create_partition_selection_strategy."""
    if not epsilon > 0:
        raise ValueError(f"Partition selection: epsilon must be positive, not {epsilon}.")
    if not 0 < delta < 1:
        raise ValueError("Partition selection: delta must be in (0, 1) for private "
                         f"partition selection, not {delta}.")
    l0 = max_partitions_contributed
    plan = SelectionPlan(strategy, epsilon, delta, l0, pre_threshold)
    if strategy == agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC:
        plan.table = truncated_geometric_table(epsilon, delta, l0)
    elif strategy == agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING:
        d = adjusted_delta(delta, l0)
        b = l0 / epsilon
        plan.noise_scale = b
        plan.threshold = (1.0 + b * math.log(2.0 * (1.0 - d)) if d > 0.5 else
                          1.0 - b * math.log(2.0 * d))
    elif strategy == agg.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING:
        noise_delta = delta / 2.0
        sigma = dp_computations.compute_sigma(epsilon, noise_delta, math.sqrt(l0))
        d = adjusted_delta(delta - noise_delta, l0)
        plan.noise_scale = sigma
        plan.threshold = 1.0 + sigma * _inverse_std_normal_cdf(1.0 - d)
    else:
        raise ValueError(f"Unknown partition selection strategy {strategy}")
    return plan


def probability_of_keep(plan: SelectionPlan, n: int) -> float:
    """Host evaluation of the keep probability (tests / analysis)."""
    if n <= 0:
        return 0.0
    if plan.pre_threshold:
        if n < plan.pre_threshold:
            return 0.0
        n = n - plan.pre_threshold + 1
    if plan.strategy == agg.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC:
        return plan.table[n] if n < len(plan.table) else 1.0
    if plan.strategy == agg.PartitionSelectionStrategy.LAPLACE_THRESHOLDING:
        x = (n - plan.threshold) / plan.noise_scale
        return 1.0 - 0.5 * math.exp(-x) if x >= 0 else 0.5 * math.exp(x)
    z = (n - plan.threshold) / plan.noise_scale
    return 0.5 * math.erfc(-z / math.sqrt(2.0))
