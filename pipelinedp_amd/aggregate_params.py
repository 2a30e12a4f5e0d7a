"""Aggregation parameters (API mirror of pipeline_dp/aggregate_params.py).

Same class names, field names, defaults and validation errors as the
reference (pipeline_dp/aggregate_params.py:28-365), so user code that builds
`AggregateParams` for PipelineDP builds them unchanged here.  Only the
host-side validation lives here; nothing in this module touches the GPU.
"""
import dataclasses
import enum
import logging
import math
from typing import Any, Callable, List, Optional, Sequence

import numpy as np


@dataclasses.dataclass
class Metric:
    """A DP metric, optionally parameterised (e.g. PERCENTILE(90))."""
    name: str
    parameter: Optional[float] = None

    def __eq__(self, other):
        return (isinstance(other, Metric) and self.name == other.name and
                self.parameter == other.parameter)

    def __hash__(self):
        return hash(str(self))

    def __str__(self):
        return self.name if self.parameter is None else f"{self.name}({self.parameter})"

    __repr__ = __str__

    @property
    def is_percentile(self) -> bool:
        return self.name == "PERCENTILE"


class Metrics:
    """All metrics of the reference (aggregate_params.py:61-72)."""
    COUNT = Metric("COUNT")
    PRIVACY_ID_COUNT = Metric("PRIVACY_ID_COUNT")
    SUM = Metric("SUM")
    MEAN = Metric("MEAN")
    VARIANCE = Metric("VARIANCE")
    VECTOR_SUM = Metric("VECTOR_SUM")

    @classmethod
    def PERCENTILE(cls, percentile_to_compute: float) -> Metric:
        return Metric("PERCENTILE", percentile_to_compute)


class NoiseKind(enum.Enum):
    LAPLACE = "laplace"
    GAUSSIAN = "gaussian"

    def convert_to_mechanism_type(self) -> "MechanismType":
        return {NoiseKind.LAPLACE: MechanismType.LAPLACE,
                NoiseKind.GAUSSIAN: MechanismType.GAUSSIAN}[self]


class MechanismType(enum.Enum):
    LAPLACE = "Laplace"
    GAUSSIAN = "Gaussian"
    GENERIC = "Generic"

    def to_noise_kind(self) -> NoiseKind:
        if self is MechanismType.LAPLACE:
            return NoiseKind.LAPLACE
        if self is MechanismType.GAUSSIAN:
            return NoiseKind.GAUSSIAN
        raise ValueError(f"MechanismType {self.value} can not be converted to "
                         f"NoiseKind")


class NormKind(enum.Enum):
    Linf = "linf"
    L0 = "l0"
    L1 = "l1"
    L2 = "l2"


class PartitionSelectionStrategy(enum.Enum):
    TRUNCATED_GEOMETRIC = "Truncated Geometric"
    LAPLACE_THRESHOLDING = "Laplace Thresholding"
    GAUSSIAN_THRESHOLDING = "Gaussian Thresholding"


def _is_int(x: Any) -> bool:
    return isinstance(x, (int, np.integer)) and not isinstance(x, bool)


def _require_positive_int(value: Any, name: str) -> None:
    if not (_is_int(value) and value > 0):
        raise ValueError(f"{name} has to be positive integer, but {value} given.")


def _require_finite(value: Any, name: str) -> None:
    if math.isnan(value) or math.isinf(value):
        raise ValueError(f"AggregateParams: {name} must be a finite number")


def validate_epsilon_delta(epsilon: float, delta: float, owner: str) -> None:
    """input_validators.py:17-34."""
    if epsilon <= 0:
        raise ValueError(f"{owner}: epsilon must be positive, not {epsilon}.")
    if delta < 0:
        raise ValueError(f"{owner}: delta must be non-negative, not {delta}.")
    if delta >= 1:
        raise ValueError(f"{owner}: delta must be less than 1, not {delta}.")


@dataclasses.dataclass
class AggregateParams:
    """Parameters of DPEngine.aggregate (aggregate_params.py:166-365)."""
    metrics: List[Metric]
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    max_partitions_contributed: Optional[int] = None
    max_contributions_per_partition: Optional[int] = None
    max_contributions: Optional[int] = None
    budget_weight: float = 1
    min_value: Optional[float] = None
    max_value: Optional[float] = None
    min_sum_per_partition: Optional[float] = None
    max_sum_per_partition: Optional[float] = None
    custom_combiners: Sequence[Any] = None
    vector_norm_kind: Optional[NormKind] = None
    vector_max_norm: Optional[float] = None
    vector_size: Optional[int] = None
    contribution_bounds_already_enforced: bool = False
    public_partitions_already_filtered: bool = False
    partition_selection_strategy: PartitionSelectionStrategy = (
        PartitionSelectionStrategy.TRUNCATED_GEOMETRIC)
    pre_threshold: Optional[int] = None

    @property
    def metrics_str(self) -> str:
        if self.custom_combiners:
            names = [c.metrics_names() for c in self.custom_combiners]
            return f"custom combiners={names}"
        if self.metrics:
            return f"metrics={[str(m) for m in self.metrics]}"
        return "metrics=[]"

    @property
    def bounds_per_contribution_are_set(self) -> bool:
        return self.min_value is not None and self.max_value is not None

    @property
    def bounds_per_partition_are_set(self) -> bool:
        return (self.min_sum_per_partition is not None and
                self.max_sum_per_partition is not None)

    def __post_init__(self):
        self._validate_pairs()
        self._validate_metric_compatibility()
        self._validate_contribution_bounds()
        if self.pre_threshold is not None:
            _require_positive_int(self.pre_threshold, "pre_threshold")

    def _validate_pairs(self):
        for a, b in (("min_value", "max_value"),
                     ("min_sum_per_partition", "max_sum_per_partition")):
            if (getattr(self, a) is None) != (getattr(self, b) is None):
                raise ValueError(f"AggregateParams: {a} and {b} should be both "
                                 f"set or both None.")
        per_value = self.min_value is not None
        per_partition = self.min_sum_per_partition is not None
        if per_value and per_partition:
            raise ValueError(
                "min_value and min_sum_per_partition can not be both set.")
        for lo, hi, on in (("min_value", "max_value", per_value),
                           ("min_sum_per_partition", "max_sum_per_partition",
                            per_partition)):
            if not on:
                continue
            _require_finite(getattr(self, lo), lo)
            _require_finite(getattr(self, hi), hi)
            if getattr(self, lo) > getattr(self, hi):
                raise ValueError(f"AggregateParams: {hi} must be equal to or "
                                 f"greater than {lo}")

    def _validate_metric_compatibility(self):
        if self.metrics:
            metrics = set(self.metrics)
            per_value = self.min_value is not None
            per_partition = self.min_sum_per_partition is not None
            if Metrics.VECTOR_SUM in metrics:
                if metrics & {Metrics.SUM, Metrics.MEAN, Metrics.VARIANCE}:
                    raise ValueError(
                        "AggregateParams: vector sum can not be computed "
                        "together with scalar metrics such as sum, mean etc")
            elif per_partition:
                bad = metrics - {Metrics.SUM, Metrics.PRIVACY_ID_COUNT,
                                 Metrics.COUNT}
                if bad:
                    raise ValueError(
                        f"AggregateParams: min_sum_per_partition is not "
                        f"compatible with metrics {bad}. Please use "
                        f"min_value/max_value.")
            elif not per_value:
                bad = metrics - {Metrics.PRIVACY_ID_COUNT, Metrics.COUNT}
                if bad:
                    raise ValueError(
                        f"AggregateParams: for metrics {bad} bounds per "
                        f"partition are required (e.g. min_value,max_value).")
            if (self.contribution_bounds_already_enforced and
                    Metrics.PRIVACY_ID_COUNT in metrics):
                raise ValueError(
                    "AggregateParams: Cannot calculate PRIVACY_ID_COUNT when "
                    "contribution_bounds_already_enforced is set to True.")
        if self.custom_combiners:
            logging.warning("Warning: custom combiners are used. This is an "
                            "experimental feature.")
            if self.metrics:
                raise ValueError(
                    "Custom combiners can not be used with standard metrics")

    def _validate_contribution_bounds(self):
        if self.max_contributions is not None:
            _require_positive_int(self.max_contributions, "max_contributions")
            if (self.max_partitions_contributed is not None or
                    self.max_contributions_per_partition is not None):
                raise ValueError(
                    "AggregateParams: only one in max_contributions or both "
                    "max_partitions_contributed and "
                    "max_contributions_per_partition must be set")
            return
        given = [x is not None for x in (self.max_partitions_contributed,
                                         self.max_contributions_per_partition)]
        if not any(given):
            raise ValueError(
                "AggregateParams: either max_contributions must be set or both "
                "max_partitions_contributed and "
                "max_contributions_per_partition must be set.")
        if not all(given):
            raise ValueError(
                "AggregateParams: either none or both max_partitions_contributed "
                "and max_contributions_per_partition must be set.")
        _require_positive_int(self.max_partitions_contributed,
                              "max_partitions_contributed")
        _require_positive_int(self.max_contributions_per_partition,
                              "max_contributions_per_partition")

    def __str__(self):
        return parameters_to_readable_string(self)


@dataclasses.dataclass
class SelectPartitionsParams:
    """Parameters of DPEngine.select_partitions (aggregate_params.py:368-395)."""
    max_partitions_contributed: int
    budget_weight: float = 1
    partition_selection_strategy: PartitionSelectionStrategy = (
        PartitionSelectionStrategy.TRUNCATED_GEOMETRIC)
    pre_threshold: Optional[int] = None

    def __post_init__(self):
        if self.pre_threshold is not None:
            _require_positive_int(self.pre_threshold, "pre_threshold")

    def __str__(self):
        return "Private Partitions"


@dataclasses.dataclass
class CalculatePrivateContributionBoundsParams:
    """Parameters of DPEngine.calculate_private_contribution_bounds
    (aggregate_params.py:113-150): the noise and budget of the COUNT /
    PRIVACY_ID_COUNT aggregation the bound is for, the budget of the
    calculation itself and the largest bound worth considering."""
    aggregation_noise_kind: NoiseKind
    aggregation_eps: float
    aggregation_delta: float
    calculation_eps: float
    max_partitions_contributed_upper_bound: int

    def __post_init__(self):
        owner = "CalculatePrivateContributionBoundsParams"
        validate_epsilon_delta(self.aggregation_eps, self.aggregation_delta, owner)
        if self.aggregation_noise_kind is None:
            raise ValueError("aggregation_noise_kind must be set.")
        if self.aggregation_noise_kind == NoiseKind.GAUSSIAN and self.aggregation_delta == 0:
            raise ValueError("The Gaussian noise requires that the aggregation_delta is "
                             "greater than 0.")
        validate_epsilon_delta(self.calculation_eps, 0, owner)
        _require_positive_int(self.max_partitions_contributed_upper_bound,
                              "max_partitions_contributed_upper_bound")


@dataclasses.dataclass
class PrivateContributionBounds:
    """Contribution bounds chosen with DP (aggregate_params.py:153-163)."""
    max_partitions_contributed: int


@dataclasses.dataclass
class SumParams:
    max_partitions_contributed: int
    max_contributions_per_partition: int
    min_value: float
    max_value: float
    partition_extractor: Callable
    value_extractor: Callable
    budget_weight: float = 1
    noise_kind: NoiseKind = NoiseKind.LAPLACE
    contribution_bounds_already_enforced: bool = False


@dataclasses.dataclass
class CountParams:
    noise_kind: NoiseKind
    max_partitions_contributed: int
    max_contributions_per_partition: int
    partition_extractor: Callable
    budget_weight: float = 1
    contribution_bounds_already_enforced: bool = False


@dataclasses.dataclass
class PrivacyIdCountParams:
    noise_kind: NoiseKind
    max_partitions_contributed: int
    partition_extractor: Callable
    budget_weight: float = 1
    contribution_bounds_already_enforced: bool = False


def parameters_to_readable_string(params, is_public_partition: Optional[bool] = None) -> str:
    """Human-readable parameter dump used by the explain report
    (aggregate_params.py:594-625)."""
    lines = [f"{type(params).__name__}:"]
    if hasattr(params, "metrics_str"):
        lines.append(f" {params.metrics_str}")
    if hasattr(params, "noise_kind"):
        lines.append(f" noise_kind={params.noise_kind.value}")
    if hasattr(params, "budget_weight"):
        lines.append(f" budget_weight={params.budget_weight}")
    lines.append(" Contribution bounding:")
    for name in ("max_partitions_contributed", "max_contributions_per_partition",
                 "max_contributions", "min_value", "max_value",
                 "min_sum_per_partition", "max_sum_per_partition"):
        value = getattr(params, name, None)
        if value is not None:
            lines.append(f"  {name}={value}")
    if getattr(params, "contribution_bounds_already_enforced", False):
        lines.append("  contribution_bounds_already_enforced=True")
    for name in ("vector_max_norm", "vector_size", "vector_norm_kind"):
        value = getattr(params, name, None)
        if value is not None:
            lines.append(f"  {name}={value}")
    if is_public_partition is not None:
        kind = "public" if is_public_partition else "private"
        lines.append(f" Partition selection: {kind} partitions")
    return "\n".join(lines)
