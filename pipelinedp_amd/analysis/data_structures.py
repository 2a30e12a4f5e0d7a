"""Utility-analysis option dataclasses (API mirror of
analysis/data_structures.py:24-151): a blueprint AggregateParams plus
per-configuration overrides; one sweep evaluates every configuration."""
import copy
import dataclasses
from typing import Iterable, Optional, Sequence

from pipelinedp_amd import aggregate_params as agg

_SWEEP_FIELDS = ("max_partitions_contributed", "max_contributions_per_partition",
                 "min_sum_per_partition", "max_sum_per_partition", "noise_kind",
                 "partition_selection_strategy")


@dataclasses.dataclass
class MultiParameterConfiguration:
    """Parameter sweep: every non-None attribute is a sequence with one value
    per configuration (all of the same length); configuration i is the
    blueprint AggregateParams with the i-th values substituted."""
    max_partitions_contributed: Sequence[int] = None
    max_contributions_per_partition: Sequence[int] = None
    min_sum_per_partition: Sequence[float] = None
    max_sum_per_partition: Sequence[float] = None
    noise_kind: Sequence[agg.NoiseKind] = None
    partition_selection_strategy: Sequence[agg.PartitionSelectionStrategy] = None

    def __post_init__(self):
        lengths = {len(getattr(self, f)) for f in _SWEEP_FIELDS if getattr(self, f)}
        if not lengths:
            raise ValueError("MultiParameterConfiguration must have at least 1"
                             " non-empty attribute.")
        if len(lengths) > 1:
            raise ValueError("All set attributes in MultiParameterConfiguration must have "
                             "the same length.")
        if (self.min_sum_per_partition is None) != (self.max_sum_per_partition is None):
            raise ValueError("MultiParameterConfiguration: min_sum_per_partition and "
                             "max_sum_per_partition must be both set or both None.")
        self._size = lengths.pop()

    @property
    def size(self) -> int:
        return self._size

    def get_aggregate_params(self, params: agg.AggregateParams,
                             index: int) -> agg.AggregateParams:
        out = copy.copy(params)
        for f in _SWEEP_FIELDS:
            values = getattr(self, f)
            if values:
                setattr(out, f, values[index])
        return out


@dataclasses.dataclass
class UtilityAnalysisOptions:
    epsilon: float
    delta: float
    aggregate_params: agg.AggregateParams
    multi_param_configuration: Optional[MultiParameterConfiguration] = None
    partitions_sampling_prob: float = 1
    pre_aggregated_data: bool = False

    def __post_init__(self):
        if self.epsilon is None or self.epsilon <= 0:
            raise ValueError(f"UtilityAnalysisOptions: epsilon must be positive, "
                             f"not {self.epsilon}.")
        if self.delta is None or self.delta < 0:
            raise ValueError(f"UtilityAnalysisOptions: delta must be non-negative, "
                             f"not {self.delta}.")
        if not 0 < self.partitions_sampling_prob <= 1:
            raise ValueError(f"partitions_sampling_prob must be in the interval (0, 1], "
                             f"but {self.partitions_sampling_prob} given.")

    @property
    def n_configurations(self) -> int:
        m = self.multi_param_configuration
        return 1 if m is None else m.size


def get_aggregate_params(options: UtilityAnalysisOptions) -> Iterable[agg.AggregateParams]:
    m = options.multi_param_configuration
    if m is None:
        yield options.aggregate_params
        return
    for i in range(m.size):
        yield m.get_aggregate_params(options.aggregate_params, i)


def get_partition_selection_strategy(
        options: UtilityAnalysisOptions) -> Sequence[agg.PartitionSelectionStrategy]:
    m = options.multi_param_configuration
    if m is not None and m.partition_selection_strategy is not None:
        return m.partition_selection_strategy
    return [options.aggregate_params.partition_selection_strategy] * options.n_configurations
