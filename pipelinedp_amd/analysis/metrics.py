"""Utility-analysis result dataclasses (API mirror of analysis/metrics.py
:24-282): field names, order and semantics as in the reference."""
from dataclasses import dataclass
from typing import List, Optional

from pipelinedp_amd import aggregate_params as agg


@dataclass(slots=True)
class SumMetrics:
    """Per-partition error terms of one DP metric (COUNT, PRIVACY_ID_COUNT
    or SUM): E(bounded value) = sum + clipping_to_min_error +
    clipping_to_max_error + expected_l0_bounding_error."""
    aggregation: agg.Metric
    sum: float
    clipping_to_min_error: float
    clipping_to_max_error: float
    expected_l0_bounding_error: float
    std_l0_bounding_error: float
    std_noise: float
    noise_kind: agg.NoiseKind


@dataclass(slots=True)
class RawStatistics:
    privacy_id_count: int
    count: int


@dataclass(slots=True)
class PerPartitionMetrics:
    partition_selection_probability_to_keep: float
    raw_statistics: RawStatistics
    metric_errors: Optional[List[SumMetrics]] = None


@dataclass(slots=True)
class MeanVariance:
    mean: float
    var: float


@dataclass(slots=True)
class ContributionBoundingErrors:
    l0: MeanVariance
    linf_min: float
    linf_max: float

    def to_relative(self, value: float) -> "ContributionBoundingErrors":
        return ContributionBoundingErrors(
            l0=MeanVariance(self.l0.mean / value, self.l0.var / value**2),
            linf_min=self.linf_min / value, linf_max=self.linf_max / value)


@dataclass(slots=True)
class ValueErrors:
    """Errors of (dp_value - actual_value) averaged across partitions; the
    *_with_dropped_partitions variants count dropped partitions as error."""
    bounding_errors: ContributionBoundingErrors
    mean: float
    variance: float
    rmse: float
    l1: float
    rmse_with_dropped_partitions: float
    l1_with_dropped_partitions: float

    def to_relative(self, value: float) -> "ValueErrors":
        if value == 0:
            zero = ContributionBoundingErrors(l0=MeanVariance(0, 0), linf_min=0, linf_max=0)
            return ValueErrors(bounding_errors=zero, mean=0, variance=0, rmse=0, l1=0,
                               rmse_with_dropped_partitions=0, l1_with_dropped_partitions=0)
        return ValueErrors(self.bounding_errors.to_relative(value), mean=self.mean / value,
                           variance=self.variance / value**2, rmse=self.rmse / value,
                           l1=self.l1 / value,
                           rmse_with_dropped_partitions=self.rmse_with_dropped_partitions / value,
                           l1_with_dropped_partitions=self.l1_with_dropped_partitions / value)


@dataclass(slots=True)
class DataDropInfo:
    l0: float
    linf: float
    partition_selection: float


@dataclass(slots=True)
class MetricUtility:
    metric: agg.Metric
    noise_std: float
    noise_kind: agg.NoiseKind
    ratio_data_dropped: Optional[DataDropInfo]
    absolute_error: ValueErrors
    relative_error: ValueErrors


@dataclass(slots=True)
class PartitionsInfo:
    public_partitions: bool
    num_dataset_partitions: int
    num_non_public_partitions: Optional[int] = None
    num_empty_partitions: Optional[int] = None
    strategy: Optional[agg.PartitionSelectionStrategy] = None
    kept_partitions: Optional[MeanVariance] = None


@dataclass(slots=True)
class UtilityReport:
    configuration_index: int
    partitions_info: PartitionsInfo
    metric_errors: Optional[List[MetricUtility]] = None
    utility_report_histogram: Optional[List["UtilityReportBin"]] = None


@dataclass(slots=True)
class UtilityReportBin:
    """Report of the partitions whose size lies in [partition_size_from,
    partition_size_to)."""
    partition_size_from: int
    partition_size_to: int
    report: UtilityReport
