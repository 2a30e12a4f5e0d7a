"""Contribution-bound tuning (API mirror of analysis/parameter_tuning.py).

tune() (:278-348) picks candidate bounds from the dataset histograms
(device: dataset_histograms/computing_histograms.py), runs one utility
analysis over all candidates (device: analysis/utility_analysis.py, 64
configurations per pass over one shared pre-aggregate) and recommends the
candidate with the smallest RMSE of the first metric.  Candidate generation
is host arithmetic over histogram bins.
"""
import dataclasses
import enum
import logging
import math
from numbers import Number
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import data_extractors as dex
from pipelinedp_amd.analysis import data_structures
from pipelinedp_amd.analysis import metrics
from pipelinedp_amd.analysis import utility_analysis
from pipelinedp_amd.dataset_histograms import histograms


class MinimizingFunction(enum.Enum):
    ABSOLUTE_ERROR = "absolute_error"
    RELATIVE_ERROR = "relative_error"


@dataclasses.dataclass
class ParametersToTune:
    max_partitions_contributed: bool = False
    max_contributions_per_partition: bool = False
    min_sum_per_partition: bool = False
    max_sum_per_partition: bool = False

    def __post_init__(self):
        if not any(dataclasses.asdict(self).values()):
            raise ValueError("ParametersToTune must have at least 1 parameter to tune.")


@dataclasses.dataclass
class TuneOptions:
    """parameter_tuning.py:52-89."""
    epsilon: float
    delta: float
    aggregate_params: agg.AggregateParams
    function_to_minimize: Union[MinimizingFunction, Callable]
    parameters_to_tune: ParametersToTune
    partitions_sampling_prob: float = 1
    pre_aggregated_data: bool = False
    number_of_parameter_candidates: int = 100

    def __post_init__(self):
        agg.validate_epsilon_delta(self.epsilon, self.delta, "TuneOptions")


@dataclasses.dataclass
class TuneResult:
    """parameter_tuning.py:92-112."""
    options: TuneOptions
    contribution_histograms: histograms.DatasetHistograms
    utility_analysis_parameters: data_structures.MultiParameterConfiguration
    index_best: int
    utility_reports: List[metrics.UtilityReport]


def _find_candidates_constant_relative_step(histogram: histograms.Histogram,
                                            max_candidates: int) -> List[int]:
    """1 = a_0 < a_1 < ... <= max_value with a constant ratio
    max_value^(1 / (n - 1)) (rounded up, strictly increasing; :236-264)."""
    max_value = histogram.max_value()
    assert max_value >= 1, "max_value has to be >= 1."
    max_candidates = min(max_candidates, max_value)
    assert max_candidates > 0, "max_candidates have to be positive"
    if max_candidates == 1:
        return [1]
    step = pow(max_value, 1 / (max_candidates - 1))
    out, acc = [1], 1
    for _ in range(1, max_candidates):
        if out[-1] >= max_value:
            break
        acc *= step
        out.append(max(out[-1] + 1, math.ceil(acc)))
    out[-1] = max_value  # float drift: the last candidate is the max itself
    return out


def _find_candidates_bins_max_values_subsample(histogram: histograms.Histogram,
                                               max_candidates: int) -> List[float]:
    """Bin maxima at evenly spaced bin indices (:267-275)."""
    max_candidates = min(max_candidates, len(histogram.bins))
    ids = np.round(np.linspace(0, len(histogram.bins) - 1, num=max_candidates)).astype(int)
    maxima = np.fromiter((b.max for b in histogram.bins), dtype=float)
    return maxima[ids].tolist()


def _find_candidates_parameters_in_2d_grid(
        hist1: histograms.Histogram, hist2: histograms.Histogram,
        find1: Callable[[histograms.Histogram, int], Sequence[Number]],
        find2: Callable[[histograms.Histogram, int], Sequence[Number]],
        max_candidates: int) -> Tuple[List[Number], List[Number]]:
    """Grid of ~sqrt(max) x sqrt(max) candidates; a parameter with fewer
    candidates hands its share to the other (:182-233)."""
    per = int(math.sqrt(max_candidates))
    c1, c2 = find1(hist1, per), find2(hist2, per)
    if len(c2) < per and len(c1) == per:
        c1 = find1(hist1, int(max_candidates / len(c2)))
    elif len(c1) < per and len(c2) == per:
        c2 = find2(hist2, int(max_candidates / len(c1)))
    return [a for a in c1 for _ in c2], [b for _ in c1 for b in c2]


def _find_candidate_parameters(hist: histograms.DatasetHistograms,
                               parameters_to_tune: ParametersToTune,
                               metric: Optional[agg.Metric],
                               max_candidates: int) -> data_structures.MultiParameterConfiguration:
    """Candidates for l0, linf (COUNT) and max_sum_per_partition (SUM)
    (:115-179)."""
    tune_l0 = parameters_to_tune.max_partitions_contributed
    tune_linf = parameters_to_tune.max_contributions_per_partition and metric == agg.Metrics.COUNT
    tune_sum = parameters_to_tune.max_sum_per_partition and metric == agg.Metrics.SUM
    l0 = linf = max_sum = min_sum = None
    if tune_sum and hist.linf_sum_contributions_histogram.bins[0].lower >= 0:
        logging.warning("max_sum_per_partition should not contain negative sums because"
                        " min_sum_per_partition tuning is not supported yet and "
                        "therefore tuning for max_sum_per_partition works only when "
                        "linf_sum_contributions_histogram does not negative sums")
    step = _find_candidates_constant_relative_step
    if tune_l0 and tune_linf:
        l0, linf = _find_candidates_parameters_in_2d_grid(
            hist.l0_contributions_histogram, hist.linf_contributions_histogram, step, step,
            max_candidates)
    elif tune_l0 and tune_sum:
        l0, max_sum = _find_candidates_parameters_in_2d_grid(
            hist.l0_contributions_histogram, hist.linf_sum_contributions_histogram, step,
            _find_candidates_bins_max_values_subsample, max_candidates)
        min_sum = [0] * len(max_sum)
    elif tune_l0:
        l0 = step(hist.l0_contributions_histogram, max_candidates)
    elif tune_linf:
        linf = step(hist.linf_contributions_histogram, max_candidates)
    elif tune_sum:
        max_sum = _find_candidates_bins_max_values_subsample(
            hist.linf_sum_contributions_histogram, max_candidates)
        min_sum = [0] * len(max_sum)
    else:
        assert False, "Nothing to tune."
    return data_structures.MultiParameterConfiguration(
        max_partitions_contributed=l0, max_contributions_per_partition=linf,
        min_sum_per_partition=min_sum, max_sum_per_partition=max_sum)


def _check_tune_args(options: TuneOptions, is_public_partitions: bool):
    """:384-411."""
    m = options.aggregate_params.metrics
    if not m:
        if is_public_partitions:
            raise ValueError("Empty metrics means tuning of partition selection"
                             " but public partitions were provided.")
    elif len(m) > 1:
        raise ValueError(f"Tuning supports only one metric, but {m} given.")
    elif m[0] not in (agg.Metrics.COUNT, agg.Metrics.PRIVACY_ID_COUNT, agg.Metrics.SUM):
        raise ValueError(f"Tuning is supported only for Count, Privacy id count and Sum, "
                         f"but {m[0]} given.")
    if options.parameters_to_tune.min_sum_per_partition:
        raise ValueError("Tuning of min_sum_per_partition is not supported yet.")
    if options.function_to_minimize != MinimizingFunction.ABSOLUTE_ERROR:
        raise NotImplementedError(f"Only {MinimizingFunction.ABSOLUTE_ERROR} is implemented.")


def _convert_utility_analysis_to_tune_result(
        utility_reports, tune_options: TuneOptions,
        run_configurations: data_structures.MultiParameterConfiguration,
        use_public_partitions: bool,
        contribution_histograms: histograms.DatasetHistograms) -> TuneResult:
    """:351-381: reports sorted by configuration; the best index minimises
    the absolute RMSE of the first metric (-1 for partition selection)."""
    assert len(utility_reports) == run_configurations.size
    assert tune_options.function_to_minimize == MinimizingFunction.ABSOLUTE_ERROR
    reports = sorted(utility_reports, key=lambda r: r.configuration_index)
    best = -1
    if tune_options.aggregate_params.metrics:
        best = int(np.argmin([r.metric_errors[0].absolute_error.rmse for r in reports]))
    return TuneResult(tune_options, contribution_histograms, run_configurations, best,
                      utility_reports=reports)


class _OneResult:
    def __init__(self, fn):
        self._fn = fn

    def __iter__(self):
        return iter([self._fn()])


def tune(col, backend, contribution_histograms: histograms.DatasetHistograms,
         options: TuneOptions,
         data_extractors: Union[dex.DataExtractors, dex.PreAggregateExtractors],
         public_partitions=None):
    """Returns (1-element collection with the TuneResult, per-partition
    utility analysis results) (:278-348).  For select_partitions tuning
    leave options.aggregate_params.metrics empty."""
    _check_tune_args(options, public_partitions is not None)
    metric = options.aggregate_params.metrics[0] if options.aggregate_params.metrics else None
    candidates = _find_candidate_parameters(contribution_histograms, options.parameters_to_tune,
                                            metric, options.number_of_parameter_candidates)
    ua_options = data_structures.UtilityAnalysisOptions(
        epsilon=options.epsilon, delta=options.delta, aggregate_params=options.aggregate_params,
        multi_param_configuration=candidates,
        partitions_sampling_prob=options.partitions_sampling_prob,
        pre_aggregated_data=options.pre_aggregated_data)
    reports, per_partition = utility_analysis.perform_utility_analysis(
        col, backend, ua_options, data_extractors, public_partitions)
    result = _OneResult(lambda: _convert_utility_analysis_to_tune_result(
        list(reports), options, candidates, public_partitions is not None,
        contribution_histograms))
    return result, per_partition
