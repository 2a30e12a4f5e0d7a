"""DPEngine (API mirror of pipeline_dp/dp_engine.py) on the MI355X backend.

`aggregate` keeps the reference's contract (dp_engine.py:56-99): argument
checks and errors, one budget scope of `budget_weight`, the combiner budget
requests in the reference's order followed by the GENERIC partition-
selection request (:322-323), the explain-report stages, a lazy result,
`_compute_budget_for_aggregation` and `annotate`.  The computational graph
(:101-176) is replaced by the fused device path in device_aggregate.py.
"""
from typing import Optional

import numpy as np
import torch

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import budget_accounting
from pipelinedp_amd import combiners
from pipelinedp_amd import data_extractors as dex
from pipelinedp_amd import device_aggregate
from pipelinedp_amd import pipeline_backend
from pipelinedp_amd import pre_aggregation
from pipelinedp_amd import private_contribution_bounds
from pipelinedp_amd import report_generator
from pipelinedp_amd.dataset_histograms import computing_histograms


def _as_collection(public_partitions):
    """Public partitions as a re-iterable collection: ranges, arrays and
    tensors stay as they are (the device builds their bitmap), anything else
    (e.g. a generator) is listed."""
    if isinstance(public_partitions, (range, list, tuple, np.ndarray, torch.Tensor)):
        return public_partitions
    return list(public_partitions)


def _check_col(col):
    if col is None or not col:
        raise ValueError("col must be non-empty")


def _check_data_extractors(extractors):
    if extractors is None:
        raise ValueError("data_extractors must be set to a DataExtractors")
    if not isinstance(extractors, dex.DataExtractors):
        raise TypeError("data_extractors must be set to a DataExtractors")


class DPEngine:
    """Performs DP aggregations on an MI355X GPU."""

    def __init__(self, budget_accountant: budget_accounting.BudgetAccountant,
                 backend: pipeline_backend.PipelineBackend):
        self._budget_accountant = budget_accountant
        self._backend = backend
        self._report_generators = []

    @property
    def _current_report_generator(self):
        return self._report_generators[-1]

    def _add_report_stage(self, stage):
        self._current_report_generator.add_stage(stage)

    def explain_computations_report(self):
        return [g.report() for g in self._report_generators]

    def _require_device_backend(self):
        if not isinstance(self._backend, pipeline_backend.MI355XBackend):
            raise NotImplementedError(
                "pipelinedp_amd.DPEngine executes on MI355XBackend only.")

    # ------------------------------------------------------------ aggregate
    def aggregate(self, col, params: agg.AggregateParams,
                  data_extractors: dex.DataExtractors, public_partitions=None,
                  out_explain_computation_report: Optional[
                      report_generator.ExplainComputationReport] = None):
        """Computes DP aggregate metrics; returns a lazy collection of
        (partition_key, MetricsTuple)."""
        self._check_aggregate_params(col, params, data_extractors)
        self._check_budget_accountant_compatibility(public_partitions is not None)
        self._require_device_backend()
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._report_generators.append(report_generator.ReportGenerator(
                params, "aggregate", public_partitions is not None))
            if out_explain_computation_report is not None:
                out_explain_computation_report._set_report_generator(
                    self._current_report_generator)
            result = self._aggregate(col, params, data_extractors, public_partitions)
            budget = self._budget_accountant._compute_budget_for_aggregation(
                params.budget_weight)
            return self._annotate(result, params=params, budget=budget)

    def _aggregate(self, col, params, data_extractors, public_partitions):
        if params.custom_combiners:
            raise NotImplementedError(
                "custom combiners run arbitrary Python per accumulator and are not "
                "supported on the MI355X backend (see DESIGN.md)")
        plan = combiners.CompoundPlan(params, self._budget_accountant)
        public = public_partitions is not None
        if public and not params.public_partitions_already_filtered:
            self._add_report_stage(
                "Public partition selection: dropped non public partitions")
        if not params.contribution_bounds_already_enforced:
            self._add_bounding_stages(params, plan.bounding_mode())
        if public:
            self._add_report_stage("Adding empty partitions for public partitions "
                                   "that are missing in data")
        spec = None
        max_rows = 1
        if not public:
            if params.contribution_bounds_already_enforced:
                max_rows = (params.max_contributions or
                            params.max_contributions_per_partition)
            spec = self._request_selection_budget(params.partition_selection_strategy,
                                                  params.pre_threshold)
        for stage in plan.explain_computation():
            self._add_report_stage(stage)
        l0 = params.max_partitions_contributed or params.max_contributions
        return device_aggregate.DeviceAggregation(
            self._backend, col, data_extractors, plan,
            public_partitions=None if not public else _as_collection(public_partitions),
            selection_spec=spec, strategy=params.partition_selection_strategy,
            max_partitions_contributed=l0, pre_threshold=params.pre_threshold,
            max_rows_per_privacy_id=max_rows,
            drop_non_public=not params.public_partitions_already_filtered,
            bounds_already_enforced=params.contribution_bounds_already_enforced)

    def _add_bounding_stages(self, params, mode):
        # report text of contribution_bounders.py:77-80, 94-97, 125-127
        if mode == combiners.MODE_PER_PID:
            self._add_report_stage(
                f"User contribution bounding: randomly selected not more than "
                f"{params.max_contributions} contributions")
        elif mode == combiners.MODE_CROSS_AND_PER:
            self._add_report_stage(
                f"Per-partition contribution bounding: for each privacy_id and each"
                f"partition, randomly select max(actual_contributions_per_partition"
                f", {params.max_contributions_per_partition}) contributions.")
            self._add_report_stage(
                f"Cross-partition contribution bounding: for each privacy_id "
                f"randomly select max(actual_partition_contributed, "
                f"{params.max_partitions_contributed}) partitions")

    def _request_selection_budget(self, strategy, pre_threshold):
        spec = self._budget_accountant.request_budget(
            mechanism_type=agg.MechanismType.GENERIC)
        pre = f", pre_threshold={pre_threshold}" if pre_threshold else ""
        self._add_report_stage(
            lambda: f"Private Partition selection: using {strategy.value} "
            f"method with (eps={spec.eps}, delta={spec.delta}{pre})")
        return spec

    # --------------------------------------------------- select_partitions
    def select_partitions(self, col, params: agg.SelectPartitionsParams,
                          data_extractors: dex.DataExtractors):
        """DP set of partitions (dp_engine.py:201-278); lazy collection of keys."""
        self._check_select_private_partitions(col, params, data_extractors)
        self._check_budget_accountant_compatibility(False)
        self._require_device_backend()
        with self._budget_accountant.scope(weight=params.budget_weight):
            self._report_generators.append(
                report_generator.ReportGenerator(params, "select_partitions"))
            spec = self._request_selection_budget(params.partition_selection_strategy,
                                                  params.pre_threshold)
            result = device_aggregate.DeviceAggregation(
                self._backend, col, data_extractors, None, selection_spec=spec,
                strategy=params.partition_selection_strategy,
                max_partitions_contributed=params.max_partitions_contributed,
                pre_threshold=params.pre_threshold, keys_only=True)
            budget = self._budget_accountant._compute_budget_for_aggregation(
                params.budget_weight)
            return self._annotate(result, params=params, budget=budget)

    # --------------------------------------- private contribution bounds
    def calculate_private_contribution_bounds(
            self, col, params: agg.CalculatePrivateContributionBoundsParams,
            data_extractors: dex.DataExtractors, partitions, partitions_already_filtered=False):
        """DP max_partitions_contributed for COUNT / PRIVACY_ID_COUNT
        (dp_engine.py:432-484): the L0 histogram of the rows restricted to
        `partitions` (device: pre-aggregate + histogram kernels), then the
        exponential mechanism over the candidate bounds.  Returns a
        1-element collection of PrivateContributionBounds."""
        _check_col(col)
        if params is None:
            raise ValueError("params must be set to a valid "
                             "CalculatePrivateContributionBoundsParams")
        if not isinstance(params, agg.CalculatePrivateContributionBoundsParams):
            raise TypeError("params must be set to a valid "
                            "CalculatePrivateContributionBoundsParams")
        _check_data_extractors(data_extractors)
        self._require_device_backend()
        partitions = _as_collection(partitions)
        backend = self._backend

        def histograms():
            ps = pre_aggregation.device_pairs(
                col, data_extractors, backend,
                None if partitions_already_filtered else partitions, backend.device)
            return computing_histograms.histograms_from_pairs(ps, backend, pre_aggregated=False)

        calc = private_contribution_bounds.PrivateL0Calculator(
            params, partitions, computing_histograms._OneElement(histograms), backend)
        return computing_histograms._OneElement(lambda: agg.PrivateContributionBounds(
            max_partitions_contributed=calc.calculate()[0]))

    # ------------------------------------------------------------- checks
    def _check_aggregate_params(self, col, params, data_extractors):
        if params is not None and getattr(params, "max_contributions", None) is not None:
            supported = {agg.Metrics.PRIVACY_ID_COUNT, agg.Metrics.COUNT,
                         agg.Metrics.SUM, agg.Metrics.MEAN}
            bad = set(params.metrics) - supported
            if bad:
                raise NotImplementedError(
                    f"max_contributions is not supported for {bad}")
        _check_col(col)
        if params is None:
            raise ValueError("params must be set to a valid AggregateParams")
        if not isinstance(params, agg.AggregateParams):
            raise TypeError("params must be set to a valid AggregateParams")
        _check_data_extractors(data_extractors)
        if params.contribution_bounds_already_enforced:
            if data_extractors.privacy_id_extractor:
                raise ValueError("privacy_id_extractor should be set iff "
                                 "contribution_bounds_already_enforced is False")
            if agg.Metrics.PRIVACY_ID_COUNT in params.metrics:
                raise ValueError("PRIVACY_ID_COUNT cannot be computed when "
                                 "contribution_bounds_already_enforced is True.")

    def _check_select_private_partitions(self, col, params, data_extractors):
        _check_col(col)
        if params is None:
            raise ValueError("params must be set to a valid SelectPrivatePartitionsParams")
        if not isinstance(params, agg.SelectPartitionsParams):
            raise TypeError("params must be set to a valid SelectPrivatePartitionsParams")
        if (not isinstance(params.max_partitions_contributed, int) or
                params.max_partitions_contributed <= 0):
            raise ValueError("params.max_partitions_contributed must be set "
                             "(to a positive integer)")
        if data_extractors is None:
            raise ValueError("data_extractors must be set to a pipeline_dp.DataExtractors")
        if not isinstance(data_extractors, dex.DataExtractors):
            raise TypeError("data_extractors must be set to a pipeline_dp.DataExtractors")

    def _check_budget_accountant_compatibility(self, is_public_partition: bool):
        if not isinstance(self._budget_accountant,
                          budget_accounting.NaiveBudgetAccountant):
            raise NotImplementedError("only NaiveBudgetAccountant is supported")

    def _annotate(self, col, params, budget):
        return self._backend.annotate(col, "annotation", params=params, budget=budget)
