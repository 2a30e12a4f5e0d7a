"""Utility analysis of many contribution-bound configurations in one device
pass (API mirror of analysis/utility_analysis.py:42-144 and
analysis/utility_analysis_engine.py:29-218).

The reference subclasses DPEngine and swaps graph nodes: the contribution
bounder becomes a per-(privacy id, partition) pre-aggregation
(analysis/contribution_bounders.py:37-77), the compound combiner holds one
set of per-partition utility combiners per configuration
(utility_analysis_engine.py:98-143) and private selection becomes a
keep-probability computation.  On MI355X that is two C-ABI calls:

  dpg_preaggregate      all (pid, pk) pairs with (count, sum, n_partitions,
                        n_contributions), sorted by partition key
  dpg_utility_analysis  every configuration's per-partition combiners in one
                        pass over the pairs (lane = configuration)

followed by the cross-partition combine (cross_partition_combiners.py
:264-343, utility_analysis.py:196-251), a weighted sum over partitions per
(configuration, partition-size bucket) done with device tensor reductions.
The budget is requested and resolved exactly as the reference does it.
"""
import bisect
import ctypes
import dataclasses
import gc
import hashlib
import math
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from pipelinedp_amd import _native
from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import budget_accounting
from pipelinedp_amd import columnar
from pipelinedp_amd import data_extractors as dex
from pipelinedp_amd import dp_computations as dpc
from pipelinedp_amd import partition_selection
from pipelinedp_amd import pipeline_backend
from pipelinedp_amd import pre_aggregation
from pipelinedp_amd.analysis import data_structures
from pipelinedp_amd.analysis import metrics

M_COUNT, M_SUM, M_PID = 1, 2, 4
# per-partition metric blocks of dpg_utility_analysis, in this order
_BLOCKS = ((agg.Metrics.SUM, M_SUM), (agg.Metrics.COUNT, M_COUNT),
           (agg.Metrics.PRIVACY_ID_COUNT, M_PID))


def _generate_bucket_bounds():
    result = [0, 1]
    for i in range(1, 10):
        result += [10**i, 2 * 10**i, 5 * 10**i]
    return tuple(result)


# partition-size histogram bounds (utility_analysis.py:29-39)
BUCKET_BOUNDS = _generate_bucket_bounds()


def _get_lower_bound(n) -> int:
    if n < 0:
        return 0
    return BUCKET_BOUNDS[bisect.bisect_right(BUCKET_BOUNDS, n) - 1]


def _get_upper_bound(n) -> int:
    if n < 0:
        return 0
    i = bisect.bisect_right(BUCKET_BOUNDS, n)
    return BUCKET_BOUNDS[i] if i < len(BUCKET_BOUNDS) else -1


def _check_options(options: data_structures.UtilityAnalysisOptions, extractors):
    """utility_analysis_engine.py:187-218."""
    if options.pre_aggregated_data:
        if not isinstance(extractors, dex.PreAggregateExtractors):
            raise ValueError(
                "options.pre_aggregated_data is set to true but PreAggregateExtractors aren't "
                "provided. PreAggregateExtractors should be specified for pre-aggregated data.")
    elif not isinstance(extractors, dex.DataExtractors):
        raise ValueError("pipeline_dp.DataExtractors should be specified for raw data.")
    params = options.aggregate_params
    if params.custom_combiners is not None:
        raise NotImplementedError("custom combiners are not supported")
    allowed = {agg.Metrics.COUNT, agg.Metrics.SUM, agg.Metrics.PRIVACY_ID_COUNT}
    if not set(params.metrics).issubset(allowed):
        raise NotImplementedError(
            f"unsupported metric in metrics={list(set(params.metrics) - allowed)}")
    if params.contribution_bounds_already_enforced:
        raise NotImplementedError("utility analysis when contribution bounds are already "
                                  "enforced is not supported")


def _noise_std(noise_kind, eps: float, delta: float, l0: float, linf: float) -> float:
    """dp_computations.py:369-388 (compute_dp_count_noise_std)."""
    if noise_kind == agg.NoiseKind.LAPLACE:
        return (l0 * linf / eps) * math.sqrt(2)
    return dpc.compute_sigma(eps, delta, math.sqrt(l0) * linf)


def _sample_bound(prob: float) -> int:
    return int(round(2**64 * prob))


def _keep_by_hash(key, bound: int) -> bool:
    """sampling_utils.ValueSampler.keep (sampling_utils.py:32-51): the
    repr of the key exactly as the user's rows hold it (columnar.decode_keys
    returns Python scalars for integer columns and the row objects for row
    input)."""
    h = int(hashlib.sha1(repr(key).encode()).hexdigest()[:16], 16)
    return h < bound


@dataclasses.dataclass
class _Config:
    params: agg.AggregateParams
    selection: Optional[partition_selection.SelectionPlan]
    noise_std: Dict[Any, float]


class UtilityAnalysis:
    """One utility-analysis run: lazy until the first report or per-partition
    result is requested; then one pre-aggregation and one sweep pass."""

    def __init__(self, col, backend, options, data_extractors, public_partitions=None):
        _check_options(options, data_extractors)
        if not isinstance(backend, pipeline_backend.MI355XBackend):
            raise NotImplementedError("utility analysis runs on MI355XBackend only")
        self.col = col
        self.backend = backend
        self.options = options
        self.extractors = data_extractors
        self.public = public_partitions
        params = options.aggregate_params
        acc = budget_accounting.NaiveBudgetAccountant(total_epsilon=options.epsilon,
                                                      total_delta=options.delta)
        mech = params.noise_kind.convert_to_mechanism_type()
        # utility_analysis_engine.py:98-113: GENERIC first (private), then one
        # mechanism per metric in the user's order, inside the aggregate scope
        with acc.scope(weight=params.budget_weight):
            self._sel_spec = (None if public_partitions is not None else
                              acc.request_budget(agg.MechanismType.GENERIC,
                                                 weight=params.budget_weight))
            self._specs = {m: acc.request_budget(mech, weight=params.budget_weight)
                           for m in params.metrics}
        acc.compute_budgets()  # utility_analysis.py:79
        self.metrics = [m for m, _ in _BLOCKS if m in params.metrics]
        self.configs = [self._config(p) for p in data_structures.get_aggregate_params(options)]
        self.strategies = data_structures.get_partition_selection_strategy(options)
        self._done = False

    # ------------------------------------------------------------ budgets
    def _config(self, p: agg.AggregateParams) -> _Config:
        sel = None
        if self._sel_spec is not None:
            sel = partition_selection.create_partition_selection_strategy(
                p.partition_selection_strategy, self._sel_spec.eps, self._sel_spec.delta,
                p.max_partitions_contributed, p.pre_threshold)
        std = {}
        l0 = p.max_partitions_contributed
        for m in self.metrics:
            spec = self._specs[m]
            # per_partition_combiners.py:289-339: SUM and COUNT use linf =
            # max_contributions_per_partition (compute_dp_count_noise_std),
            # PRIVACY_ID_COUNT linf = 1
            linf = 1 if m == agg.Metrics.PRIVACY_ID_COUNT else p.max_contributions_per_partition
            std[m] = _noise_std(p.noise_kind, spec.eps, spec.delta, l0, linf)
        return _Config(p, sel, std)

    # ------------------------------------------------------------ device
    def _pairs(self, dev):
        """Sorted pre-aggregate (pairs, partition_start, P, key_table,
        public bitmap)."""
        if self.options.pre_aggregated_data:
            ps = pre_aggregation.host_preaggregated_pairs(self.col, self.extractors, self.public,
                                                          dev)
        else:
            ps = pre_aggregation.device_pairs(self.col, self.extractors, self.backend,
                                              self.public, dev)
        self.n_pairs = ps.n_pairs
        return ps.pairs, ps.starts, ps.n_partitions, ps.key_table, ps.public_mask

    def _sample_mask(self, P, key_table, dev):
        prob = self.options.partitions_sampling_prob
        if prob >= 1:
            return None
        bound = _sample_bound(prob)
        keys = columnar.decode_keys(np.arange(P), key_table)
        keep = np.array([_keep_by_hash(k, bound) for k in keys], bool)
        self.sampled = keep
        return torch.from_numpy(np.packbits(keep, bitorder="little")).to(dev)

    def run(self):
        if self._done:
            return
        dev = self.backend.device
        ctx = self.backend.ctx
        pairs, starts, P, key_table, pub_mask = self._pairs(dev)
        sample = self._sample_mask(P, key_table, dev)
        C = len(self.configs)
        M = len(self.metrics)
        cfgs = (_native.UaConfig * C)()
        tables = []
        for i, cf in enumerate(self.configs):
            p = cf.params
            x = cfgs[i]
            x.max_partitions_contributed = p.max_partitions_contributed
            x.max_contributions_per_partition = p.max_contributions_per_partition or 1
            lo, hi = p.min_sum_per_partition, p.max_sum_per_partition
            x.min_sum_per_partition = -math.inf if lo is None else float(lo)
            x.max_sum_per_partition = math.inf if hi is None else float(hi)
            if cf.selection is not None:
                s = cf.selection
                x.selection_strategy = s.native_strategy
                x.pre_threshold = int(s.pre_threshold or 0)
                x.threshold, x.noise_scale = s.threshold, s.noise_scale
                if s.table is not None:
                    t = np.ascontiguousarray(s.table, dtype=np.float64)
                    tables.append(t)
                    x.keep_table, x.table_len = t.ctypes.data, len(t)
        slot = {agg.Metrics.SUM: 0, agg.Metrics.COUNT: 1, agg.Metrics.PRIVACY_ID_COUNT: 2}
        for i, cf in enumerate(self.configs):
            for m in self.metrics:
                cfgs[i].noise_std[slot[m]] = cf.noise_std[m]
        f64 = dict(dtype=torch.float64, device=dev)
        raw = torch.empty((P, 2), **f64)
        err = torch.empty((P, max(M, 1), 5, C), **f64)
        keep = torch.empty((P, C), **f64) if self.public is None else None
        F = 4 + 24 * M
        rep = torch.empty((len(BUCKET_BOUNDS), F, C), **f64)
        # one device pass per 64 configurations (lane = configuration); the
        # pre-aggregate is shared, the outputs are stitched along C
        for c0 in range(0, C, 64):
            c1 = min(C, c0 + 64)
            whole = c0 == 0 and c1 == C
            up = _native.UaParams()
            up.n_configs = c1 - c0
            up.metric_mask = sum(bit for m, bit in _BLOCKS if m in self.metrics)
            up.public_partitions = int(self.public is not None)
            up.configs = ctypes.addressof(cfgs) + c0 * ctypes.sizeof(_native.UaConfig)
            up.sample_mask = sample.data_ptr() if sample is not None else None
            up.public_mask = pub_mask.data_ptr() if pub_mask is not None else None
            e_c = err if whole else torch.empty((P, max(M, 1), 5, c1 - c0), **f64)
            k_c = keep if whole or keep is None else torch.empty((P, c1 - c0), **f64)
            r_c = rep if whole else torch.empty((len(BUCKET_BOUNDS), F, c1 - c0), **f64)
            with torch.cuda.device(dev):
                sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                self.n_out = ctx.utility_analysis(
                    ctypes.c_void_p(pairs.data_ptr()), ctypes.c_void_p(starts.data_ptr()), P, up,
                    ctypes.c_void_p(raw.data_ptr()), ctypes.c_void_p(e_c.data_ptr()),
                    ctypes.c_void_p(k_c.data_ptr()) if k_c is not None else None,
                    ctypes.c_void_p(r_c.data_ptr()), sptr)
            if not whole:
                err[..., c0:c1] = e_c
                rep[..., c0:c1] = r_c
                if keep is not None:
                    keep[:, c0:c1] = k_c
        self.pairs, self.starts, self.key_table = pairs, starts, key_table
        self.sample, self.pub_mask = sample, pub_mask
        self.raw_all, self.err_all, self.keep_all, self.rep = raw, err, keep, rep
        self.stage_ms = ctx.stage_times()
        self._done = True

    def output_ids(self) -> torch.Tensor:
        """Dense ids of the result's partitions: the public ones, or those
        with pairs (and kept by partition sampling)."""
        P = self.starts.numel() - 1
        dev = self.starts.device
        if self.public is not None:
            bits = np.unpackbits(self.pub_mask.cpu().numpy(), bitorder="little")[:P]
            return torch.nonzero(torch.from_numpy(bits).to(dev)).flatten()
        has = (self.starts[1:] - self.starts[:-1]) > 0
        if self.sample is not None:
            has &= torch.from_numpy(self.sampled).to(dev)
        return torch.nonzero(has).flatten()

    # ------------------------------------------------ cross-partition combine
    def _scaled(self, rows: np.ndarray) -> np.ndarray:
        """The report fields of rows [..., F] with every per-partition
        average already divided out (one vectorised pass instead of ~10
        Python multiplies per ValueErrors object): the ValueErrors blocks
        times 1 / (total weight), the DataDropInfo fields times 1 / (the
        metric's total); IEEE products, identical to the scalar form."""
        out = rows.copy()
        with np.errstate(divide="ignore"):
            tw = rows[..., 1]
            ws = np.where(tw == 0, 0.0, 1.0 / np.where(tw == 0, 1.0, tw))
            for mi in range(len(self.metrics)):
                b = 4 + 24 * mi
                tot = rows[..., b]
                ds = np.where(tot == 0, 1.0, 1.0 / np.where(tot == 0, 1.0, tot))
                out[..., b + 1:b + 4] *= ds[..., None]
                out[..., b + 4:b + 24] *= ws[..., None]
        return out

    def _report(self, c: int, v: list, sc: list) -> metrics.UtilityReport:
        """UtilityReport of configuration c from its summed fields v and
        their scaled form sc (_scaled), both the field layout of
        dpg_utility_analysis' report output as lists of Python floats
        (per-element numpy scalar access dominated the report assembly of a
        64-configuration sweep)."""
        # positional construction throughout (fields in declaration order,
        # metrics.py): keyword matching was half of the assembly time of a
        # 64-configuration report set
        public = self.public is not None
        if public:
            info = metrics.PartitionsInfo(True, int(round(v[2])), 0, int(round(v[3])))
        else:
            # the reference sets strategies[configuration_index] while the
            # index is still -1 (utility_analysis.py:117-129 runs before
            # :218-229 assigns it): every report names the LAST strategy
            info = metrics.PartitionsInfo(False, int(round(v[0])), None, None,
                                          self.strategies[-1], metrics.MeanVariance(v[2], v[3]))
        report = metrics.UtilityReport(c, info)
        if not self.metrics:
            return report
        errs = []
        noise_kind = self.configs[c].params.noise_kind
        VE, CBE, MV = metrics.ValueErrors, metrics.ContributionBoundingErrors, metrics.MeanVariance
        MU, DDI = metrics.MetricUtility, metrics.DataDropInfo
        # the reference labels metric_errors by zipping them with the user's
        # metric order (cross_partition_combiners.py:208-212)
        for mi, (um, std) in enumerate(zip(self._user_metrics, self.configs[c].std_list)):
            b = 4 + 24 * mi
            a, r = b + 4, b + 14
            errs.append(MU(
                um, std, noise_kind, DDI(sc[b + 1], sc[b + 2], sc[b + 3]),
                VE(CBE(MV(sc[a], sc[a + 1]), sc[a + 2], sc[a + 3]), sc[a + 4], sc[a + 5],
                   sc[a + 6], sc[a + 7], sc[a + 8], sc[a + 9]),
                VE(CBE(MV(sc[r], sc[r + 1]), sc[r + 2], sc[r + 3]), sc[r + 4], sc[r + 5],
                   sc[r + 6], sc[r + 7], sc[r + 8], sc[r + 9])))
        report.metric_errors = errs
        return report

    def reports(self) -> List[metrics.UtilityReport]:
        """One UtilityReport per configuration with its partition-size
        histogram (utility_analysis.py:196-251), from the device's summed
        report fields per (size bucket, configuration)."""
        self.run()
        byb = self.rep.permute(0, 2, 1).cpu().numpy()        # [bucket, C, F]
        present = np.nonzero(byb[:, 0, 0] > 0)[0].tolist()
        # totals and the present buckets as one [1 + buckets, C, F] block
        block = np.concatenate([byb.sum(axis=0)[None], byb[present]], axis=0)
        raw = block.tolist()
        scaled = self._scaled(block).tolist()
        self._user_metrics = list(self.options.aggregate_params.metrics)
        for cf in self.configs:
            cf.std_list = [cf.noise_std[m] for m in self.metrics]
        bins = [(j + 1, BUCKET_BOUNDS[bi], _get_upper_bound(BUCKET_BOUNDS[bi]))
                for j, bi in enumerate(present)]
        out = []
        # tens of thousands of small result objects: a generational collection
        # triggered midway scans the whole process heap (~60 ms measured on the
        # GPU box, every few steps); nothing here forms reference cycles
        gc_on = gc.isenabled()
        gc.disable()
        try:
            Bin = metrics.UtilityReportBin
            for c in range(len(self.configs)):
                rep = self._report(c, raw[0][c], scaled[0][c])
                hist = [Bin(lo, hi, self._report(c, raw[j][c], scaled[j][c])) for j, lo, hi in bins]
                rep.utility_report_histogram = hist if hist else None
                out.append(rep)
        finally:
            if gc_on:
                gc.enable()
        return out

    def per_partition(self) -> Iterable[Tuple[Tuple[Any, int], metrics.PerPartitionMetrics]]:
        """((partition_key, configuration_index), PerPartitionMetrics), lazily
        (utility_analysis.py:86-100)."""
        self.run()
        ids = self.output_ids()
        keys = columnar.decode_keys(ids.cpu().numpy(), self.key_table)
        std = {m: [cf.noise_std[m] for cf in self.configs] for m in self.metrics}
        C = len(self.configs)
        M = len(self.metrics)
        chunk = 4096
        for s in range(0, len(keys), chunk):
            sel = ids[s:s + chunk]
            raw = self.raw_all[sel].cpu().numpy()
            err = self.err_all[sel][:, :M].cpu().numpy()
            keep = self.keep_all[sel].cpu().numpy() if self.keep_all is not None else None
            for j, key in enumerate(keys[s:s + chunk]):
                rs = metrics.RawStatistics(int(round(raw[j, 0])), int(round(raw[j, 1])))
                for c in range(C):
                    errs = []
                    for mi, m in enumerate(self.metrics):
                        e = err[j, mi, :, c]
                        total = float(e[0]) if m == agg.Metrics.SUM else int(round(e[0]))
                        errs.append(metrics.SumMetrics(
                            aggregation=m, sum=total, clipping_to_min_error=float(e[1]),
                            clipping_to_max_error=float(e[2]),
                            expected_l0_bounding_error=float(e[3]),
                            std_l0_bounding_error=math.sqrt(max(float(e[4]), 0.0)),
                            std_noise=std[m][c], noise_kind=self.configs[c].params.noise_kind))
                    prob = 1 if keep is None else float(keep[j, c])
                    yield (key, c), metrics.PerPartitionMetrics(prob, rs, errs)


class _Lazy:
    def __init__(self, fn):
        self._fn = fn

    def __iter__(self):
        return iter(self._fn())


def perform_utility_analysis(col, backend, options: data_structures.UtilityAnalysisOptions,
                             data_extractors: Union[dex.DataExtractors,
                                                    dex.PreAggregateExtractors],
                             public_partitions=None):
    """Utility analysis of DP aggregations (utility_analysis.py:42-144).

    Returns (reports, per_partition_result): a lazy collection with one
    metrics.UtilityReport per configuration, and a lazy collection of
    ((partition_key, configuration_index), metrics.PerPartitionMetrics).
    The analysis object itself is available as `reports.analysis` for bulk
    (tensor) access."""
    run = UtilityAnalysis(col, backend, options, data_extractors, public_partitions)
    reports = _Lazy(run.reports)
    reports.analysis = run
    per_partition = _Lazy(run.per_partition)
    per_partition.analysis = run
    return reports, per_partition
