"""Compound-combiner plan for the device path.

In the reference a `CompoundCombiner` (pipeline_dp/combiners.py:640-739)
owns one Python combiner per metric; every (privacy id, partition) pair
gets a Python accumulator tuple which is merged per partition and finally
noised by PyDP.  On MI355X the accumulators are device arrays, so the
combiner collapses into a *plan*: which accumulators the bounding kernel
must produce, which budgets were requested (in the reference's order, so
the budget split is identical -- combiners.py:791-858), how the output
MetricsTuple is laid out (the reference's field order, combiners.py:708-730)
and, once budgets are computed, the per-slot noise scales for the
selection+noise kernel.
"""
import collections
from typing import Dict, List, Optional, Tuple

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import budget_accounting
from pipelinedp_amd import dp_computations as dpc

# native enums (include/dpg.h)
M_COUNT, M_SUM, M_PID, M_MEAN, M_VARIANCE = 1, 2, 4, 8, 16
FAMILY_SCALAR, FAMILY_MEAN, FAMILY_VARIANCE = 0, 1, 2
SLOT_COUNT, SLOT_SUM, SLOT_NSQ, SLOT_PID = 0, 1, 2, 3
V_COUNT, V_SUM, V_MEAN, V_VARIANCE, V_PID = 0, 1, 2, 3, 4
MODE_CROSS_AND_PER, MODE_PER_PID, MODE_CROSS = 0, 1, 2
SUM_NONE, SUM_CLIP_VALUE, SUM_CLIP_PARTITION = 0, 1, 2
NOISE_NONE, NOISE_LAPLACE, NOISE_GAUSSIAN = 0, 1, 2

_FIELD_SOURCE = {"count": V_COUNT, "sum": V_SUM, "mean": V_MEAN,
                 "variance": V_VARIANCE, "privacy_id_count": V_PID}

_named_tuples: Dict[Tuple[str, ...], type] = {}


def metrics_tuple_type(fields: Tuple[str, ...]) -> type:
    """MetricsTuple namedtuple with the reference's field order."""
    t = _named_tuples.get(fields)
    if t is None:
        t = collections.namedtuple("MetricsTuple", fields)
        _named_tuples[fields] = t
    return t


class CompoundPlan:
    """What one DPEngine.aggregate call computes on the device."""

    def __init__(self, params: agg.AggregateParams,
                 accountant: budget_accounting.BudgetAccountant):
        self.params = params
        metrics = set(params.metrics or [])
        unsupported = [m for m in metrics
                       if m == agg.Metrics.VECTOR_SUM or m.is_percentile]
        if unsupported:
            raise NotImplementedError(
                f"{unsupported} are not supported by the MI355X backend "
                f"(see DESIGN.md, out of scope)")
        mech = params.noise_kind.convert_to_mechanism_type()
        w = params.budget_weight
        self.noise_kind = params.noise_kind
        self.specs: Dict[str, budget_accounting.MechanismSpec] = {}
        fields: List[str] = []
        self.mask = 0
        # combiners.py:798-837 -- same request order, same weights
        if agg.Metrics.VARIANCE in metrics:
            self.family = FAMILY_VARIANCE
            self.specs["variance"] = accountant.request_budget(mech, weight=w)
            fields.append("variance")
            fields += [n for n, m in (("count", agg.Metrics.COUNT),
                                      ("sum", agg.Metrics.SUM),
                                      ("mean", agg.Metrics.MEAN)) if m in metrics]
            self.mask |= M_COUNT | M_VARIANCE
        elif agg.Metrics.MEAN in metrics:
            self.family = FAMILY_MEAN
            self.specs["count"] = accountant.request_budget(mech, weight=w)
            self.specs["sum"] = accountant.request_budget(mech, weight=w)
            fields.append("mean")
            fields += [n for n, m in (("count", agg.Metrics.COUNT),
                                      ("sum", agg.Metrics.SUM)) if m in metrics]
            self.mask |= M_COUNT | M_MEAN
            self._count_sens = dpc.sensitivities_for_count(params)
            self._nsum_sens = dpc.sensitivities_for_normalized_sum(params)
        else:
            self.family = FAMILY_SCALAR
            if agg.Metrics.COUNT in metrics:
                self.specs["count"] = accountant.request_budget(mech, weight=w)
                fields.append("count")
                self.mask |= M_COUNT
                self._count_sens = dpc.sensitivities_for_count(params)
            if agg.Metrics.SUM in metrics:
                self.specs["sum"] = accountant.request_budget(mech, weight=w)
                fields.append("sum")
                self.mask |= M_SUM
                self._sum_sens = dpc.sensitivities_for_sum(params)
        if agg.Metrics.PRIVACY_ID_COUNT in metrics:
            self.specs["privacy_id_count"] = accountant.request_budget(mech, weight=w)
            fields.append("privacy_id_count")
            self.mask |= M_PID
            self._pid_sens = dpc.sensitivities_for_privacy_id_count(params)
        self.fields = tuple(fields)
        self.MetricsTuple = metrics_tuple_type(self.fields)
        self._mechanisms = None

    # ------------------------------------------------------------ bounding
    def expects_per_partition_sampling(self) -> bool:
        """combiners.py:76-85, 323-324, 364-365, 738-739."""
        if self.family != FAMILY_SCALAR or "count" in self.specs:
            return True
        if "sum" in self.specs:
            return not self.params.bounds_per_partition_are_set
        return False

    def bounding_mode(self) -> int:
        """dp_engine.py:370-382."""
        if self.params.max_contributions:
            return MODE_PER_PID
        if self.expects_per_partition_sampling():
            return MODE_CROSS_AND_PER
        return MODE_CROSS

    def sum_mode(self) -> int:
        if not (self.mask & (M_SUM | M_MEAN | M_VARIANCE)):
            return SUM_NONE
        if self.params.bounds_per_partition_are_set:
            return SUM_CLIP_PARTITION
        return SUM_CLIP_VALUE

    def needs_values(self) -> bool:
        return bool(self.mask & (M_SUM | M_MEAN | M_VARIANCE))

    def bound_fields(self, n_partitions: int) -> dict:
        """Field values of dpg_bound_params."""
        p = self.params
        return dict(
            mode=self.bounding_mode(), sum_mode=self.sum_mode(),
            metric_mask=self.mask,
            max_partitions_contributed=p.max_partitions_contributed or 0,
            max_contributions_per_partition=p.max_contributions_per_partition or 0,
            max_contributions=p.max_contributions or 0,
            min_value=float(p.min_value) if p.min_value is not None else 0.0,
            max_value=float(p.max_value) if p.max_value is not None else 0.0,
            min_sum_per_partition=float(p.min_sum_per_partition)
            if p.min_sum_per_partition is not None else 0.0,
            max_sum_per_partition=float(p.max_sum_per_partition)
            if p.max_sum_per_partition is not None else 0.0,
            n_partitions=int(n_partitions))

    # ------------------------------------------------------------- noise
    def _mech(self, name: str, sens: dpc.Sensitivities) -> dpc.AdditiveMechanism:
        spec = self.specs[name]
        return dpc.AdditiveMechanism(self.noise_kind, spec.eps, spec.delta, sens)

    def mechanisms(self) -> Dict[str, dpc.AdditiveMechanism]:
        """Resolved after compute_budgets(); raises AssertionError before,
        like the reference's lazy MechanismSpec (budget_accounting.py:66-84)."""
        if self._mechanisms is None:
            m = {}
            if self.family == FAMILY_MEAN:
                m["count"] = self._mech("count", self._count_sens)
                m["normalized_sum"] = self._mech("sum", self._nsum_sens)
            elif self.family == FAMILY_SCALAR:
                if "count" in self.specs:
                    m["count"] = self._mech("count", self._count_sens)
                if "sum" in self.specs:
                    m["sum"] = self._mech("sum", self._sum_sens)
            if "privacy_id_count" in self.specs:
                m["privacy_id_count"] = self._mech("privacy_id_count", self._pid_sens)
            self._mechanisms = m
        return self._mechanisms

    def _variance_scales(self) -> dict:
        """compute_dp_var (dp_computations.py:307-366): 3-way budget split."""
        p = self.params
        spec = self.specs["variance"]
        (ce, cd), (se, sd), (qe, qd) = dpc.equally_split_budget(spec.eps, spec.delta, 3)
        l0 = p.max_partitions_contributed
        mcpp = p.max_contributions_per_partition
        kind = self.noise_kind
        mid = dpc.compute_middle(p.min_value, p.max_value)
        sq_lo, sq_hi = dpc.compute_squares_interval(p.min_value, p.max_value)
        sq_mid = dpc.compute_middle(sq_lo, sq_hi)
        out = dict(count=dpc.noise_scale(kind, ce, cd, l0, mcpp), mid=mid,
                   mean_const=p.min_value == p.max_value, mean_const_value=p.min_value,
                   msq_const=sq_lo == sq_hi, msq_const_value=sq_lo)
        out["nsum"] = (0.0 if out["mean_const"] else
                       dpc.noise_scale(kind, se, sd, l0, mcpp * abs(mid - p.min_value)))
        out["nsq"] = (0.0 if out["msq_const"] else
                      dpc.noise_scale(kind, qe, qd, l0, mcpp * abs(sq_mid - sq_lo)))
        return out

    def noise_fields(self, with_noise: bool = True) -> dict:
        """Field values of dpg_noise_params (after compute_budgets())."""
        kind = {agg.NoiseKind.LAPLACE: NOISE_LAPLACE,
                agg.NoiseKind.GAUSSIAN: NOISE_GAUSSIAN}[self.noise_kind]
        scale = [0.0, 0.0, 0.0, 0.0]
        slot_mask = 0
        extra = dict(mid=0.0, mean_const=0, msq_const=0, mean_const_value=0.0,
                     msq_const_value=0.0)
        if self.family == FAMILY_VARIANCE:
            v = self._variance_scales()
            scale[SLOT_COUNT], scale[SLOT_SUM], scale[SLOT_NSQ] = v["count"], v["nsum"], v["nsq"]
            slot_mask |= 0b111
            extra.update(mid=v["mid"], mean_const=int(v["mean_const"]),
                         msq_const=int(v["msq_const"]),
                         mean_const_value=float(v["mean_const_value"]),
                         msq_const_value=float(v["msq_const_value"]))
        else:
            mech = self.mechanisms()
            if self.family == FAMILY_MEAN:
                scale[SLOT_COUNT] = mech["count"].scale
                scale[SLOT_SUM] = mech["normalized_sum"].scale
                slot_mask |= 0b11
                extra["mid"] = dpc.compute_middle(self.params.min_value,
                                                  self.params.max_value)
            else:
                if "count" in mech:
                    scale[SLOT_COUNT] = mech["count"].scale
                    slot_mask |= 1 << SLOT_COUNT
                if "sum" in mech:
                    scale[SLOT_SUM] = mech["sum"].scale
                    slot_mask |= 1 << SLOT_SUM
        if "privacy_id_count" in self.specs:
            scale[SLOT_PID] = self.mechanisms()["privacy_id_count"].scale
            slot_mask |= 1 << SLOT_PID
        out_src = [_FIELD_SOURCE[f] for f in self.fields] + [0] * (8 - len(self.fields))
        return dict(noise_kind=kind if with_noise else NOISE_NONE, family=self.family,
                    slot_mask=slot_mask, n_outputs=len(self.fields), out_src=out_src,
                    scale=scale, **extra)

    # ------------------------------------------------------------ report
    def explain_computation(self) -> List:
        stages = []
        if self.family == FAMILY_VARIANCE:
            spec = self.specs["variance"]
            stages.append(lambda: f"Computed variance with (eps={spec.eps} delta={spec.delta})")
            return stages + self._pid_explain()
        if self.family == FAMILY_MEAN:
            mid = dpc.compute_middle(self.params.min_value, self.params.max_value)

            def mean_report():
                m = self.mechanisms()
                return ("DP mean computation:\n"
                        f"    a. Computed 'normalized_sum' = sum of (value - {mid})\n"
                        f"    b. Applied to 'count' {m['count'].describe()}\n"
                        f"    c. Applied to 'normalized_sum' {m['normalized_sum'].describe()}")
            stages.append(mean_report)
            return stages + self._pid_explain()
        for name in ("count", "sum"):
            if name in self.specs:
                stages.append(lambda name=name: (
                    f"Computed DP {name} with\n     "
                    f"{self.mechanisms()[name].describe()}"))
        return stages + self._pid_explain()

    def _pid_explain(self) -> List:
        if "privacy_id_count" not in self.specs:
            return []
        return [lambda: ("Computed DP privacy_id_count with\n     "
                         f"{self.mechanisms()['privacy_id_count'].describe()}")]
