"""The CPU oracle against the reference's own outputs (tests/golden, produced
by running /root/reference with a no-noise PyDP stand-in): pre-noise
aggregates with non-binding bounds must match exactly (counts) or to 1e-9
relative (float64), for every combiner and bounding mode on the hot path."""
import numpy as np
import pytest

import pipelinedp_amd as pdp
from oracle import oracle
from pipelinedp_amd import combiners
from tests import golden_cases as gc


def _dense_P(d):
    hi = int(d["pk"].max())
    if "public_partitions" in d:
        hi = max(hi, int(d["public_partitions"].max()))
    return hi + 1


def oracle_metrics(meta, d, seed=1):
    params = gc.params_of(meta)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    plan = combiners.CompoundPlan(params, acc)
    acc.compute_budgets()
    P = _dense_P(d)
    public = d.get("public_partitions")
    pm = oracle.bitmap(public, P) if public is not None else None
    value = d["value"] if plan.needs_values() else None
    part = oracle.bound_aggregate(d["pid"], d["pk"], value, plan.bound_fields(P), seed,
                                  public_mask=pm)
    keep_ids = public if public is not None else np.nonzero(part["rows"])[0]
    sel = dict(strategy=0, max_rows_per_privacy_id=1, pk_offset=0)
    keep, out = oracle.select_and_noise(part, sel, plan.noise_fields(with_noise=False), seed,
                                        public_mask=oracle.bitmap(keep_ids, P))
    ids = np.nonzero(keep)[0]
    return plan, ids, out[ids], part


@pytest.mark.parametrize("meta", gc.cases(), ids=lambda m: m["name"])
def test_oracle_matches_reference_fixture(meta):
    d = gc.load(meta)
    plan, ids, out, _ = oracle_metrics(meta, d)
    assert list(plan.fields) == meta["fields"], "MetricsTuple field order"
    assert np.array_equal(ids, d["out_keys"]), "set of output partitions"
    for j, f in enumerate(plan.fields):
        assert gc.tolerance_ok(f, out[:, j], d["out_" + f]), f
