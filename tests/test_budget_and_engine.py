"""Host-side engine logic: budget split parity with the reference
(tests/golden/budget_splits.json), laziness, explain report, errors."""
import json
import os

import numpy as np
import pytest

import pipelinedp_amd as pdp
from tests import golden_cases as gc

M = {"COUNT": pdp.Metrics.COUNT, "SUM": pdp.Metrics.SUM,
     "PRIVACY_ID_COUNT": pdp.Metrics.PRIVACY_ID_COUNT, "MEAN": pdp.Metrics.MEAN,
     "VARIANCE": pdp.Metrics.VARIANCE}


def _cases():
    with open(os.path.join(gc.GOLDEN, "budget_splits.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", _cases(),
                         ids=lambda c: f"{'+'.join(c['metrics'])}-{c['noise_kind']}-"
                                       f"{'pub' if c['public'] else 'priv'}-w{c['budget_weight']}")
def test_budget_split_matches_reference(case):
    """Same mechanism specs, same order, same (eps, delta) after
    compute_budgets() as the reference (budget_accounting.py:380-408,
    combiners.py:791-858, dp_engine.py:322)."""
    acc = pdp.NaiveBudgetAccountant(2.0, 1e-5)
    specs = []
    orig = acc.request_budget

    def rec(*a, **k):
        s = orig(*a, **k)
        specs.append(s)
        return s
    acc.request_budget = rec
    eng = pdp.DPEngine(acc, pdp.MI355XBackend(device=0, seed=1))
    kw = dict(metrics=[M[m] for m in case["metrics"]],
              noise_kind=pdp.NoiseKind[case["noise_kind"]], max_partitions_contributed=2,
              max_contributions_per_partition=3, budget_weight=case["budget_weight"])
    if any(m in case["metrics"] for m in ("SUM", "MEAN", "VARIANCE")):
        kw.update(min_value=0.0, max_value=1.0)
    eng.aggregate([(1, 1, 0.5)], pdp.AggregateParams(**kw),
                  pdp.DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2]),
                  public_partitions=[1] if case["public"] else None)
    eng.select_partitions([(1, 1)], pdp.SelectPartitionsParams(max_partitions_contributed=1),
                          pdp.DataExtractors(lambda r: r[0], lambda r: r[1]))
    acc.compute_budgets()
    want = case["specs"]
    assert [s.mechanism_type.name for s in specs] == [w["type"] for w in want]
    for s, w in zip(specs, want):
        assert s.eps == pytest.approx(w["eps"], rel=1e-12)
        assert s.delta == pytest.approx(w["delta"], rel=1e-12, abs=1e-300)


def _engine():
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    return acc, pdp.DPEngine(acc, pdp.MI355XBackend(device=0, seed=3))


def _params(**kw):
    base = dict(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM],
                max_partitions_contributed=2, max_contributions_per_partition=1,
                min_value=0.0, max_value=5.0)
    base.update(kw)
    return pdp.AggregateParams(**base)


EX = pdp.DataExtractors(lambda r: r[0], lambda r: r[1], lambda r: r[2])


def test_aggregate_is_lazy_and_budget_bound():
    acc, eng = _engine()
    res = eng.aggregate([(1, 1, 1.0)], _params(), EX)
    # nothing ran: iterating before compute_budgets fails like the reference
    with pytest.raises(AssertionError, match="not calculated"):
        res.plan.noise_fields()
    acc.compute_budgets()
    f = res.plan.noise_fields()
    assert f["n_outputs"] == 2 and f["out_src"][:2] == [0, 1]
    # Laplace b = l1 / eps: eps = 1/3 each (count, sum, selection)
    assert f["scale"][0] == pytest.approx(2 * 1 / (1 / 3))
    assert f["scale"][1] == pytest.approx(2 * 5.0 / (1 / 3))


def test_explain_report_stages():
    acc, eng = _engine()
    rep = pdp.ExplainComputationReport()
    eng.aggregate([(1, 1, 1.0)], _params(), EX, out_explain_computation_report=rep)
    acc.compute_budgets()
    text = rep.text()
    assert "DPEngine method: aggregate" in text
    assert "Per-partition contribution bounding" in text
    assert "Cross-partition contribution bounding" in text
    assert "Private Partition selection: using Truncated Geometric method" in text
    assert "Computed DP count with" in text and "Laplace mechanism:" in text


@pytest.mark.parametrize("bad,err", [
    (dict(col=[]), ValueError),
    (dict(params=None), ValueError),
    (dict(extractors=None), ValueError),
])
def test_aggregate_argument_errors(bad, err):
    acc, eng = _engine()
    col = bad.get("col", [(1, 1, 1.0)])
    params = bad.get("params", _params()) if "params" in bad else _params()
    ex = bad.get("extractors", EX) if "extractors" in bad else EX
    with pytest.raises(err):
        eng.aggregate(col, params, ex)


def test_max_contributions_rejects_variance():
    acc, eng = _engine()
    p = pdp.AggregateParams(metrics=[pdp.Metrics.VARIANCE], max_contributions=2,
                            min_value=0.0, max_value=1.0)
    with pytest.raises(NotImplementedError):
        eng.aggregate([(1, 1, 1.0)], p, EX)


def test_percentile_is_out_of_scope():
    acc, eng = _engine()
    p = pdp.AggregateParams(metrics=[pdp.Metrics.PERCENTILE(50)],
                            max_partitions_contributed=1, max_contributions_per_partition=1,
                            min_value=0.0, max_value=1.0)
    with pytest.raises(NotImplementedError):
        eng.aggregate([(1, 1, 1.0)], p, EX)


@pytest.mark.parametrize("kw,msg", [
    (dict(max_partitions_contributed=None, max_contributions_per_partition=None),
     "either max_contributions must be set"),
    (dict(max_contributions_per_partition=None), "either none or both"),
    (dict(min_value=None), "should be both set"),
    (dict(min_value=6.0), "must be equal to or greater"),
    (dict(max_partitions_contributed=0), "has to be positive integer"),
    (dict(min_sum_per_partition=0.0, max_sum_per_partition=1.0), "can not be both set"),
    (dict(pre_threshold=0), "has to be positive integer"),
])
def test_params_validation(kw, msg):
    with pytest.raises(ValueError, match=msg):
        _params(**kw)


def test_budget_accountant_errors():
    with pytest.raises(ValueError):
        pdp.NaiveBudgetAccountant(0, 1e-6)
    acc = pdp.NaiveBudgetAccountant(1, 0)
    with pytest.raises(ValueError, match="Gaussian"):
        acc.request_budget(pdp.MechanismType.GAUSSIAN)
    acc = pdp.NaiveBudgetAccountant(1, 1e-6)
    acc.request_budget(pdp.MechanismType.LAPLACE)
    acc.compute_budgets()
    with pytest.raises(Exception, match="twice"):
        acc.compute_budgets()
    with pytest.raises(Exception, match="after compute_budgets"):
        acc.request_budget(pdp.MechanismType.LAPLACE)
