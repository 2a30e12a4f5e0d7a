"""Distributional parity of contribution bounding with the reference.

The reference samples with numpy's global RNG (sampling_utils.py:19-29,
pipeline_backend.py:531-547); its outcome histogram over 4000 seeds on a
tiny input is committed in tests/golden/sampling_distribution.json.  The
oracle's keyed-priority sampler (the same one the HIP kernels run, bit for
bit -- tests/test_gpu_parity.py) must produce the same distribution:
chi-square homogeneity test, and exact analytic probabilities.
"""
import json
import math
import os

import numpy as np
from scipy import stats

import pipelinedp_amd as pdp
from oracle import oracle
from pipelinedp_amd import combiners
from tests import golden_cases as gc


def _fixture():
    with open(os.path.join(gc.GOLDEN, "sampling_distribution.json")) as f:
        return json.load(f)


def _oracle_histogram_params(rows, trials, params, fields):
    """Outcome histogram of the oracle's keyed sampler over `trials` seeds:
    per partition 10, 11, 12 the given partial columns."""
    pid = np.array([r[0] for r in rows])
    pk = np.array([r[1] for r in rows])
    val = np.array([r[2] for r in rows], dtype=float)
    plan = combiners.CompoundPlan(params, pdp.NaiveBudgetAccountant(1.0, 1e-6))
    bf = plan.bound_fields(13)
    hist = {}
    for seed in range(1, trials + 1):
        p = oracle.bound_aggregate(pid, pk, val, bf, seed * 0x9E3779B97F4A7C15 % 2**64)
        key = json.dumps([[float(p[c][k]) for c in fields] for k in (10, 11, 12)])
        hist[key] = hist.get(key, 0) + 1
    return hist


def _params_from(fx):
    kw = dict(fx["params"])
    kw["metrics"] = [getattr(pdp.Metrics, m) for m in kw["metrics"]]
    return pdp.AggregateParams(**kw)


def _chi2_same(ref, ours):
    keys = sorted(set(ours) | set(ref))
    table = np.array([[ref.get(k, 0) for k in keys], [ours.get(k, 0) for k in keys]])
    return stats.chi2_contingency(table)[1]


def test_per_privacy_id_and_cross_partition_distributions_match_reference():
    """The two secondary bounders (contribution_bounders.py:108-150 and
    :153-195), reference outcome histograms over 4000 numpy seeds
    (tests/golden/gen_golden.py gen_sampling_distribution_modes) against
    the oracle's keyed sampler -- which the GPU kernels reproduce bit for bit
    (tests/test_gpu_parity.py): same support, chi-square homogeneity."""
    for name, cols in (("per_privacy_id", ("count", "sum")),
                       ("cross_partition", ("sum", "rows"))):
        with open(os.path.join(gc.GOLDEN, f"sampling_distribution_{name}.json")) as f:
            fx = json.load(f)
        ours = _oracle_histogram_params(fx["rows"], fx["trials"], _params_from(fx), cols)
        assert set(ours) == set(fx["histogram"]), name
        p = _chi2_same(fx["histogram"], ours)
        assert p > 1e-4, (name, p)


def test_per_privacy_id_marginals_are_exact():
    """max_contributions = 2 keeps a uniform 2-subset of each pid's records:
    pid 2 keeps 2 of its 4 (all in partition 10), pid 1 keeps 2 of its 6 --
    so partition 12 (one record of pid 1) is present w.p.
    1 - C(5,2)/C(6,2) = 1/3."""
    with open(os.path.join(gc.GOLDEN, "sampling_distribution_per_privacy_id.json")) as f:
        fx = json.load(f)
    ours = _oracle_histogram_params(fx["rows"], 6000, _params_from(fx), ("count", "sum"))
    n = sum(ours.values())
    has12 = sum(c for k, c in ours.items() if json.loads(k)[2][0] == 1.0)
    assert abs(has12 / n - 1 / 3) < 4 * math.sqrt(2 / 9 / n)
    # every outcome keeps exactly 4 records: 2 per privacy id
    assert all(sum(x[0] for x in json.loads(k)) == 4.0 for k in ours)


def _oracle_histogram(rows, trials, mpc, mcpp):
    pid = np.array([r[0] for r in rows])
    pk = np.array([r[1] for r in rows])
    val = np.array([r[2] for r in rows], dtype=float)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=mpc,
                                 max_contributions_per_partition=mcpp,
                                 min_value=0.0, max_value=10.0)
    plan = combiners.CompoundPlan(params, pdp.NaiveBudgetAccountant(1.0, 1e-6))
    fields = plan.bound_fields(13)
    hist = {}
    for seed in range(1, trials + 1):
        p = oracle.bound_aggregate(pid, pk, val, fields, seed * 0x9E3779B97F4A7C15 % 2**64)
        key = json.dumps([[float(p["count"][k]), float(p["sum"][k]), float(p["rows"][k])]
                          for k in (10, 11, 12)])
        hist[key] = hist.get(key, 0) + 1
    return hist


def test_bounding_distribution_matches_reference():
    fx = _fixture()
    ours = _oracle_histogram(fx["rows"], fx["trials"], fx["mpc"], fx["mcpp"])
    keys = sorted(set(ours) | set(fx["histogram"]))
    assert set(ours) == set(fx["histogram"]), "same support of outcomes"
    table = np.array([[fx["histogram"].get(k, 0) for k in keys], [ours.get(k, 0) for k in keys]])
    chi2, p, _, _ = stats.chi2_contingency(table)
    assert p > 1e-4, (chi2, p)


def test_bounding_marginals_are_exact():
    """Uniform sampling marginals: pid 1 keeps each of its 3 partitions with
    probability 2/3; in pair (1,10) = {1,1,5} value 1 survives w.p. 2/3."""
    fx = _fixture()
    ours = _oracle_histogram(fx["rows"], 6000, fx["mpc"], fx["mcpp"])
    n = sum(ours.values())
    kept11 = sum(c for k, c in ours.items() if json.loads(k)[1][2] == 1.0)
    assert abs(kept11 / n - 2 / 3) < 4 * math.sqrt(2 / 9 / n)
    one_in_10 = sum(c for k, c in ours.items()
                    if json.loads(k)[0][2] == 2.0 and json.loads(k)[0][1] in (4.0, 5.0, 10.0))
    both_10 = sum(c for k, c in ours.items() if json.loads(k)[0][2] == 2.0)
    # both pids kept partition 10: its sum is v1 + v2 with pid 1's value v1 in
    # {1, 1, 5} and pid 2's v2 in {3, 4, 4, 9}, one each (mcpp = 1); v1 = 1
    # (w.p. 2/3) iff the sum is 4, 5 or 10, v2 = 4 (w.p. 1/2) iff it is 5 or 9
    assert both_10 > 0
    assert abs(one_in_10 / both_10 - 2 / 3) < 4 * math.sqrt(2 / 9 / both_10)
    four = sum(c for k, c in ours.items()
               if json.loads(k)[0][2] == 2.0 and json.loads(k)[0][1] in (5.0, 9.0))
    assert abs(four / both_10 - 0.5) < 4 * math.sqrt(0.25 / both_10)
