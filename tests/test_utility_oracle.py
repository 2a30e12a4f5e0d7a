"""The utility-analysis oracle (oracle/utility_oracle.py) against the
reference's own known answers (analysis/tests/utility_analysis_test.py,
per_partition_combiners_test.py, poisson_binomial_test.py) and the host
logic of pipelinedp_amd.analysis (no GPU)."""
import math

import numpy as np
import pytest

from oracle import utility_oracle as uo
from tests import ua_cases as uc


def _cfg(mpc, mcpp, kind="GAUSSIAN", strategy="TRUNCATED_GEOMETRIC", pre=None,
         min_sum=None, max_sum=None):
    return dict(mpc=mpc, mcpp=mcpp, noise_kind=kind, strategy=strategy, pre_threshold=pre,
                min_sum=-np.inf if min_sum is None else min_sum,
                max_sum=np.inf if max_sum is None else max_sum)


def _rows_preagg(rows, value=1.0):
    pid = [r[0] for r in rows]
    pk = [f"pk{r[1]}" for r in rows]
    return uo.preaggregate(pid, pk, [value] * len(rows))


def test_wo_public_partitions_known_answer():
    pairs = _rows_preagg(uc.WO_PUBLIC_ROWS)
    per, reports = uo.analyze(pairs, [_cfg(1, 2)], ["COUNT", "PRIVACY_ID_COUNT"], 3, 0.9,
                              "GAUSSIAN")
    assert len(reports) == 1 and len(per) == 10
    rep = reports[0]
    uc.assert_close(uc.WO_PUBLIC_EXPECTED, rep)
    (b,) = rep["utility_report_histogram"]
    assert (b["partition_size_from"], b["partition_size_to"]) == uc.WO_PUBLIC_BIN
    uc.assert_close(dict(uc.WO_PUBLIC_EXPECTED), b["report"])


@pytest.mark.parametrize("kind", ["GAUSSIAN", "LAPLACE"])
def test_w_public_partitions_noise_std(kind):
    pid = list(range(100))
    pairs = uo.preaggregate(pid, [f"pk{x}" for x in pid], [0.0] * 100, ["pk0", "pk1", "pk101"])
    _, reports = uo.analyze(pairs, [_cfg(1, 1, kind)], ["COUNT", "PRIVACY_ID_COUNT"], 2, 1e-10,
                            kind, public=["pk0", "pk1", "pk101"])
    errs = reports[0]["metric_errors"]
    assert len(errs) == 2
    for e in errs:
        assert e["noise_std"] == uc.W_PUBLIC_STD[kind]


def test_multi_parameters_known_answer():
    pairs = uo.preaggregate([0, 0, 0], ["pk0", "pk1", "pk1"], [0.0] * 3, ["pk0", "pk1"])
    _, reports = uo.analyze(pairs, [_cfg(1, 1), _cfg(2, 2)], ["COUNT"], 2, 1e-10, "GAUSSIAN",
                            public=["pk0", "pk1"])
    assert len(reports) == 2
    for i, r in enumerate(reports):
        assert r["configuration_index"] == i
        assert r["partitions_info"] == dict(public_partitions=True, num_dataset_partitions=2,
                                            num_non_public_partitions=0, num_empty_partitions=0,
                                            strategy=None, kept_partitions=None)
        (e,) = r["metric_errors"]
        assert e["metric"] == "COUNT"
        assert e["noise_std"] == uc.MULTI_STD[i]
        assert e["absolute_error"]["bounding_errors"]["l0"]["mean"] == uc.MULTI_L0_MEAN[i]


@pytest.mark.parametrize("pre", [None, 3])
def test_select_partition_probability(pre):
    pairs = _rows_preagg(uc.WO_PUBLIC_ROWS)
    per, _ = uo.analyze(pairs, [_cfg(1, 2, pre=pre)], [], 3, 0.9, "GAUSSIAN")
    prob = per[("pk0", 0)]["partition_selection_probability_to_keep"]
    assert abs(prob - uc.SELECT_PROB[pre]) < 1e-7


def test_poisson_binomial_exact_and_approximation():
    """analysis/tests/poisson_binomial_test.py: the exact PMF sums to 1 and
    matches the binomial for equal p; the refined normal approximation is
    close to the exact PMF for many pairs."""
    from scipy.stats import binom
    st, pm = uo.pmf([0.3] * 40)
    assert st == 0 and np.allclose(pm, binom.pmf(np.arange(41), 40, 0.3), atol=1e-12)
    rng = np.random.default_rng(3)
    probs = rng.uniform(0.05, 0.95, 400)
    st, approx = uo.pmf(probs)
    c = np.array([1.0])
    for p in probs:
        c = np.concatenate([c * (1 - p), [0]]) + np.concatenate([[0], c * p])
    assert abs(approx.sum() - 1) < 1e-9
    assert np.abs(c[st:st + len(approx)] - approx).max() < 1e-3


def test_bucket_bounds():
    """utility_analysis_test.py:294-315."""
    from pipelinedp_amd.analysis import utility_analysis as ua
    assert len(ua.BUCKET_BOUNDS) == 29
    assert ua.BUCKET_BOUNDS[:10] == (0, 1, 10, 20, 50, 100, 200, 500, 1000, 2000)
    for n, lo in [(-1, 0), (0, 0), (1, 1), (5, 1), (11, 10), (20, 20), (1234, 1000)]:
        assert ua._get_lower_bound(n) == lo == uo.lower_bound(n)
    for n, hi in [(-1, 0), (0, 1), (1, 10), (5, 10), (11, 20), (20, 50), (1234, 2000)]:
        assert ua._get_upper_bound(n) == hi == uo.upper_bound(n)


def test_multi_parameter_configuration_validation():
    """analysis/tests/data_structures_test.py: lengths must agree, min/max sum
    set together, at least one attribute."""
    import pipelinedp_amd as pdp
    from pipelinedp_amd import analysis
    with pytest.raises(ValueError, match="at least 1"):
        analysis.MultiParameterConfiguration()
    with pytest.raises(ValueError, match="same length"):
        analysis.MultiParameterConfiguration(max_partitions_contributed=[1, 2],
                                             max_contributions_per_partition=[1])
    with pytest.raises(ValueError, match="both set"):
        analysis.MultiParameterConfiguration(min_sum_per_partition=[1.0])
    m = analysis.MultiParameterConfiguration(max_partitions_contributed=[1, 2],
                                             noise_kind=[pdp.NoiseKind.LAPLACE,
                                                         pdp.NoiseKind.GAUSSIAN])
    p = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT], max_partitions_contributed=5,
                            max_contributions_per_partition=3)
    q = m.get_aggregate_params(p, 1)
    assert (q.max_partitions_contributed, q.max_contributions_per_partition, q.noise_kind) == \
        (2, 3, pdp.NoiseKind.GAUSSIAN)
    assert p.max_partitions_contributed == 5
    with pytest.raises(ValueError, match="partitions_sampling_prob"):
        analysis.UtilityAnalysisOptions(1, 1e-5, p, partitions_sampling_prob=0)


@pytest.mark.parametrize("case", uc.load_fixture(), ids=lambda c: c["name"])
def test_oracle_matches_reference_fixture(case):
    """tests/golden/utility_analysis.json (the reference's
    perform_utility_analysis on seeded inputs): every per-partition result
    and every report, to 1e-9 relative."""
    pairs = uo.preaggregate(case["pid"], case["pk"], case["value"], case["public"])
    per, reports = uo.analyze(pairs, uc.oracle_configs(case), case["metrics"], case["eps"],
                              case["delta"], case["noise"], public=case["public"],
                              sampled=uc.sampler(case["sampling"]))
    assert len(per) == len(case["per_partition"])
    for k, i, want in case["per_partition"]:
        uc.assert_close(want, per[(k, i)], f"per[{k},{i}]", atol=1e-9, rtol=1e-9)
    assert len(reports) == len(case["reports"])
    for want, got in zip(case["reports"], reports):
        uc.assert_close(want, got, "report", atol=1e-9, rtol=1e-9)


def test_vectorised_sweep_matches_oracle():
    """oracle/utility_sweep_np.py (the config-5 CPU baseline) reproduces the
    per-partition results of the loop restatement: keep probability (exact
    PMF and the normal approximation past 100 pairs) and every metric's
    error terms, for several configurations, serial and on 2 workers."""
    from oracle import utility_sweep_np as us
    rng = np.random.default_rng(5)
    n = 6000
    pid = rng.integers(0, 400, n)
    pk = (rng.zipf(1.3, n) - 1) % 60
    val = rng.uniform(-1.0, 6.0, n)
    metrics = ["COUNT", "SUM", "PRIVACY_ID_COUNT"]
    cfgs = [dict(mpc=a, mcpp=b, min_sum=0.0, max_sum=3.0 * b, noise_kind="LAPLACE",
                 strategy=s, pre_threshold=pre)
            for a, b, s, pre in [(1, 1, "TRUNCATED_GEOMETRIC", None), (3, 2, "TRUNCATED_GEOMETRIC", 2),
                                 (8, 4, "LAPLACE_THRESHOLDING", None),
                                 (2, 3, "GAUSSIAN_THRESHOLDING", None)]]
    pairs = uo.preaggregate(pid.tolist(), pk.tolist(), val.tolist())
    assert max(len(v) for v in pairs.values()) > uo.MAX_EXACT  # both PMF paths
    per, _ = uo.analyze(pairs, cfgs, metrics, 1.0, 1e-6, "LAPLACE")
    for workers in (1, 2):
        pa, res = us.sweep(pid, pk, val, cfgs, metrics, 1.0, 1e-6, workers=workers)
        for i in range(len(cfgs)):
            for r, k in enumerate(pa["pk"].tolist()):
                ref = per[(k, i)]
                assert res[i]["keep"][r] == pytest.approx(
                    ref["partition_selection_probability_to_keep"], rel=1e-9, abs=1e-12)
                for me in ref["metric_errors"]:
                    got = res[i][me["aggregation"]]
                    for f in ("sum", "clipping_to_min_error", "clipping_to_max_error",
                              "expected_l0_bounding_error"):
                        assert got[f][r] == pytest.approx(me[f], rel=1e-9, abs=1e-9), (i, k, f)
                    assert math.sqrt(got["var_l0_bounding_error"][r]) == pytest.approx(
                        me["std_l0_bounding_error"], rel=1e-9, abs=1e-9)
