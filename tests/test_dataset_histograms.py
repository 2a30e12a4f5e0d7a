"""CPU tests of the dataset histograms, the private contribution bounds and
parameter-tuning candidates: the oracle and the host logic against the
reference's outputs (tests/golden/dataset_histograms.json, written by
tests/golden/gen_golden_hist.py from the reference itself)."""
import json
import math
import os

import numpy as np
import pytest

import pipelinedp_amd as pdp
from oracle import hist_oracle
from pipelinedp_amd import dp_computations
from pipelinedp_amd import private_contribution_bounds as pcb
from pipelinedp_amd.dataset_histograms import computing_histograms as ch
from pipelinedp_amd.dataset_histograms import histograms as hist

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "dataset_histograms.json")))
T = hist.HistogramType


def assert_bins_equal(got, want, tag):
    """got: [(name, [[lower, upper, count, sum, max]])], want: fixture list."""
    for (name, bins), h in zip(got, want):
        assert name == h["name"]
        assert len(bins) == len(h["bins"]), (tag, name)
        for x, y in zip(bins, h["bins"]):
            assert (x[0], x[1], x[2], x[4]) == (y[0], y[1], y[2], y[4]), (tag, name, x, y)
            assert x[3] == pytest.approx(y[3], rel=1e-9, abs=1e-9), (tag, name, x, y)


def to_histogram(h) -> hist.Histogram:
    return hist.Histogram(T(h["name"]), [hist.FrequencyBin(*b) for b in h["bins"]])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_raw(case):
    got = hist_oracle.dataset_histograms(case["pid"], case["pk"], case["value"])
    assert_bins_equal(got, case["histograms"], case["name"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_preaggregated(case):
    got = hist_oracle.dataset_histograms_preaggregated(case["preaggregated"])
    assert_bins_equal(got, case["histograms_preaggregated"], case["name"])


def device_int_bin(v: int) -> int:
    """Restatement of dpg_hist.h int_bin (the index the kernels use)."""
    if v < 1000:
        return v
    p, e = 10, 0
    while e < 16 and v // p >= 1000:
        p, e = p * 10, e + 1
    return 1000 + 900 * e + v // p - 100


def test_int_bin_decode_matches_reference_rule():
    vals = list(range(1, 3000)) + [9999, 10000, 10001, 10099, 10100, 99999, 100000, 123456789,
                                   2**32 - 1, 10**15 + 7, 2**63 - 1]
    idx = np.array([device_int_bin(v) for v in vals])
    lower, upper = ch.int_bin_bounds(idx)
    for v, lo, up in zip(vals, lower, upper):
        assert (lo, up) == ch._to_bin_lower_upper_logarithmic(v) == hist_oracle.int_lower_upper(v), v
        assert lo <= v < up


def test_int_bins_cover_uint64():
    from pipelinedp_amd import _native
    assert device_int_bin(2**64 - 1) < _native.HIST_INT_BINS


def test_generate_possible_contribution_bounds():
    b = pcb.generate_possible_contribution_bounds(12345)
    assert b[:3] == [1, 2, 3] and 999 in b and 1000 in b and 1010 in b and 1005 not in b
    assert b[-1] == 12300 and all(x < y for x, y in zip(b, b[1:]))
    # the candidates are exactly the integer bin lowers
    assert all(ch._to_bin_lower_upper_logarithmic(x)[0] == x for x in b)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_l0_scoring_probabilities_match_reference(case):
    l0 = to_histogram(case["histograms"][0])
    for b in case["contribution_bounds"]:
        params = pdp.CalculatePrivateContributionBoundsParams(
            aggregation_noise_kind=pdp.NoiseKind[b["noise"]], aggregation_eps=b["eps"],
            aggregation_delta=b["delta"], calculation_eps=b["calculation_eps"],
            max_partitions_contributed_upper_bound=b["upper_bound"])
        sf = pcb.L0ScoringFunction(params, b["n_partitions"], l0)
        cands = pcb.generate_possible_contribution_bounds(
            sf._max_partitions_contributed_best_upper_bound())
        assert cands == b["candidates"]
        p = dp_computations.ExponentialMechanism(sf)._calculate_probabilities(
            b["calculation_eps"], cands)
        assert np.isfinite(p).all() and p.sum() == pytest.approx(1.0)
        ref = np.array(b["probabilities"], dtype=np.float64)
        if np.isfinite(ref).all():
            np.testing.assert_allclose(p, ref, rtol=1e-9, atol=1e-300)
        # else: every reference weight underflowed (0 / 0); ours is the
        # stable form of the same distribution -- most mass on the best score
        assert sf.score(cands[int(np.argmax(p))]) == pytest.approx(
            max(sf.score(k) for k in cands))


def test_exponential_mechanism_draw_distribution():
    """The draw follows the probabilities (chi-square over 20000 draws)."""
    from scipy import stats

    class S(dp_computations.ExponentialMechanism.ScoringFunction):
        def score(self, k):
            return -abs(k - 3)

        global_sensitivity = 1.0
        is_monotonic = False

    em = dp_computations.ExponentialMechanism(S())
    cands = [1, 2, 3, 4, 5, 6]
    p = em._calculate_probabilities(1.5, cands)
    draws = [em.apply(1.5, cands) for _ in range(20000)]
    obs = np.array([draws.count(c) for c in cands])
    assert stats.chisquare(obs, p * len(draws)).pvalue > 1e-4


def test_histogram_quantiles_and_ratio_dropped():
    h = hist.Histogram(T.L0_CONTRIBUTIONS, [hist.FrequencyBin(1, 2, 5, 5, 1),
                                            hist.FrequencyBin(2, 3, 3, 6, 2),
                                            hist.FrequencyBin(10, 11, 2, 20, 10)])
    assert h.lower == 1 and h.upper is None and h.total_count() == 10 and h.max_value() == 10
    assert h.quantiles([0.1, 0.5, 0.9]) == [1, 2, 10]
    r = dict(hist.compute_ratio_dropped(h))
    assert r[0] == 1 and r[10] == 0 and r[2] == pytest.approx(16 / 31) and r[1] == pytest.approx(21 / 31)


def test_calculate_private_contribution_bounds_argument_errors():
    eng = pdp.DPEngine(pdp.NaiveBudgetAccountant(1, 1e-6), pdp.MI355XBackend(device=0, seed=1))
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                            value_extractor=lambda r: 0)
    with pytest.raises(ValueError):
        eng.calculate_private_contribution_bounds([], None, ex, [1])
    with pytest.raises(TypeError):
        eng.calculate_private_contribution_bounds([(1, 1)], object(), ex, [1])
    with pytest.raises(ValueError):
        pdp.CalculatePrivateContributionBoundsParams(pdp.NoiseKind.GAUSSIAN, 1.0, 0.0, 1.0, 10)
    with pytest.raises(ValueError):
        pdp.CalculatePrivateContributionBoundsParams(pdp.NoiseKind.LAPLACE, 1.0, 0.0, 1.0, 0)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_tuning_candidates_match_reference(case):
    from pipelinedp_amd.analysis import parameter_tuning as pt
    hs = hist.DatasetHistograms(*[to_histogram(h) for h in case["histograms"]])
    for t in case["tuning"]:
        c = pt._find_candidate_parameters(hs, pt.ParametersToTune(*t["to_tune"]),
                                          getattr(pdp.Metrics, t["metric"]), t["max_candidates"])
        assert c.max_partitions_contributed == t["max_partitions_contributed"]
        assert c.max_contributions_per_partition == t["max_contributions_per_partition"]
        assert c.min_sum_per_partition == t["min_sum_per_partition"]
        assert c.max_sum_per_partition == t["max_sum_per_partition"]


def test_tune_argument_checks():
    from pipelinedp_amd.analysis import parameter_tuning as pt
    p = pdp.AggregateParams(metrics=[pdp.Metrics.MEAN], max_partitions_contributed=1,
                            max_contributions_per_partition=1, min_value=0, max_value=1)
    opts = pt.TuneOptions(1.0, 1e-6, p, pt.MinimizingFunction.ABSOLUTE_ERROR,
                          pt.ParametersToTune(max_partitions_contributed=True))
    with pytest.raises(ValueError):
        pt._check_tune_args(opts, False)
    with pytest.raises(ValueError):
        pt.ParametersToTune()
    p2 = pdp.AggregateParams(metrics=[], max_partitions_contributed=1,
                             max_contributions_per_partition=1)
    opts2 = pt.TuneOptions(1.0, 1e-6, p2, pt.MinimizingFunction.ABSOLUTE_ERROR,
                           pt.ParametersToTune(max_partitions_contributed=True))
    with pytest.raises(ValueError):
        pt._check_tune_args(opts2, True)
