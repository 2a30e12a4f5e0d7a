"""GPU dataset histograms (dpg_preaggregate + dpg_dataset_histograms through
the C ABI), private contribution bounds and parameter tuning, against the
reference's outputs (tests/golden/dataset_histograms.json) and the oracle
(oracle/hist_oracle.py) on inputs that reach every bounding kernel's leader
marking (single-wave, 256-thread and global-memory chunks)."""
import json
import os

import numpy as np
import pytest
import torch

import pipelinedp_amd as pdp
from oracle import hist_oracle
from pipelinedp_amd import dp_computations
from pipelinedp_amd import private_contribution_bounds as pcb
from pipelinedp_amd.analysis import data_structures
from pipelinedp_amd.analysis import parameter_tuning as pt
from pipelinedp_amd.analysis import utility_analysis
from pipelinedp_amd.dataset_histograms import computing_histograms as ch
from pipelinedp_amd.dataset_histograms import histograms as hist

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "dataset_histograms.json")))


def plain(hs: hist.DatasetHistograms):
    return [(h.name.value, [[b.lower, b.upper, b.count, b.sum, b.max] for b in h.bins])
            for h in (hs.l0_contributions_histogram, hs.l1_contributions_histogram,
                      hs.linf_contributions_histogram, hs.linf_sum_contributions_histogram,
                      hs.count_per_partition_histogram, hs.count_privacy_id_per_partition)]


def assert_same(got, want, tag):
    """want: [(name, bins)] -- integer histograms exact; LINF_SUM: exact
    counts, and edges / sums / maxima to 1e-9 (the pair sums, hence the min /
    max the edges come from, depend on the summation order in the last ulp,
    as the reference's own do)."""
    for (n1, b1), (n2, b2) in zip(got, want):
        assert n1 == n2
        assert len(b1) == len(b2), (tag, n1, len(b1), len(b2))
        for x, y in zip(b1, b2):
            if n1 == "linf_sum_contributions":
                assert x[2] == y[2], (tag, n1, x, y)
                for i in (0, 1, 3, 4):
                    assert x[i] == pytest.approx(y[i], rel=1e-9, abs=1e-9), (tag, n1, x, y)
            else:
                assert x == y, (tag, n1, x, y)


def columnar(pid, pk, val):
    return pdp.ColumnarData(pid=torch.as_tensor(np.asarray(pid, np.int64)).cuda(),
                            pk=torch.as_tensor(np.asarray(pk, np.int64)).cuda(),
                            value=torch.as_tensor(np.asarray(val, np.float64)).cuda())


EX = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                        value_extractor=lambda r: r[2])
EXC = pdp.DataExtractors(privacy_id_extractor="pid", partition_extractor="pk",
                         value_extractor="value")  # columnar input


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_histograms_match_reference(built, case):
    backend = pdp.MI355XBackend(device=0, seed=3)
    want = [(h["name"], h["bins"]) for h in case["histograms"]]
    (hs,) = list(ch.compute_dataset_histograms(
        columnar(case["pid"], case["pk"], case["value"]), EXC, backend))
    assert_same(plain(hs), want, case["name"] + "/columnar")
    rows = list(zip(case["pid"], case["pk"], case["value"]))
    (hs2,) = list(ch.compute_dataset_histograms(rows, EX, backend))
    assert_same(plain(hs2), want, case["name"] + "/rows")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_preaggregated_histograms_match_reference(built, case):
    backend = pdp.MI355XBackend(device=0, seed=3)
    ex = pdp.PreAggregateExtractors(partition_extractor=lambda r: r[0],
                                    preaggregate_extractor=lambda r: r[1])
    rows = [(k, tuple(v)) for k, v in case["preaggregated"]]
    (hs,) = list(ch.compute_dataset_histograms_on_preaggregated_data(rows, ex, backend))
    assert_same(plain(hs), [(h["name"], h["bins"]) for h in case["histograms_preaggregated"]],
                case["name"])


def heavy_dataset(seed=5, n=1_500_000, n_pid=40_000, n_pk=30_000):
    """Zipf partitions plus privacy ids large enough for the 256-thread
    chunk kernel (~800 records) and the global-memory kernel (6000 records
    over 4000 partitions), so every kernel's leader marking is exercised."""
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, n_pid, n)
    pk = (rng.zipf(1.2, n) - 1) % n_pk
    val = rng.uniform(-3.0, 9.0, n)
    pid[:6000] = n_pid + 1
    pk[:6000] = rng.integers(0, 4000, 6000)
    for j in range(20):
        pid[6000 + 800 * j:6000 + 800 * (j + 1)] = n_pid + 2 + j
    return pid, pk, val


def test_histograms_match_oracle_every_kernel(built):
    pid, pk, val = heavy_dataset()
    backend = pdp.MI355XBackend(device=0, seed=9)
    (hs,) = list(ch.compute_dataset_histograms(columnar(pid, pk, val), EXC, backend))
    assert_same(plain(hs), hist_oracle.dataset_histograms(pid, pk, val), "heavy")
    # the LINF_SUM bin edges are np.linspace(min, max, 10001) bit for bit
    sums = hs.linf_sum_contributions_histogram
    lw = np.linspace(sums.bins[0].lower, sums.bins[-1].upper, 10001)
    assert all(b.lower in set(lw.tolist()) for b in sums.bins)


def test_private_contribution_bounds_end_to_end(built):
    """The engine's DP l0 is a candidate bound; with a huge calculation eps
    the exponential mechanism returns the best-scoring candidate, computed
    here from the oracle's L0 histogram."""
    pid, pk, val = heavy_dataset(n=300_000, n_pid=5_000, n_pk=3_000)
    parts = list(range(0, 3_000, 2))
    keep = np.isin(pk, parts)
    (name, l0_bins), *_ = hist_oracle.dataset_histograms(pid[keep], pk[keep], val[keep])
    l0 = hist.Histogram(hist.HistogramType.L0_CONTRIBUTIONS,
                        [hist.FrequencyBin(*b) for b in l0_bins])
    for noise, delta in ((pdp.NoiseKind.LAPLACE, 0.0), (pdp.NoiseKind.GAUSSIAN, 1e-6)):
        params = pdp.CalculatePrivateContributionBoundsParams(
            aggregation_noise_kind=noise, aggregation_eps=1.0, aggregation_delta=delta,
            calculation_eps=1e6, max_partitions_contributed_upper_bound=200)
        sf = pcb.L0ScoringFunction(params, len(parts), l0)
        cands = pcb.generate_possible_contribution_bounds(200)
        best = cands[int(np.argmax(sf.scores(cands)))]
        eng = pdp.DPEngine(pdp.NaiveBudgetAccountant(1, 1e-6), pdp.MI355XBackend(device=0, seed=1))
        (res,) = list(eng.calculate_private_contribution_bounds(
            columnar(pid, pk, val), params, EXC, parts))
        assert isinstance(res, pdp.PrivateContributionBounds)
        assert res.max_partitions_contributed == best


def test_tune_over_100_candidates(built):
    """tune() with l0 x linf candidates (100 configurations: two device
    passes of the utility sweep); the stitched reports equal sweeps of the
    two halves run separately, and index_best minimises the RMSE."""
    pid, pk, val = heavy_dataset(n=200_000, n_pid=3_000, n_pk=2_000)
    backend = pdp.MI355XBackend(device=0, seed=11)
    col = columnar(pid, pk, val)
    (hs,) = list(ch.compute_dataset_histograms(col, EXC, backend))
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.LAPLACE, metrics=[pdp.Metrics.COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=1)
    opts = pt.TuneOptions(epsilon=1.0, delta=1e-6, aggregate_params=params,
                          function_to_minimize=pt.MinimizingFunction.ABSOLUTE_ERROR,
                          parameters_to_tune=pt.ParametersToTune(True, True),
                          number_of_parameter_candidates=100)
    res_col, _ = pt.tune(col, backend, hs, opts, EXC)
    (res,) = list(res_col)
    n = res.utility_analysis_parameters.size
    assert n > 64 and len(res.utility_reports) == n
    rmse = [r.metric_errors[0].absolute_error.rmse for r in res.utility_reports]
    assert res.index_best == int(np.argmin(rmse))
    cand = res.utility_analysis_parameters
    for lo, hi in ((0, 64), (64, n)):
        sub = data_structures.MultiParameterConfiguration(
            max_partitions_contributed=cand.max_partitions_contributed[lo:hi],
            max_contributions_per_partition=cand.max_contributions_per_partition[lo:hi])
        o = data_structures.UtilityAnalysisOptions(epsilon=1.0, delta=1e-6, aggregate_params=params,
                                                   multi_param_configuration=sub)
        reps, _ = utility_analysis.perform_utility_analysis(col, backend, o, EXC)
        for r_half, r_all in zip(list(reps), res.utility_reports[lo:hi]):
            a, b = r_half.metric_errors[0].absolute_error, r_all.metric_errors[0].absolute_error
            assert a.rmse == pytest.approx(b.rmse, rel=1e-9)
            assert a.bounding_errors.l0.mean == pytest.approx(b.bounding_errors.l0.mean, rel=1e-9,
                                                              abs=1e-12)
