"""GPU utility analysis (pipelinedp_amd.analysis, through libdpg's
dpg_preaggregate + dpg_utility_analysis) against the reference's own known
answers, the reference fixture tests/golden/utility_analysis.json and the
oracle (oracle/utility_oracle.py) on larger sweeps."""
import numpy as np
import pytest
import torch

import pipelinedp_amd as pdp
from pipelinedp_amd import analysis
from oracle import utility_oracle as uo
from tests import ua_cases as uc

pytestmark = pytest.mark.gpu

M = {"COUNT": pdp.Metrics.COUNT, "SUM": pdp.Metrics.SUM,
     "PRIVACY_ID_COUNT": pdp.Metrics.PRIVACY_ID_COUNT}


def _backend():
    return pdp.MI355XBackend(device=0, seed=7)


def _run(col, options, extractors, public=None):
    reports, per = analysis.perform_utility_analysis(col, _backend(), options, extractors,
                                                     public_partitions=public)
    return [uc.to_plain(r) for r in reports], {k: uc.to_plain(v) for k, v in per}


def test_wo_public_partitions_known_answer(built):
    """analysis/tests/utility_analysis_test.py:59-195 (both input forms)."""
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.GAUSSIAN,
                                 metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=2)
    opts = analysis.UtilityAnalysisOptions(epsilon=3, delta=0.9, aggregate_params=params)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda x: x[0],
                            partition_extractor=lambda x: f"pk{x[1]}",
                            value_extractor=lambda x: 1)
    reports, per = _run(uc.WO_PUBLIC_ROWS, opts, ex)
    assert len(reports) == 1 and len(per) == 10
    uc.assert_close(uc.WO_PUBLIC_EXPECTED, reports[0])
    (b,) = reports[0]["utility_report_histogram"]
    assert (b["partition_size_from"], b["partition_size_to"]) == uc.WO_PUBLIC_BIN
    # pre-aggregated form: (partition_key, (count, sum, n_partitions))
    opts2 = analysis.UtilityAnalysisOptions(epsilon=3, delta=0.9, aggregate_params=params,
                                            pre_aggregated_data=True)
    col = [(i, (3, 1, 10)) for i in range(10)] * 10
    ex2 = pdp.PreAggregateExtractors(partition_extractor=lambda x: f"pk{x[0]}",
                                     preaggregate_extractor=lambda x: x[1])
    reports2, per2 = _run(col, opts2, ex2)
    uc.assert_close(uc.WO_PUBLIC_EXPECTED, reports2[0])
    assert len(per2) == 10


@pytest.mark.parametrize("kind", ["GAUSSIAN", "LAPLACE"])
def test_w_public_partitions_noise_std(built, kind):
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind[kind],
                                 metrics=[pdp.Metrics.COUNT, pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=1)
    opts = analysis.UtilityAnalysisOptions(epsilon=2, delta=1e-10, aggregate_params=params)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda x: x, partition_extractor=lambda x: f"pk{x}",
                            value_extractor=lambda x: 0)
    reports, _ = _run(list(range(100)), opts, ex, public=["pk0", "pk1", "pk101"])
    errs = reports[0]["metric_errors"]
    assert len(errs) == 2
    assert all(e["noise_std"] == uc.W_PUBLIC_STD[kind] for e in errs)


def test_multi_parameters_known_answer(built):
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.GAUSSIAN, metrics=[pdp.Metrics.COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=1)
    multi = analysis.MultiParameterConfiguration(max_partitions_contributed=[1, 2],
                                                 max_contributions_per_partition=[1, 2])
    opts = analysis.UtilityAnalysisOptions(epsilon=2, delta=1e-10, aggregate_params=params,
                                           multi_param_configuration=multi)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda x: x[0], partition_extractor=lambda x: x[1],
                            value_extractor=lambda x: 0)
    reports, _ = _run([(0, "pk0"), (0, "pk1"), (0, "pk1")], opts, ex, public=["pk0", "pk1"])
    assert len(reports) == 2
    for i, r in enumerate(reports):
        assert r["configuration_index"] == i
        assert r["partitions_info"] == dict(public_partitions=True, num_dataset_partitions=2,
                                            num_non_public_partitions=0, num_empty_partitions=0,
                                            strategy=None, kept_partitions=None)
        (e,) = r["metric_errors"]
        assert e["metric"] == "COUNT" and e["noise_std"] == uc.MULTI_STD[i]
        assert e["absolute_error"]["bounding_errors"]["l0"]["mean"] == uc.MULTI_L0_MEAN[i]


@pytest.mark.parametrize("pre", [None, 3])
def test_select_partition_probability(built, pre):
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.GAUSSIAN, metrics=[],
                                 max_partitions_contributed=1, max_contributions_per_partition=2,
                                 pre_threshold=pre)
    opts = analysis.UtilityAnalysisOptions(epsilon=3, delta=0.9, aggregate_params=params)
    ex = pdp.DataExtractors(privacy_id_extractor=lambda x: x[0],
                            partition_extractor=lambda x: f"pk{x[1]}", value_extractor=lambda x: 1)
    _, per = _run(uc.WO_PUBLIC_ROWS, opts, ex)
    prob = per[("pk0", 0)]["partition_selection_probability_to_keep"]
    assert abs(prob - uc.SELECT_PROB[pre]) < 1e-7


def _case_options(case):
    cfg = dict(case["configs"])
    if "partition_selection_strategy" in cfg:
        cfg["partition_selection_strategy"] = [pdp.PartitionSelectionStrategy[s]
                                               for s in cfg["partition_selection_strategy"]]
    first = lambda k: (case["configs"].get(k) or [None])[0]
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind[case["noise"]],
                                 metrics=[M[m] for m in case["metrics"]],
                                 max_partitions_contributed=first("max_partitions_contributed"),
                                 max_contributions_per_partition=first(
                                     "max_contributions_per_partition"),
                                 min_sum_per_partition=first("min_sum_per_partition"),
                                 max_sum_per_partition=first("max_sum_per_partition"),
                                 pre_threshold=case["pre_threshold"])
    return analysis.UtilityAnalysisOptions(
        epsilon=case["eps"], delta=case["delta"], aggregate_params=params,
        multi_param_configuration=analysis.MultiParameterConfiguration(**cfg),
        partitions_sampling_prob=case["sampling"])


@pytest.mark.parametrize("case", uc.load_fixture(), ids=lambda c: c["name"])
def test_matches_reference_fixture(built, case):
    """Every per-partition result and report of the reference's
    perform_utility_analysis on the fixture's inputs (row input, integer
    keys): GPU within 1e-7."""
    rows = list(zip(case["pid"], case["pk"], case["value"]))
    ex = pdp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                            partition_extractor=lambda r: r[1], value_extractor=lambda r: r[2])
    reports, per = _run(rows, _case_options(case), ex, public=case["public"])
    assert len(per) == len(case["per_partition"])
    for k, i, want in case["per_partition"]:
        uc.assert_close(want, per[(k, i)], f"per[{k},{i}]", atol=1e-7, rtol=1e-7)
    assert len(reports) == len(case["reports"])
    for want, got in zip(case["reports"], reports):
        uc.assert_close(want, got, "report", atol=1e-7, rtol=1e-7)


def _grid_configs(n_side):
    vals = [2**i for i in range(n_side)]
    mpc = [a for a in vals for _ in vals]
    mcpp = [b for _ in vals for b in vals]
    return mpc, mcpp


@pytest.mark.parametrize("public", [False, True], ids=["private", "public"])
def test_64_config_sweep_matches_oracle(built, public):
    """Config-5 shape (64 configurations: mpc x mcpp in {1..128}^2) on 2e5
    records: both partition regimes of the Poisson-binomial (exact <= 100
    pairs, refined normal approximation beyond), SUM + COUNT +
    PRIVACY_ID_COUNT; every per-partition value and report within 1e-7."""
    rng = np.random.default_rng(55)
    n, n_pid, P = 200_000, 4_000, 300
    pid = rng.integers(0, n_pid, n)
    w = np.arange(1, P + 1, dtype=np.float64) ** -1.1
    pk = rng.choice(P, size=n, p=w / w.sum())
    val = rng.uniform(-1, 6, n)
    mpc, mcpp = _grid_configs(8)
    multi = analysis.MultiParameterConfiguration(
        max_partitions_contributed=mpc, max_contributions_per_partition=mcpp,
        min_sum_per_partition=[0.0] * 64, max_sum_per_partition=[float(b) for b in mcpp])
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.LAPLACE,
                                 metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_sum_per_partition=0.0, max_sum_per_partition=1.0)
    opts = analysis.UtilityAnalysisOptions(epsilon=1.0, delta=1e-6, aggregate_params=params,
                                           multi_param_configuration=multi)
    pub = list(range(0, P + 20, 3)) if public else None
    cols = pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                            value=torch.as_tensor(val), n_partitions=P + 20)
    reports, per = _run(cols, opts, pdp.DataExtractors("pid", "pk", "value"), public=pub)
    cfgs = [dict(mpc=a, mcpp=b, min_sum=0.0, max_sum=float(b), noise_kind="LAPLACE",
                 strategy="TRUNCATED_GEOMETRIC", pre_threshold=None) for a, b in zip(mpc, mcpp)]
    pairs = uo.preaggregate(pid.tolist(), pk.tolist(), val.tolist(), pub)
    assert max(len(v) for v in pairs.values()) > 100 and min(len(v) for v in pairs.values()) < 100
    want_per, want_rep = uo.analyze(pairs, cfgs, ["COUNT", "SUM", "PRIVACY_ID_COUNT"], 1.0, 1e-6,
                                    "LAPLACE", public=pub)
    assert set(per) == set(want_per)
    for key, want in want_per.items():
        uc.assert_close(want, per[key], f"per{key}", atol=1e-7, rtol=1e-7)
    for want, got in zip(want_rep, reports):
        uc.assert_close(want, got, "report", atol=1e-7, rtol=1e-7)


def _sorted_pairs(ps):
    from pipelinedp_amd import pre_aggregation as pa
    a = pa.to_numpy(ps)
    nc = a["ncl"] & pa.NC_MASK
    return a[np.lexsort((nc, a["np"], a["sum"], a["count"], a["pk"]))], ps.starts.cpu()


@pytest.mark.parametrize("exact", [True, False], ids=["quarter_values", "uniform_values"])
def test_preaggregate_value_records_match_gather_path(built, exact, monkeypatch):
    """dpg_preaggregate carries the value inside 16-byte records through the
    partition levels (R16); DPG_PA_GATHER=1 keeps 8-byte records and gathers
    each value by record index.  Both must produce the same pairs: counts,
    partition / contribution counts bit-exact, one leader pair per privacy id
    in each (which pair leads follows the record order, so it may differ),
    sums exact for quarter-integer values (any summation order) and within
    1e-12 relative otherwise."""
    from pipelinedp_amd import pre_aggregation as pa
    rng = np.random.default_rng(77 + exact)
    n, n_pid, P = 1_500_000, 30_000, 5_000
    pid = rng.integers(0, n_pid, n)
    w = np.arange(1, P + 1, dtype=np.float64) ** -1.05
    pk = rng.choice(P, size=n, p=w / w.sum())
    val = rng.integers(-8, 40, n) * 0.25 if exact else rng.uniform(-1, 6, n)
    cols = pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                            value=torch.as_tensor(val), n_partitions=P)
    ex = pdp.DataExtractors("pid", "pk", "value")
    be = pdp.MI355XBackend(device=0, seed=5)
    dev = torch.device("cuda", 0)
    monkeypatch.delenv("DPG_PA_GATHER", raising=False)
    got, gs = _sorted_pairs(pa.device_pairs(cols, ex, be, None, dev))
    monkeypatch.setenv("DPG_PA_GATHER", "1")
    want, ws = _sorted_pairs(pa.device_pairs(cols, ex, be, None, dev))
    assert torch.equal(gs, ws)
    assert len(got) == len(want) == len(np.unique(pid * P + pk))
    for f in ("pk", "count", "np"):
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)
    np.testing.assert_array_equal(got["ncl"] & pa.NC_MASK, want["ncl"] & pa.NC_MASK)
    assert int((got["ncl"] >> 31).sum()) == int((want["ncl"] >> 31).sum()) == len(np.unique(pid))
    if exact:
        np.testing.assert_array_equal(got["sum"], want["sum"])
    else:
        np.testing.assert_allclose(got["sum"], want["sum"], rtol=1e-12, atol=1e-9)


def test_64_config_sweep_with_partition_sampling_matches_oracle(built):
    """The 64-configuration sweep with partitions_sampling_prob = 0.5:
    sampled-out partitions are skipped by the accumulate (their rows are
    neither written nor, being outside the output, read -- including rows
    of partitions split between accumulate runs, which the sweep zeroes
    without a full fill), by the selection and by the report; per-partition
    values and reports equal the oracle's on the sampled set within 1e-7."""
    from pipelinedp_amd.analysis import utility_analysis as ua_mod
    rng = np.random.default_rng(56)
    n, n_pid, P = 200_000, 4_000, 300
    pid = rng.integers(0, n_pid, n)
    w = np.arange(1, P + 1, dtype=np.float64) ** -1.1
    pk = rng.choice(P, size=n, p=w / w.sum())
    val = rng.uniform(-1, 6, n)
    mpc, mcpp = _grid_configs(8)
    multi = analysis.MultiParameterConfiguration(
        max_partitions_contributed=mpc, max_contributions_per_partition=mcpp,
        min_sum_per_partition=[0.0] * 64, max_sum_per_partition=[float(b) for b in mcpp])
    params = pdp.AggregateParams(noise_kind=pdp.NoiseKind.LAPLACE,
                                 metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_sum_per_partition=0.0, max_sum_per_partition=1.0)
    prob = 0.5
    opts = analysis.UtilityAnalysisOptions(epsilon=1.0, delta=1e-6, aggregate_params=params,
                                           multi_param_configuration=multi,
                                           partitions_sampling_prob=prob)
    cols = pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                            value=torch.as_tensor(val), n_partitions=P)
    reports, per = _run(cols, opts, pdp.DataExtractors("pid", "pk", "value"))
    bound = ua_mod._sample_bound(prob)
    keep = lambda k: ua_mod._keep_by_hash(k, bound)
    cfgs = [dict(mpc=a, mcpp=b, min_sum=0.0, max_sum=float(b), noise_kind="LAPLACE",
                 strategy="TRUNCATED_GEOMETRIC", pre_threshold=None) for a, b in zip(mpc, mcpp)]
    pairs = uo.preaggregate(pid.tolist(), pk.tolist(), val.tolist(), None)
    # partitions split between runs of 1024 pairs, sampled in and out
    assert sum(len(v) > 1024 for k, v in pairs.items() if keep(k)) > 0
    assert sum(len(v) > 1024 for k, v in pairs.items() if not keep(k)) > 0
    want_per, want_rep = uo.analyze(pairs, cfgs, ["COUNT", "SUM", "PRIVACY_ID_COUNT"], 1.0, 1e-6,
                                    "LAPLACE", sampled=keep)
    assert set(per) == set(want_per) and len(want_per) > 0
    for key, want in want_per.items():
        uc.assert_close(want, per[key], f"per{key}", atol=1e-7, rtol=1e-7)
    for want, got in zip(want_rep, reports):
        uc.assert_close(want, got, "report", atol=1e-7, rtol=1e-7)
