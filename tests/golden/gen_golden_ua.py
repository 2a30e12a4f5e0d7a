"""Utility-analysis golden-vector generator (TEST INFRASTRUCTURE, build
container only).

Imports the read-only reference (/root/reference) with the PyDP stand-in in
tests/golden/pydp_stub_ua (noise std and keep probabilities restated from
oracle/mechanisms.py, which the reference's own known answers pin) and runs
analysis.perform_utility_analysis on small seeded inputs.  Writes inputs,
the per-partition results and the reports to tests/golden/utility_analysis.json.

What the fixture pins beyond the known answers of the reference's tests:
the per-partition combiners on partitions of > 100 pairs (refined normal
approximation), SUM clipping, several configurations, partition sampling,
public partitions with empty partitions, and the size histogram.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_ua.py
"""
import dataclasses
import enum
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pydp_stub_ua"))
sys.path.insert(0, "/root/reference")

import pipeline_dp  # noqa: E402  (the reference, read-only)
import analysis  # noqa: E402


def plain(x):
    if isinstance(x, pipeline_dp.Metric) if hasattr(pipeline_dp, "Metric") else False:
        return str(x)
    if dataclasses.is_dataclass(x):
        return {f.name: plain(getattr(x, f.name)) for f in dataclasses.fields(x)}
    if isinstance(x, enum.Enum):
        return x.name
    if isinstance(x, (list, tuple)):
        return [plain(v) for v in x]
    if isinstance(x, (np.floating, np.integer)):
        return x.item()
    return x


def dataset(seed, n, n_pid, n_pk, heavy=False):
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, n_pid, n)
    w = np.arange(1, n_pk + 1, dtype=np.float64) ** -1.1
    pk = rng.choice(n_pk, size=n, p=w / w.sum())
    if heavy:  # a few privacy ids with many partitions
        pid[: n // 10] = rng.integers(0, 5, n // 10)
    val = np.round(rng.uniform(-2, 8, n), 3)
    return pid, pk, val


METRIC = {"COUNT": pipeline_dp.Metrics.COUNT, "SUM": pipeline_dp.Metrics.SUM,
          "PRIVACY_ID_COUNT": pipeline_dp.Metrics.PRIVACY_ID_COUNT}


def run_case(name, seed, n, n_pid, n_pk, metrics, noise, configs, public=None,
             sampling=1.0, heavy=False, eps=2.0, delta=1e-6, pre_threshold=None):
    pid, pk, val = dataset(seed, n, n_pid, n_pk, heavy)
    params = pipeline_dp.AggregateParams(
        noise_kind=pipeline_dp.NoiseKind[noise], metrics=[METRIC[m] for m in metrics],
        max_partitions_contributed=configs["max_partitions_contributed"][0],
        max_contributions_per_partition=configs["max_contributions_per_partition"][0],
        min_sum_per_partition=(configs.get("min_sum_per_partition") or [None])[0],
        max_sum_per_partition=(configs.get("max_sum_per_partition") or [None])[0],
        pre_threshold=pre_threshold)
    kw = dict(configs)
    if "partition_selection_strategy" in kw:
        kw["partition_selection_strategy"] = [pipeline_dp.PartitionSelectionStrategy[s]
                                              for s in kw["partition_selection_strategy"]]
    multi = analysis.MultiParameterConfiguration(**kw)
    opts = analysis.UtilityAnalysisOptions(epsilon=eps, delta=delta, aggregate_params=params,
                                           multi_param_configuration=multi,
                                           partitions_sampling_prob=sampling)
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    reports, per = analysis.perform_utility_analysis(rows, pipeline_dp.LocalBackend(), opts, ex,
                                                     public_partitions=public)
    reports = [plain(r) for r in reports]
    per = [[k[0], k[1], plain(v)] for k, v in per]
    return dict(name=name, pid=pid.tolist(), pk=pk.tolist(), value=val.tolist(),
                metrics=metrics, noise=noise, configs=configs, public=public,
                sampling=sampling, eps=eps, delta=delta, pre_threshold=pre_threshold,
                reports=reports, per_partition=per)


def main():
    cases = [
        run_case("private_count_pid_3cfg", 1, 6000, 300, 60, ["COUNT", "PRIVACY_ID_COUNT"],
                 "GAUSSIAN", dict(max_partitions_contributed=[1, 3, 8],
                                  max_contributions_per_partition=[1, 2, 4])),
        run_case("private_sum_count_heavy", 2, 8000, 400, 40, ["SUM", "COUNT"], "LAPLACE",
                 dict(max_partitions_contributed=[2, 5], max_contributions_per_partition=[1, 3],
                      min_sum_per_partition=[0.0, -1.0], max_sum_per_partition=[5.0, 10.0]),
                 heavy=True),
        run_case("public_sum_pid", 3, 4000, 250, 50, ["PRIVACY_ID_COUNT", "SUM"], "GAUSSIAN",
                 dict(max_partitions_contributed=[1, 4], max_contributions_per_partition=[2, 2],
                      min_sum_per_partition=[1.0, -3.0], max_sum_per_partition=[4.0, 6.0]),
                 public=list(range(0, 70, 2))),
        run_case("private_strategies_pre", 4, 5000, 500, 30, ["COUNT"], "GAUSSIAN",
                 dict(max_partitions_contributed=[1, 2, 2],
                      max_contributions_per_partition=[1, 1, 3],
                      partition_selection_strategy=["TRUNCATED_GEOMETRIC",
                                                    "LAPLACE_THRESHOLDING",
                                                    "GAUSSIAN_THRESHOLDING"]),
                 pre_threshold=2),
        run_case("private_sampling", 5, 6000, 300, 80, ["COUNT", "SUM"], "LAPLACE",
                 dict(max_partitions_contributed=[2], max_contributions_per_partition=[2],
                      min_sum_per_partition=[0.0], max_sum_per_partition=[3.0]),
                 sampling=0.5),
    ]
    with open(os.path.join(HERE, "utility_analysis.json"), "w") as f:
        json.dump(cases, f)
    print("wrote", len(cases), "utility-analysis cases")


if __name__ == "__main__":
    main()
