"""Dataset-histogram golden-vector generator (TEST INFRASTRUCTURE, build
container only).

Imports the read-only reference (/root/reference) with the PyDP stand-in in
tests/golden/pydp_stub_ua and records, on small seeded inputs:
  * compute_dataset_histograms (raw rows, LocalBackend) -- all six
    histograms, including bins >= 1000 (a privacy id in > 1000 partitions,
    one with > 1000 records, partitions with > 1000 records);
  * compute_dataset_histograms_on_preaggregated_data on the reference's own
    pre-aggregation of the same rows (analysis/pre_aggregation.py);
  * the exponential-mechanism probabilities of L0ScoringFunction over
    generate_possible_contribution_bounds (Laplace and Gaussian) -- the
    draw itself is random, its distribution is what is pinned;
  * parameter_tuning._find_candidate_parameters for every tunable pair.
Writes tests/golden/dataset_histograms.json.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_hist.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pydp_stub_ua"))
sys.path.insert(0, "/root/reference")

import pipeline_dp  # noqa: E402  (the reference, read-only)
from pipeline_dp import private_contribution_bounds as pcb  # noqa: E402
from pipeline_dp.dataset_histograms import computing_histograms as ch  # noqa: E402
from analysis import parameter_tuning as pt  # noqa: E402
from analysis import pre_aggregation  # noqa: E402


def dataset(seed, n, n_pid, n_pk, heavy):
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, n_pid, n)
    w = np.arange(1, n_pk + 1, dtype=np.float64) ** -1.1
    pk = rng.choice(n_pk, size=n, p=w / w.sum())
    val = np.round(rng.uniform(-2, 8, n), 3)
    if heavy:
        # privacy id 0: 1500 records over up to 1200 partitions (L0, L1 >= 1000)
        pid[:1500] = 0
        pk[:1500] = rng.permutation(np.arange(1500) % 1200)
    return pid, pk, val


def plain_hist(h):
    return dict(name=h.name.value, bins=[[b.lower, b.upper, b.count, b.sum, b.max]
                                         for b in h.bins])


def plain_all(hs):
    return [plain_hist(h) for h in (hs.l0_contributions_histogram, hs.l1_contributions_histogram,
                                    hs.linf_contributions_histogram,
                                    hs.linf_sum_contributions_histogram,
                                    hs.count_per_partition_histogram,
                                    hs.count_privacy_id_per_partition)]


def run_case(name, seed, n, n_pid, n_pk, heavy=False):
    pid, pk, val = dataset(seed, n, n_pid, n_pk, heavy)
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    backend = pipeline_dp.LocalBackend()
    (hs,) = list(ch.compute_dataset_histograms(rows, ex, backend))
    pre = list(pre_aggregation.preaggregate(rows, backend, ex))
    pre_ex = pipeline_dp.PreAggregateExtractors(partition_extractor=lambda r: r[0],
                                                preaggregate_extractor=lambda r: r[1])
    (hs_pre,) = list(ch.compute_dataset_histograms_on_preaggregated_data(pre, pre_ex, backend))
    n_partitions = len(set(pk.tolist()))
    bounds = []
    for noise, eps, delta, cal_eps, ub in (("LAPLACE", 1.0, 0.0, 0.5, 100),
                                           ("GAUSSIAN", 2.0, 1e-5, 1.0, 2000),
                                           ("LAPLACE", 0.3, 0.0, 3.0, 10)):
        params = pipeline_dp.CalculatePrivateContributionBoundsParams(
            aggregation_noise_kind=pipeline_dp.NoiseKind[noise], aggregation_eps=eps,
            aggregation_delta=delta, calculation_eps=cal_eps,
            max_partitions_contributed_upper_bound=ub)
        sf = pcb.L0ScoringFunction(params, n_partitions, hs.l0_contributions_histogram)
        cands = pcb.generate_possible_contribution_bounds(
            sf._max_partitions_contributed_best_upper_bound())
        probs = pipeline_dp.dp_computations.ExponentialMechanism(sf)._calculate_probabilities(
            cal_eps, cands)
        bounds.append(dict(noise=noise, eps=eps, delta=delta, calculation_eps=cal_eps,
                           upper_bound=ub, n_partitions=n_partitions, candidates=cands,
                           probabilities=[float(p) for p in probs]))
    tuning = []
    for metric, to_tune, max_c in (("COUNT", (True, True, False, False), 100),
                                   ("COUNT", (True, False, False, False), 30),
                                   ("COUNT", (False, True, False, False), 20),
                                   ("SUM", (True, False, False, True), 100),
                                   ("SUM", (False, False, False, True), 16),
                                   ("PRIVACY_ID_COUNT", (True, False, False, False), 50)):
        ptt = pt.ParametersToTune(*to_tune)
        c = pt._find_candidate_parameters(hs, ptt, pipeline_dp.Metrics.__dict__[metric], max_c)
        tuning.append(dict(metric=metric, to_tune=list(to_tune), max_candidates=max_c,
                           max_partitions_contributed=c.max_partitions_contributed,
                           max_contributions_per_partition=c.max_contributions_per_partition,
                           min_sum_per_partition=c.min_sum_per_partition,
                           max_sum_per_partition=c.max_sum_per_partition))
    return dict(name=name, pid=pid.tolist(), pk=pk.tolist(), value=val.tolist(),
                histograms=plain_all(hs), preaggregated=[[k, list(v)] for k, v in pre],
                histograms_preaggregated=plain_all(hs_pre), contribution_bounds=bounds,
                tuning=tuning)


def main():
    cases = [run_case("zipf_small", 11, 3000, 200, 80),
             run_case("heavy_ids", 12, 12000, 300, 1500, heavy=True)]
    with open(os.path.join(HERE, "dataset_histograms.json"), "w") as f:
        json.dump(cases, f)
    print("wrote", len(cases), "dataset-histogram cases")


if __name__ == "__main__":
    main()
