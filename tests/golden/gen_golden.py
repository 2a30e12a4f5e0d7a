"""Golden-vector generator (TEST INFRASTRUCTURE, build container only).

Imports the read-only reference PipelineDP from /root/reference together with
the test-only no-noise PyDP stand-in in tests/golden/pydp_stub, runs
`DPEngine.aggregate` / `select_partitions` on small seeded inputs, and writes
the inputs and the reference's outputs as fixtures under tests/golden/.

Nothing here is imported by the product, `smoke()` or `bench.py`, and the GPU
box never runs it: it only reads the committed fixture files.

What the fixtures pin (reference call sites in parentheses):
  * pre-noise aggregates with non-binding contribution bounds, for every
    combiner and bounding mode on the hot path
    (dp_engine.py:101-176, contribution_bounders.py:56-195,
     combiners.py:241-529, 640-739, 791-858);
  * the MetricsTuple field order per metric set (combiners.py:682-689, 708-730);
  * the budget split per metric set x noise kind after compute_budgets()
    (budget_accounting.py:333-408, combiners.py:791-858, dp_engine.py:322);
  * the empirical distribution of the reference's sampling-based bounding on
    tiny inputs where bounding triggers (LocalBackend sample_fixed_per_key,
    pipeline_backend.py:531-547), for chi-square parity tests.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pydp_stub"))
sys.path.insert(0, "/root/reference")

import pipeline_dp  # noqa: E402  (the reference, read-only)
from pipeline_dp import budget_accounting  # noqa: E402

M = pipeline_dp.Metrics


def _metric_names(metrics):
    return [str(m) for m in metrics]


def run_reference_aggregate(pid, pk, val, params_kwargs, public_partitions=None,
                            eps=1.0, delta=1e-6):
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    backend = pipeline_dp.LocalBackend()
    acc = pipeline_dp.NaiveBudgetAccountant(eps, delta)
    engine = pipeline_dp.DPEngine(acc, backend)
    params = pipeline_dp.AggregateParams(**params_kwargs)
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    res = engine.aggregate(rows, params, ex, public_partitions=public_partitions)
    acc.compute_budgets()
    out = list(res)
    out.sort(key=lambda kv: kv[0])
    fields = list(out[0][1]._fields) if out else []
    keys = np.array([k for k, _ in out], dtype=np.int64)
    cols = {f: np.array([float(getattr(m, f)) for _, m in out], dtype=np.float64)
            for f in fields}
    return keys, fields, cols


def _params_to_json(kw):
    out = {}
    for k, v in kw.items():
        if k == "metrics":
            out[k] = _metric_names(v)
        elif isinstance(v, (pipeline_dp.NoiseKind,
                            pipeline_dp.PartitionSelectionStrategy)):
            out[k] = v.name
        else:
            out[k] = v
    return out


def write_case(name, pid, pk, val, kw, public_partitions=None):
    keys, fields, cols = run_reference_aggregate(pid, pk, val, kw,
                                                 public_partitions)
    arrays = dict(pid=pid.astype(np.int64), pk=pk.astype(np.int64),
                  value=val.astype(np.float64), out_keys=keys)
    for f in fields:
        arrays["out_" + f] = cols[f]
    if public_partitions is not None:
        arrays["public_partitions"] = np.array(sorted(public_partitions),
                                               dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, f"agg_{name}.npz"), **arrays)
    meta = dict(name=name, params=_params_to_json(kw), fields=fields,
                n_records=int(len(pid)), n_out=int(len(keys)),
                public=public_partitions is not None)
    return meta


def synthetic(seed, n, n_pid, n_pk, vlo, vhi, zipf=1.1, integer_values=False):
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, n_pid, n)
    ranks = np.arange(1, n_pk + 1, dtype=np.float64)
    w = ranks ** (-zipf)
    w /= w.sum()
    pk = rng.choice(n_pk, size=n, p=w)
    if integer_values:
        val = rng.integers(int(vlo), int(vhi) + 1, n).astype(np.float64)
    else:
        val = rng.uniform(vlo, vhi, n)
    return pid, pk, val


def nonbinding(pid, pk):
    """Bounds that never trigger sampling for this input."""
    pairs = {}
    per_pid = {}
    for a, b in zip(pid.tolist(), pk.tolist()):
        pairs[(a, b)] = pairs.get((a, b), 0) + 1
        per_pid.setdefault(a, set()).add(b)
    mcpp = max(pairs.values())
    mpc = max(len(s) for s in per_pid.values())
    per_pid_total = {}
    for a in pid.tolist():
        per_pid_total[a] = per_pid_total.get(a, 0) + 1
    return mpc, mcpp, max(per_pid_total.values())


def parse_movie_file(path):
    pid, pk, val = [], [], []
    movie = None
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        if line.endswith(":"):
            movie = int(line[:-1])
        else:
            u, r, _ = line.split(",")
            pid.append(int(u))
            pk.append(movie)
            val.append(float(r))
    return (np.array(pid, np.int64), np.array(pk, np.int64),
            np.array(val, np.float64))


def gen_aggregate_cases():
    metas = []
    # a/b: COUNT+SUM+PRIVACY_ID_COUNT, values inside / outside the bounds.
    pid, pk, val = synthetic(1, 6000, 300, 200, 0.0, 10.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    kw = dict(metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=0.0, max_value=10.0)
    metas.append(write_case("count_sum_pid", pid, pk, val, kw))
    pid, pk, val = synthetic(2, 6000, 250, 150, -5.0, 15.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    kw = dict(metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=0.0, max_value=10.0)
    metas.append(write_case("count_sum_pid_clip", pid, pk, val, kw))
    # c: MEAN + VARIANCE (+COUNT, SUM) with Laplace and Gaussian.
    pid, pk, val = synthetic(3, 5000, 200, 120, -2.0, 7.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    for noise in (pipeline_dp.NoiseKind.LAPLACE, pipeline_dp.NoiseKind.GAUSSIAN):
        kw = dict(metrics=[M.COUNT, M.SUM, M.MEAN, M.VARIANCE],
                  noise_kind=noise,
                  max_partitions_contributed=mpc,
                  max_contributions_per_partition=mcpp,
                  min_value=-1.0, max_value=5.0)
        metas.append(write_case(f"mean_var_{noise.name.lower()}", pid, pk,
                                val, kw))
    kw = dict(metrics=[M.MEAN, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=-1.0, max_value=5.0)
    metas.append(write_case("mean_pid", pid, pk, val, kw))
    # d: SUM with per-partition bounds (CrossPartition bounder).
    pid, pk, val = synthetic(4, 5000, 220, 100, -3.0, 6.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    kw = dict(metrics=[M.SUM, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_sum_per_partition=-4.0, max_sum_per_partition=9.0)
    metas.append(write_case("sum_per_partition", pid, pk, val, kw))
    kw = dict(metrics=[M.COUNT, M.SUM],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_sum_per_partition=-4.0, max_sum_per_partition=9.0)
    metas.append(write_case("count_sum_per_partition", pid, pk, val, kw))
    # e: max_contributions (PerPrivacyId bounder).
    pid, pk, val = synthetic(5, 5000, 260, 90, 0.0, 4.0)
    _, _, l1 = nonbinding(pid, pk)
    kw = dict(metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT, M.MEAN],
              max_contributions=l1, min_value=0.0, max_value=3.0)
    metas.append(write_case("max_contributions", pid, pk, val, kw))
    # f: public partitions (half of the data partitions + absent ones).
    pid, pk, val = synthetic(6, 5000, 240, 100, 0.0, 10.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    public = list(range(0, 100, 2)) + list(range(1000, 1010))
    kw = dict(metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=0.0, max_value=10.0)
    metas.append(write_case("public_partitions", pid, pk, val, kw, public))
    kw = dict(metrics=[M.MEAN, M.VARIANCE],
              noise_kind=pipeline_dp.NoiseKind.GAUSSIAN,
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=0.0, max_value=10.0)
    metas.append(write_case("public_mean_var", pid, pk, val, kw, public))
    # h: single metrics.
    pid, pk, val = synthetic(7, 4000, 150, 80, 0.0, 1.0)
    mpc, mcpp, _ = nonbinding(pid, pk)
    metas.append(write_case("count_only", pid, pk, val, dict(
        metrics=[M.COUNT], max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp)))
    metas.append(write_case("pid_count_only", pid, pk, val, dict(
        metrics=[M.PRIVACY_ID_COUNT], max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp)))
    # i: integer values (movie-like ratings).
    pid, pk, val = synthetic(8, 6000, 400, 60, 1, 5, integer_values=True)
    mpc, mcpp, _ = nonbinding(pid, pk)
    metas.append(write_case("integer_values", pid, pk, val, dict(
        metrics=[M.SUM, M.COUNT], max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp, min_value=1, max_value=5)))
    # g: config 1 (movie_view_ratings sample), non-binding bounds.
    mpath = "/root/reference/contributing/sample_combined_data_1.txt"
    pid, pk, val = parse_movie_file(mpath)
    mpc, mcpp, _ = nonbinding(pid, pk)
    kw = dict(metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
              max_partitions_contributed=mpc,
              max_contributions_per_partition=mcpp,
              min_value=1, max_value=5)
    metas.append(write_case("movie_private", pid, pk, val, kw))
    metas.append(write_case("movie_public", pid, pk, val, kw,
                            list(range(1, 100))))
    return metas


def gen_budget_splits():
    """MechanismSpec (eps, delta) in request order, for each metric set."""
    cases = []
    metric_sets = [
        [M.COUNT], [M.SUM], [M.PRIVACY_ID_COUNT],
        [M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
        [M.MEAN], [M.MEAN, M.COUNT, M.SUM], [M.VARIANCE],
        [M.VARIANCE, M.MEAN, M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
    ]
    orig = budget_accounting.NaiveBudgetAccountant.request_budget
    for noise in (pipeline_dp.NoiseKind.LAPLACE, pipeline_dp.NoiseKind.GAUSSIAN):
        for public in (False, True):
            for weight in (1, 0.5):
                for ms in metric_sets:
                    specs = []

                    def rec(self, *a, **k):
                        s = orig(self, *a, **k)
                        specs.append(s)
                        return s

                    budget_accounting.NaiveBudgetAccountant.request_budget = rec
                    try:
                        acc = pipeline_dp.NaiveBudgetAccountant(2.0, 1e-5)
                        eng = pipeline_dp.DPEngine(acc, pipeline_dp.LocalBackend())
                        kw = dict(metrics=ms, noise_kind=noise,
                                  max_partitions_contributed=2,
                                  max_contributions_per_partition=3,
                                  budget_weight=weight)
                        if any(m in ms for m in (M.SUM, M.MEAN, M.VARIANCE)):
                            kw.update(min_value=0.0, max_value=1.0)
                        params = pipeline_dp.AggregateParams(**kw)
                        ex = pipeline_dp.DataExtractors(
                            privacy_id_extractor=lambda r: r[0],
                            partition_extractor=lambda r: r[1],
                            value_extractor=lambda r: r[2])
                        # a second aggregation with weight 1 shares the budget
                        eng.aggregate([(1, 1, 0.5)], params, ex,
                                      public_partitions=[1] if public else None)
                        eng.select_partitions(
                            [(1, 1)], pipeline_dp.SelectPartitionsParams(
                                max_partitions_contributed=1),
                            pipeline_dp.DataExtractors(
                                privacy_id_extractor=lambda r: r[0],
                                partition_extractor=lambda r: r[1]))
                        acc.compute_budgets()
                    finally:
                        budget_accounting.NaiveBudgetAccountant.request_budget = orig
                    cases.append(dict(
                        metrics=_metric_names(ms), noise_kind=noise.name,
                        public=public, budget_weight=weight,
                        specs=[dict(type=s.mechanism_type.name, eps=s.eps,
                                    delta=s.delta) for s in specs]))
    with open(os.path.join(HERE, "budget_splits.json"), "w") as f:
        json.dump(cases, f, indent=1)


def gen_sampling_distribution(trials=4000):
    """Empirical outcome distribution of the reference's sampling bounding.

    Input: pid 1 contributes to partitions 10, 11, 12 (mpc=2 keeps two of
    three); pair (1, 10) has values {1, 1, 5} and pair (1, 11) has {2, 7}
    (mcpp=1 keeps one).  pid 2 contributes {3, 4, 4, 9} to partition 10.
    Each outcome is the tuple of per-partition (count, sum, pid_count).
    """
    rows = [(1, 10, 1.0), (1, 10, 1.0), (1, 10, 5.0), (1, 11, 2.0),
            (1, 11, 7.0), (1, 12, 4.0), (2, 10, 3.0), (2, 10, 4.0),
            (2, 10, 4.0), (2, 10, 9.0)]
    hist = {}
    for t in range(trials):
        np.random.seed(t)
        acc = pipeline_dp.NaiveBudgetAccountant(1.0, 1e-6)
        eng = pipeline_dp.DPEngine(acc, pipeline_dp.LocalBackend())
        params = pipeline_dp.AggregateParams(
            metrics=[M.COUNT, M.SUM, M.PRIVACY_ID_COUNT],
            max_partitions_contributed=2, max_contributions_per_partition=1,
            min_value=0.0, max_value=10.0)
        ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                        partition_extractor=lambda r: r[1],
                                        value_extractor=lambda r: r[2])
        res = eng.aggregate(rows, params, ex, public_partitions=[10, 11, 12])
        acc.compute_budgets()
        out = dict((k, (float(m.count), float(m.sum), float(m.privacy_id_count)))
                   for k, m in res)
        key = json.dumps([out[10], out[11], out[12]])
        hist[key] = hist.get(key, 0) + 1
    with open(os.path.join(HERE, "sampling_distribution.json"), "w") as f:
        json.dump(dict(rows=rows, trials=trials, mpc=2, mcpp=1,
                       partitions=[10, 11, 12], histogram=hist), f, indent=1)


def gen_sampling_distribution_modes(trials=4000):
    """The same outcome histograms for the two other bounders on the same
    rows (public partitions 10, 11, 12), seeded like the cross + per one:

    * PER_PRIVACY_ID (contribution_bounders.py:108-150): max_contributions=2
      keeps 2 of pid 1's 6 records and 2 of pid 2's 4, uniformly; outcome =
      per-partition (count, sum) of COUNT + SUM;
    * CROSS_PARTITION (:153-195): SUM with min/max_sum_per_partition keeps
      mpc=2 of pid 1's 3 partitions with ALL their values, then clips each
      pair's sum to [0, 6]; outcome = per-partition (sum, privacy_id_count).
    """
    rows = [(1, 10, 1.0), (1, 10, 1.0), (1, 10, 5.0), (1, 11, 2.0),
            (1, 11, 7.0), (1, 12, 4.0), (2, 10, 3.0), (2, 10, 4.0),
            (2, 10, 4.0), (2, 10, 9.0)]
    modes = {
        "per_privacy_id": (dict(metrics=[M.COUNT, M.SUM], max_contributions=2,
                                min_value=0.0, max_value=10.0),
                           ("count", "sum")),
        "cross_partition": (dict(metrics=[M.SUM, M.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=2,
                                 max_contributions_per_partition=1,
                                 min_sum_per_partition=0.0, max_sum_per_partition=6.0),
                            ("sum", "privacy_id_count")),
    }
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    for name, (kw, fields) in modes.items():
        hist = {}
        for t in range(trials):
            np.random.seed(t)
            acc = pipeline_dp.NaiveBudgetAccountant(1.0, 1e-6)
            eng = pipeline_dp.DPEngine(acc, pipeline_dp.LocalBackend())
            res = eng.aggregate(rows, pipeline_dp.AggregateParams(**kw), ex,
                                public_partitions=[10, 11, 12])
            acc.compute_budgets()
            out = dict((k, tuple(float(getattr(m, f)) for f in fields)) for k, m in res)
            key = json.dumps([out[10], out[11], out[12]])
            hist[key] = hist.get(key, 0) + 1
        with open(os.path.join(HERE, f"sampling_distribution_{name}.json"), "w") as f:
            json.dump(dict(rows=rows, trials=trials, params=_params_to_json(kw),
                           fields=list(fields), partitions=[10, 11, 12], histogram=hist),
                      f, indent=1)


def gen_select_partitions():
    """select_partitions with a keep-all strategy: the set of partitions."""
    pid, pk, _ = synthetic(9, 3000, 200, 150, 0, 1)
    acc = pipeline_dp.NaiveBudgetAccountant(1.0, 1e-6)
    eng = pipeline_dp.DPEngine(acc, pipeline_dp.LocalBackend())
    res = eng.select_partitions(
        list(zip(pid.tolist(), pk.tolist())),
        pipeline_dp.SelectPartitionsParams(max_partitions_contributed=3),
        pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                   partition_extractor=lambda r: r[1]))
    acc.compute_budgets()
    keys = sorted(res)
    np.savez_compressed(os.path.join(HERE, "select_partitions.npz"),
                        pid=pid, pk=pk, out_keys=np.array(keys, np.int64))


def main():
    metas = gen_aggregate_cases()
    with open(os.path.join(HERE, "aggregate_cases.json"), "w") as f:
        json.dump(metas, f, indent=1)
    gen_budget_splits()
    gen_sampling_distribution()
    gen_sampling_distribution_modes()
    gen_select_partitions()
    print("wrote", len(metas), "aggregate cases")


if __name__ == "__main__":
    main()
