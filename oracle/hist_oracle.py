"""CPU restatement of the dataset histograms (TEST INFRASTRUCTURE ONLY: the
checker of tests/ and smoke(); never imported by pipelinedp_amd).

Follows pipeline_dp/dataset_histograms/computing_histograms.py:
  _to_bin_lower_upper_logarithmic :28-47, _bin_lower_index :50-59,
  L0 :237-261, L1 :264-287, LINF :290-311, LINF_SUM :314-362 (10^4 equal
  bins from np.linspace(min, max, 10^4 + 1)), COUNT_PER_PARTITION :365-389,
  PRIVACY_ID_PER_PARTITION :392-417; pre-aggregated variants :482-639
  (L0 / L1 weighted by 1 / n_partitions, rounded per value, :81-102).
Pinned by tests/golden/dataset_histograms.json (gen_golden_hist.py runs the
reference on the same inputs).  Output per histogram: (name, [[lower, upper,
count, sum, max], ...]) sorted by lower.
"""
import bisect

import numpy as np

NAMES = ("l0_contributions", "l1_contributions", "linf_contributions",
         "linf_sum_contributions", "count_per_partition", "privacy_id_per_partition_count")
N_SUM_BINS = 10000


def int_lower_upper(value: int):
    bound = 1000
    while value > bound:
        bound *= 10
    base = bound // 1000
    lower = value // base * base
    return lower, lower + (base if value != bound else base * 10)


def _int_hist(values, freq=None):
    """values (and their frequencies) -> bins of 3 significant digits."""
    values = np.asarray(values, dtype=np.int64)
    freq = np.ones(len(values), np.int64) if freq is None else np.asarray(freq, np.int64)
    bins = {}
    for v, f in zip(values.tolist(), freq.tolist()):
        lo, up = int_lower_upper(v)
        b = bins.setdefault(lo, [lo, up, 0, 0, v])
        b[2] += f
        b[3] += f * v
        b[4] = max(b[4], v)
    return [bins[k] for k in sorted(bins)]


def _sum_hist(sums):
    sums = np.asarray(sums, dtype=np.float64)
    if len(sums) == 0:
        return []
    lowers = np.linspace(sums.min(), sums.max(), N_SUM_BINS + 1)
    lw = lowers.tolist()
    bins = {}
    for v in sums.tolist():
        i = len(lw) - 2 if v == lw[-1] else bisect.bisect_right(lw, v) - 1
        b = bins.setdefault(i, [lw[i], lw[i + 1], 0, 0.0, v])
        b[2] += 1
        b[3] += v
        b[4] = max(b[4], v)
    return [bins[k] for k in sorted(bins)]


def dataset_histograms(pid, pk, value):
    """compute_dataset_histograms over rows (pid, pk, value)."""
    pid, pk = np.asarray(pid, np.int64), np.asarray(pk, np.int64)
    value = np.asarray(value, np.float64)
    pairs, inv = np.unique(np.stack([pid, pk], 1), axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    pair_cnt = np.bincount(inv, minlength=len(pairs))
    pair_sum = np.zeros(len(pairs))
    np.add.at(pair_sum, inv, value)
    _, l0 = np.unique(pairs[:, 0], return_counts=True)
    _, l1 = np.unique(pid, return_counts=True)
    _, cpp = np.unique(pk, return_counts=True)
    _, ppp = np.unique(pairs[:, 1], return_counts=True)
    return [(NAMES[0], _int_hist(l0)), (NAMES[1], _int_hist(l1)), (NAMES[2], _int_hist(pair_cnt)),
            (NAMES[3], _sum_hist(pair_sum)), (NAMES[4], _int_hist(cpp)),
            (NAMES[5], _int_hist(ppp))]


def _weighted(values, weights):
    acc = {}
    for v, w in zip(values, weights):
        acc[v] = acc.get(v, 0.0) + w
    vals = sorted(acc)
    return _int_hist(vals, [int(round(acc[v])) for v in vals])


def dataset_histograms_preaggregated(rows):
    """compute_dataset_histograms_on_preaggregated_data over rows
    (pk, (count, sum, n_partitions, n_contributions))."""
    pk = np.array([r[0] for r in rows], np.int64)
    x = np.array([r[1] for r in rows], np.float64).reshape(len(rows), 4)
    cnt, sm, npart, ncon = x[:, 0].astype(np.int64), x[:, 1], x[:, 2].astype(np.int64), \
        x[:, 3].astype(np.int64)
    keys, inv = np.unique(pk, return_inverse=True)
    cpp = np.bincount(inv.reshape(-1), weights=cnt, minlength=len(keys)).astype(np.int64)
    ppp = np.bincount(inv.reshape(-1), minlength=len(keys))
    w = (1.0 / npart).tolist()
    return [(NAMES[0], _weighted(npart.tolist(), w)), (NAMES[1], _weighted(ncon.tolist(), w)),
            (NAMES[2], _int_hist(cnt)), (NAMES[3], _sum_hist(sm)), (NAMES[4], _int_hist(cpp)),
            (NAMES[5], _int_hist(ppp))]
