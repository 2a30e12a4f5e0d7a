"""Vectorised numpy restatement of the utility-analysis sweep's per-partition
part (TEST INFRASTRUCTURE: the CPU baseline of bench.py --workload config5
and a checker; nothing in pipelinedp_amd/ imports it).

Same arithmetic as oracle/utility_oracle.py (whose per-partition results it
is tested against, tests/test_utility_oracle.py), restated over arrays so
that it runs on >= 1e6 records:
  * pre-aggregation (analysis/contribution_bounders.py:37-77): pairs
    (pid, pk) -> (count, sum, n_partitions, n_contributions), grouped by pk;
  * PartitionSelectionCombiner (analysis/per_partition_combiners.py:195-240):
    the privacy-id-count PMF from the pairs' l0 keep probabilities
    min(1, l0 / n_partitions) -- exact for <= 100 pairs (all partitions of
    one pair count in one vectorised recursion), the refined normal
    approximation beyond (analysis/poisson_binomial.py:61-83) -- dotted with
    the selection strategy's keep probability;
  * Sum/Count/PrivacyIdCount combiners (:243-339): clipping and l0-bounding
    error terms per partition (np.add.reduceat over the pk runs).
Configurations are split over worker processes (fork; the pair arrays are
shared copy-on-write).  The cross-partition report (a few sums per size
bucket) is not part of this restatement.
"""
import math
import os
from typing import List

import numpy as np
from scipy.stats import norm

from oracle import utility_oracle as uo

MAX_EXACT = uo.MAX_EXACT


def preaggregate(pid: np.ndarray, pk: np.ndarray, val: np.ndarray):
    """Pairs sorted by pk: (pk, count, sum, n_partitions) and the run starts."""
    order = np.lexsort((pk, pid))
    a, b, v = pid[order], pk[order], val[order]
    new = np.ones(a.size, bool)
    new[1:] = (a[1:] != a[:-1]) | (b[1:] != b[:-1])
    st = np.flatnonzero(new)
    cnt = np.diff(np.append(st, a.size))
    sm = np.add.reduceat(v, st)
    ppid, ppk = a[st], b[st]
    newp = np.ones(ppid.size, bool)
    newp[1:] = ppid[1:] != ppid[:-1]
    pst = np.flatnonzero(newp)
    npart = np.diff(np.append(pst, ppid.size))[np.cumsum(newp) - 1]
    o = np.argsort(ppk, kind="stable")
    ppk, cnt, sm, npart = ppk[o], cnt[o], sm[o], npart[o]
    runs = np.flatnonzero(np.r_[True, ppk[1:] != ppk[:-1]])
    return dict(pk=ppk[runs], start=runs, n=np.diff(np.append(runs, ppk.size)),
                cnt=cnt.astype(np.float64), sum=sm, npart=npart.astype(np.float64))


def _keep_probability(pa, p, keep_fn):
    """Expected keep probability per partition (PMF of the privacy-id count
    dotted with keep_fn)."""
    n = pa["n"]
    st = pa["start"]
    out = np.zeros(n.size)
    fvals = np.array([keep_fn(i) for i in range(MAX_EXACT + 1)])
    for m in np.unique(n[n <= MAX_EXACT]):
        rows = np.flatnonzero(n == m)
        probs = p[st[rows][:, None] + np.arange(m)[None, :]]  # [rows, m]
        c = np.zeros((rows.size, m + 1))
        c[:, 0] = 1.0
        for j in range(m):
            pj = probs[:, j:j + 1]
            c[:, 1:j + 2] = c[:, 1:j + 2] * (1.0 - pj) + c[:, 0:j + 1] * pj
            c[:, 0:1] *= 1.0 - pj
        out[rows] = c @ fvals[:m + 1]
    big = np.flatnonzero(n > MAX_EXACT)
    for r in big:  # refined normal approximation (few, large partitions)
        pr = p[st[r]:st[r] + n[r]]
        s0, pm = uo.pmf(pr)
        out[r] = float(sum(q * keep_fn(s0 + j) for j, q in enumerate(pm)))
    return out


def _sum_terms(x, pc_lo, pc_hi, p, q, st):
    pc = np.clip(x, pc_lo, pc_hi)
    e = pc - x
    red = lambda y: np.add.reduceat(y, st)  # noqa: E731
    return dict(sum=red(x), clipping_to_min_error=red(np.where(x < pc_lo, e, 0.0)),
                clipping_to_max_error=red(np.where(x > pc_hi, e, 0.0)),
                expected_l0_bounding_error=red(-pc * (1.0 - p)),
                var_l0_bounding_error=red(pc * pc * q))


def per_partition(pa, cfg: dict, eps_sel: float, delta_sel: float, metrics: List[str]):
    """One configuration's per-partition results: keep probability and the
    error terms of each metric (arrays over the partitions)."""
    l0 = cfg["mpc"]
    p = np.where(pa["npart"] > 0, np.minimum(1.0, l0 / np.maximum(pa["npart"], 1.0)), 0.0)
    q = p * (1.0 - p)
    st = pa["start"]
    f = uo.keep_fn(cfg["strategy"], eps_sel, delta_sel, l0, cfg["pre_threshold"])
    res = dict(keep=_keep_probability(pa, p, f))
    if "SUM" in metrics:
        res["SUM"] = _sum_terms(pa["sum"], cfg["min_sum"], cfg["max_sum"], p, q, st)
    if "COUNT" in metrics:
        res["COUNT"] = _sum_terms(pa["cnt"], 0.0, float(cfg["mcpp"]), p, q, st)
    if "PRIVACY_ID_COUNT" in metrics:
        res["PRIVACY_ID_COUNT"] = _sum_terms((pa["cnt"] > 0).astype(np.float64), 0.0, 1.0, p, q,
                                             st)
    return res


_SHARED = {}


def _work(args):
    lo, hi = args
    sh = _SHARED
    return [per_partition(sh["pa"], c, sh["eps"], sh["delta"], sh["metrics"])
            for c in sh["cfgs"][lo:hi]]


def sweep(pid, pk, val, cfgs: List[dict], metrics: List[str], eps: float, delta: float,
          noise_kind: str = "LAPLACE", workers: int = 0):
    """Pre-aggregation + every configuration's per-partition results, the
    configurations split over `workers` processes.  Returns (pairs, list of
    per-configuration results)."""
    pa = preaggregate(np.asarray(pid), np.asarray(pk), np.asarray(val, dtype=np.float64))
    bud = uo.budgets(eps, delta, metrics, noise_kind, True)
    eps_sel, delta_sel = bud["GENERIC"]
    workers = workers or min(16, os.cpu_count() or 1)
    if workers <= 1:
        return pa, [per_partition(pa, c, eps_sel, delta_sel, metrics) for c in cfgs]
    import multiprocessing as mp
    _SHARED.update(pa=pa, cfgs=cfgs, eps=eps_sel, delta=delta_sel, metrics=metrics)
    step = math.ceil(len(cfgs) / workers)
    spans = [(i, min(len(cfgs), i + step)) for i in range(0, len(cfgs), step)]
    with mp.get_context("fork").Pool(len(spans)) as pool:
        parts = pool.map(_work, spans)
    _SHARED.clear()
    return pa, [r for part in parts for r in part]
