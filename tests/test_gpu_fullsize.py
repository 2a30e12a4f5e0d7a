"""configs[1] at its full size: 1e9 device-generated records (bench.generate,
the bench's own generator), 1e7 privacy ids, 1e6 Zipf(1.1) partitions.  The
oracle cannot run this size, so the checks are size-independent properties
against device group-bys (torch):

(i) bounds that never trigger (mpc, mcpp far above any privacy id's pairs /
    any pair's records): the partials ARE the exact group-by of the input --
    counts and privacy-id counts bit-exact against bincount / unique(pid * P
    + pk), sums within 1e-9 relative (combiners.py:255-379 with nothing
    sampled, contribution_bounders.py:66-105);
(ii) the bench's bounds (mpc 8, mcpp 2): sum over partitions of the kept
    pairs = sum over privacy ids of min(distinct pairs, mpc) exactly (every
    privacy id keeps min(#pairs, mpc) pairs, contribution_bounders.py:90-92);
    per partition rows <= true rows, rows <= count <= mcpp * rows, count <=
    true count, 0 <= sum <= max_value * count.

This exercises the 32-bit bucket offsets, the level totals and the scratch
sizes at the size the bench line claims (missing item 3)."""
import time

import numpy as np
import pytest
import torch

import bench
import pipelinedp_amd as pdp

pytestmark = pytest.mark.gpu

N, U, P = 1_000_000_000, 10_000_000, 1_000_000
SEED = 0xF1115


def _log(msg, t0):
    # progress on stdout (run with -s): these steps take seconds each
    torch.cuda.synchronize()
    print(f"[fullsize] {msg}: {time.perf_counter() - t0:.1f} s", flush=True)


@pytest.fixture(scope="module")
def full():
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    pid, pk, val = bench.generate(N, U, P, 0, 1, dev)
    _log("generated", t0)
    # device group-by references (exact integers; the float sum by bincount)
    count = torch.bincount(pk, minlength=P)
    _log("count", t0)
    pair = torch.unique(pid * P + pk)
    _log(f"{pair.numel()} distinct pairs", t0)
    rows = torch.bincount(pair % P, minlength=P)
    pairs_per_pid = torch.bincount(pair // P, minlength=U)
    del pair
    _log("rows", t0)
    # the float sums on the host: a weighted device bincount funnels ~1e8
    # float64 atomic adds into the hottest Zipf partition (minutes)
    s = np.bincount(pk.cpu().numpy(), weights=val.clamp(0.0, 10.0).cpu().numpy(), minlength=P)
    s = torch.from_numpy(s).to(dev)
    _log("reference group-by", t0)
    yield dict(pid=pid, pk=pk, val=val, count=count, rows=rows, sum=s,
               pairs_per_pid=pairs_per_pid)
    torch.cuda.empty_cache()


def _partials(d, mpc, mcpp):
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    cols = pdp.ColumnarData(pid=d["pid"], pk=d["pk"], value=d["val"], n_partitions=P,
                            privacy_id_range=(0, U))
    params = pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp, min_value=0.0, max_value=10.0)
    res = pdp.DPEngine(acc, backend).aggregate(cols, params,
                                               pdp.DataExtractors("pid", "pk", "value"))
    acc.compute_budgets()
    res.noise_enabled = False
    res.nonce = 77
    t0 = time.perf_counter()
    out = res.materialize(gather=False)
    got = {k: v for k, v in res.last_partials.items() if v is not None}
    _log(f"aggregate mpc {mpc} mcpp {mcpp}", t0)
    return res, out, got


def test_fullsize_nonbinding_bounds_equal_device_groupby(built, full):
    # non-binding: no privacy id has 4096 pairs, no pair 4096 records
    assert int(full["pairs_per_pid"].max()) < 4096
    _, _, got = _partials(full, 4096, 4096)
    assert torch.equal(got["count"].to(torch.int64), full["count"])
    assert torch.equal(got["rows"].to(torch.int64), full["rows"])
    assert torch.allclose(got["sum"], full["sum"], rtol=1e-9, atol=1e-9)
    assert int(got["count"].sum()) == N


def test_fullsize_bench_bounds_invariants(built, full):
    mpc, mcpp = 8, 2
    res, out, got = _partials(full, mpc, mcpp)
    rows = got["rows"].to(torch.int64)
    cnt = got["count"].to(torch.int64)
    s = got["sum"]
    # every privacy id keeps min(#distinct pairs, mpc) pairs
    want_pairs = int(full["pairs_per_pid"].clamp(max=mpc).sum())
    assert int(rows.sum()) == want_pairs
    assert bool((rows <= full["rows"]).all())
    assert bool((cnt >= rows).all()) and bool((cnt <= mcpp * rows).all())
    assert bool((cnt <= full["count"]).all())
    assert bool((s >= 0).all()) and bool((s <= 10.0 * cnt.to(torch.float64) + 1e-9).all())
    # a pair with a single record keeps it: at least one record per kept pair,
    # and the records kept are at most mcpp per kept pair (whole-sum form)
    assert want_pairs <= int(cnt.sum()) <= mcpp * want_pairs
    # selection ran over the same partials (kept ids are occupied partitions)
    ids = out.partition_ids
    if ids.numel():
        assert bool((rows[ids] > 0).all())
