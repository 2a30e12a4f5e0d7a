"""GPU parity at BASELINE.json shapes (reduced record counts so the oracle
finishes in seconds): the config-2 generator at 1e7 records, and the config-4
shape (Pareto(1.2) records per privacy id, mpc = 50, mcpp = 4, P = 1e8,
MEAN+VARIANCE with Gaussian noise) with public and with private partitions.
The config-4 data holds privacy ids with tens of thousands of records, so
their buckets take the heavy-id filter and the global-memory kernel
(k_bound_big), with 24-byte MEAN/VARIANCE items (ItemV: no SUM requested) and
12-byte records (P = 1e8 needs a 70-bit record key)."""
import numpy as np
import pytest
import torch

import bench
import pipelinedp_amd as pdp
from oracle import oracle

pytestmark = pytest.mark.gpu

SEED = 0xC0F16


def _run(pid, pk, val, params, P, public=None, noise=False, nonce=1234, pid_range=None):
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    cols = pdp.ColumnarData(pid=torch.from_numpy(pid).cuda(), pk=torch.from_numpy(pk).cuda(),
                            value=torch.from_numpy(val).cuda(), n_partitions=P,
                            privacy_id_range=pid_range)
    res = pdp.DPEngine(acc, backend).aggregate(cols, params, pdp.DataExtractors("pid", "pk", "value"),
                                               public_partitions=public)
    acc.compute_budgets()
    res.noise_enabled = noise
    res.nonce = nonce
    out = res.materialize()
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    return res, out, got


def _assert_partials(got, ref, keys=("sum",)):
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in keys:
        assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


# ------------------------------------------------------------------ config 2
N2, U2, P2 = 10_000_000, 100_000, 1_000_000


@pytest.fixture(scope="module")
def config2_data():
    pid, pk, val = bench.host_sample(N2, U2, P2, 2024)
    return pid.astype(np.int64), pk.astype(np.int64), val


def _c2_params(mpc, mcpp):
    return pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp, min_value=0.0, max_value=10.0)


def test_config2_nonbinding_bounds_equal_exact_groupby(built, config2_data):
    """SURVEY 8(d) parity variant: 1e7 records of the config-2 generator with
    bounds that never trigger; the partials are the exact group-by of the
    input (numpy, independent of the oracle): counts and privacy-id counts
    bit-exact, sums within 1e-9 relative."""
    pid, pk, val = config2_data
    # 1000 exceeds every privacy id's pairs and every pair's records here
    assert np.bincount(pid).max() < 1000
    _, _, got = _run(pid, pk, val, _c2_params(1000, 1000), P2, pid_range=(0, U2))
    count = np.bincount(pk, minlength=P2)
    s = np.bincount(pk, weights=np.clip(val, 0.0, 10.0), minlength=P2)
    pairs = np.unique(pid * P2 + pk)
    rows = np.bincount(pairs % P2, minlength=P2)
    assert np.array_equal(got["count"], count)
    assert np.array_equal(got["rows"], rows)
    assert np.allclose(got["sum"], s, rtol=1e-9, atol=1e-9)


def test_config2_bounding_triggered_matches_oracle(built, config2_data):
    """mpc = 8, mcpp = 2 (the bench's bounds): partials equal the oracle's,
    then selection + Laplace noise equal the oracle's release."""
    pid, pk, val = config2_data
    res, out, got = _run(pid, pk, val, _c2_params(8, 2), P2, noise=True)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    _assert_partials(got, ref)
    assert got["rows"].sum() <= 8 * U2
    keep, o = oracle.select_and_noise(ref, res.last_select_fields, res.plan.noise_fields(True),
                                      SEED, keep_table=res._table)
    ids = np.nonzero(keep)[0]
    gid = out.partition_ids.cpu().numpy()
    assert np.array_equal(np.sort(gid), ids)
    assert np.allclose(out.values.cpu().numpy()[np.argsort(gid)], o[ids], rtol=1e-12, atol=1e-6)


@pytest.mark.parametrize("mode", ["pieces", "team", "grouped", "team_abort", "piece_overflow"])
def test_config2_level2_paths_match_oracle(built, config2_data, monkeypatch, mode):
    """The first two partition levels five ways, every one bit-exact against
    the oracle (kept pairs, counts; sums to 1e-9):
    pieces -- the default for 8-byte records (round 5): level 1 without a
      histogram pass (per-XCD fixed-capacity regions, k_scatter's piece
      mode), level 2 by teams reading the pieces;
    team -- level 1 with its histogram (DPG_L1_PIECES=0), level 2 by teams
      without one;
    grouped -- both levels with histograms (DPG_TEAM_L2=0);
    team_abort -- pieces, and a team barrier that gives up (test hook
      DPG_DEBUG_TEAM_ABORT: abort flag + err bit 8, as after a timeout); the
      host sees it at the chunking sync and redoes both levels with the
      histogram paths;
    piece_overflow -- pieces in regions far too small
      (DPG_DEBUG_PIECE_CAP=64): runs go to the dump area, err bit 16, and
      the host redoes level 1 with its histogram before level 2."""
    if mode == "grouped":
        monkeypatch.setenv("DPG_TEAM_L2", "0")
    monkeypatch.setenv("DPG_L1_PIECES", "1" if mode in ("pieces", "team_abort", "piece_overflow")
                       else "0")
    if mode == "team_abort":
        monkeypatch.setenv("DPG_DEBUG_TEAM_ABORT", "1")
        monkeypatch.setenv("DPG_DEBUG_TEAM_BACKOFF", "1")
    if mode == "piece_overflow":
        monkeypatch.setenv("DPG_DEBUG_PIECE_CAP", "64")
    pid, pk, val = config2_data
    res, _, got = _run(pid, pk, val, _c2_params(8, 2), P2)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    _assert_partials(got, ref)
    stages = res.backend.ctx.stage_times()
    assert ("partition1:pieces" in stages) == (mode in ("pieces", "team_abort", "piece_overflow"))
    assert ("partition1:hist" in stages) == (mode != "pieces")
    assert ("partition2:team" in stages) == (mode != "grouped")
    assert ("partition2:hist" in stages) == (mode in ("grouped", "team_abort"))
    assert ("partition2:team_redo" in stages) == (mode == "team_abort")
    if mode == "team_abort":
        # the timeout backs off on the context: the next
        # release on the same backend (back-off of 1 call, test hook
        # DPG_DEBUG_TEAM_BACKOFF; 64 calls by default) takes the histogram
        # level 2 directly and says so in its stage times; the one after
        # tries the team path again; both still match the oracle
        monkeypatch.delenv("DPG_DEBUG_TEAM_ABORT")
        cols = pdp.ColumnarData(pid=torch.from_numpy(pid).cuda(), pk=torch.from_numpy(pk).cuda(),
                                value=torch.from_numpy(val).cuda(), n_partitions=P2)
        for again in (False, True):
            acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
            res2 = pdp.DPEngine(acc, res.backend).aggregate(
                cols, _c2_params(8, 2), pdp.DataExtractors("pid", "pk", "value"))
            acc.compute_budgets()
            res2.noise_enabled = False
            res2.nonce = 1234
            res2.materialize()
            got2 = {k: v.cpu().numpy() for k, v in res2.last_partials.items() if v is not None}
            _assert_partials(got2, ref)
            stages2 = res.backend.ctx.stage_times()
            assert ("partition2:team" in stages2) == again
            assert ("team_backoff" in stages2) == (not again)


def test_config2_pieces_range_error(built, config2_data, monkeypatch):
    """The histogram-free level 1 checks whole privacy ids itself: an id past
    the declared range (high word differs, low word in range) fails the
    call with the key-range error, as the histogram path does."""
    monkeypatch.setenv("DPG_L1_PIECES", "1")
    pid, pk, val = config2_data
    bad = pid.copy()
    bad[123457] += 1 << 32
    with pytest.raises(Exception, match="range"):
        _run(bad, pk, val, _c2_params(8, 2), P2, pid_range=(0, U2))


# ------------------------------------------------------------------ config 4
N4, U4, P4 = 20_000_000, 100_000, 100_000_000


@pytest.fixture(scope="module")
def config4_data():
    pid, pk, val = bench.host_sample(N4, U4, P4, 4242, pareto=(1.2, 1000.0))
    pid, pk = pid.astype(np.int64), pk.astype(np.int64)
    # heavy privacy ids: far beyond one LDS chunk (1024 records), so the
    # global-memory bounding kernel runs
    assert np.bincount(pid).max() > 8192
    return pid, pk, val


def _c4_params():
    return pdp.AggregateParams(
        metrics=[pdp.Metrics.MEAN, pdp.Metrics.VARIANCE], noise_kind=pdp.NoiseKind.GAUSSIAN,
        max_partitions_contributed=50, max_contributions_per_partition=4,
        min_value=0.0, max_value=10.0)


def test_config4_public_partitions_match_oracle(built, config4_data):
    """public_partitions = range(1e8): empty partitions kept (the set covers
    every id, so level 1 drops nothing), MEAN/VARIANCE moments through every
    bounding kernel (ItemV), noise-free outputs equal the oracle's for all
    1e8 partitions."""
    pid, pk, val = config4_data
    res, out, got = _run(pid, pk, val, _c4_params(), P4, public=range(P4))
    mask = np.full((P4 + 7) // 8, 0xFF, np.uint8)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED, public_mask=mask)
    _assert_partials(got, ref, keys=("nsum", "nsq"))
    assert out.partition_ids.numel() == P4
    keep, o = oracle.select_and_noise(ref, res.last_select_fields, res.plan.noise_fields(False),
                                      SEED, public_mask=mask)
    assert keep.all()
    gid = out.partition_ids.cpu().numpy()
    assert np.array_equal(gid, np.arange(P4))
    assert np.allclose(out.values.cpu().numpy(), o, rtol=1e-9, atol=1e-9, equal_nan=True)


def test_config4_private_selection_gaussian_matches_oracle(built, config4_data):
    """Private selection (truncated geometric, l0 = 50) + Gaussian noise on
    the 3-way-split VARIANCE mechanism: keep set and noised mean/variance
    equal the oracle's release."""
    pid, pk, val = config4_data
    res, out, got = _run(pid, pk, val, _c4_params(), P4, noise=True, nonce=99)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    _assert_partials(got, ref, keys=("nsum", "nsq"))
    assert got["rows"].max() > 0
    keep, o = oracle.select_and_noise(ref, res.last_select_fields, res.plan.noise_fields(True),
                                      SEED, keep_table=res._table)
    ids = np.nonzero(keep)[0]
    gid = out.partition_ids.cpu().numpy()
    assert np.array_equal(np.sort(gid), ids)
    assert len(ids) > 100
    assert np.allclose(out.values.cpu().numpy()[np.argsort(gid)], o[ids], rtol=1e-9, atol=1e-6)
