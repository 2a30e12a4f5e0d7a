"""The fast path's envelope: inputs whose level-1 buckets
exceed the team level 2's single-round capacity (heavy privacy ids, N past
2^30) and 23-bit plans keep the histogram-free level 1 and the team level 2.

* multi-round team: a bucket whose member share exceeds the round capacity
  is done by a second launch in rounds (count, reserve, team barrier, then
  rank / stage / write each round); the test hook DPG_DEBUG_TEAM_SUB shrinks
  the round capacity so that 1e7 records take it;
* 12 + 11 bits: a 23-bit plan (forced at 1e7 records by DPG_DEBUG_TARGET=1
  with 2^23 privacy-id hash values) takes a 4096-digit level 1 (pieces, or
  the histogram path) and an 11-bit team level 2 instead of 11 + 12 bits.

Every variant's partials equal the oracle's (counts and privacy-id counts
bit-exact, sums to 1e-9) and its stage times name the path it took."""
import numpy as np
import pytest
import torch

import bench
import pipelinedp_amd as pdp
from oracle import oracle

pytestmark = pytest.mark.gpu

SEED = 0xE7E10


def _params(mpc=8, mcpp=2):
    return pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=mpc,
        max_contributions_per_partition=mcpp, min_value=0.0, max_value=10.0)


def _run_and_check(pid, pk, val, P, pid_range):
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    cols = pdp.ColumnarData(pid=torch.from_numpy(pid).cuda(), pk=torch.from_numpy(pk).cuda(),
                            value=torch.from_numpy(val).cuda(), n_partitions=P,
                            privacy_id_range=pid_range)
    res = pdp.DPEngine(acc, backend).aggregate(cols, _params(), pdp.DataExtractors("pid", "pk", "value"))
    acc.compute_budgets()
    res.noise_enabled = False
    res.nonce = 77
    res.materialize()
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)
    return backend.ctx.stage_times()


N, P = 10_000_000, 1_000_000


@pytest.fixture(scope="module")
def heavy_data():
    """The config-2 generator with 10x heavier privacy ids (1e5 ids of ~100
    records -> 1e4 ids of ~1000), as (N = 1e9, U = 1e6) is to config 2."""
    pid, pk, val = bench.host_sample(N, 10_000, P, 31)
    return pid.astype(np.int64), pk.astype(np.int64), val


@pytest.mark.parametrize("level1", ["pieces", "histogram"])
def test_multi_round_team_matches_oracle(built, heavy_data, monkeypatch, level1):
    """Round capacity 64 records per member (DPG_DEBUG_TEAM_SUB): every
    level-1 bucket (~4900 records, ~153 per member) is done in 3 rounds by
    the multi-round launch."""
    monkeypatch.setenv("DPG_DEBUG_TEAM_SUB", "64")
    monkeypatch.setenv("DPG_L1_PIECES", "1" if level1 == "pieces" else "0")
    pid, pk, val = heavy_data
    st = _run_and_check(pid, pk, val, P, (0, 10_000))
    assert "partition2:team" in st and "partition2:team_multi" in st
    assert ("partition1:pieces" in st) == (level1 == "pieces")
    assert "partition2:hist" not in st


def test_multi_round_team_some_buckets(built, heavy_data, monkeypatch):
    """A round capacity between the bucket sizes: the single-round launch
    takes the buckets that fit, the multi-round one the others."""
    pid, pk, val = heavy_data
    monkeypatch.setenv("DPG_DEBUG_TEAM_SUB", "154")
    st = _run_and_check(pid, pk, val, P, (0, 10_000))
    assert "partition2:team_multi" in st and "partition1:pieces" in st


@pytest.fixture(scope="module")
def wide_plan_data():
    """2^23 privacy-id values (23 hash bits) over 1e7 records."""
    rng = np.random.default_rng(5)
    U = 1 << 23
    pid = rng.integers(0, U, N).astype(np.int64)
    pk = ((rng.zipf(1.1, N) - 1) % P).astype(np.int64)
    val = rng.uniform(-1.0, 11.0, N)
    return pid, pk, val, U


@pytest.mark.parametrize("level1", ["pieces", "histogram", "piece_overflow", "eleven_twelve"])
def test_twelve_bit_level1_matches_oracle(built, wide_plan_data, monkeypatch, level1):
    """DPG_DEBUG_TARGET=1 makes the plan take 23 hash bits at 1e7 records:
    12 + 11 bits (4096-digit level 1, team level 2) -- by pieces, by the
    histogram path, by pieces redone with the histogram after a region
    overflow (DPG_DEBUG_PIECE_CAP) -- or 11 + 12 bits with DPG_B1W=0 (the
    4096-digit grouped level 2)."""
    monkeypatch.setenv("DPG_DEBUG_TARGET", "1")
    monkeypatch.setenv("DPG_L1_PIECES", "0" if level1 == "histogram" else "1")
    if level1 == "piece_overflow":
        monkeypatch.setenv("DPG_DEBUG_PIECE_CAP", "64")
    if level1 == "eleven_twelve":
        monkeypatch.setenv("DPG_B1W", "0")
    pid, pk, val, U = wide_plan_data
    st = _run_and_check(pid, pk, val, P, (0, U))
    if level1 == "eleven_twelve":
        assert "partition2:team" not in st and "partition2:hist" in st
    else:
        assert "partition2:team" in st
        assert ("partition1:pieces" in st) == (level1 != "histogram")
        assert ("partition1:hist" in st) == (level1 != "pieces")
