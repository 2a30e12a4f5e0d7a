"""GPU parity: the HIP path (through libdpg's C ABI) against the reference
fixtures and against the oracle on the same seeded inputs."""
import numpy as np
import pytest
import torch

import pipelinedp_amd as pdp
from oracle import oracle
from pipelinedp_amd import combiners
from tests import golden_cases as gc

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def run_engine(pid, pk, value, params, public=None, seed=SEED, noise=False,
               n_partitions=None, eps=1.0, delta=1e-6, nonce=None):
    backend = pdp.MI355XBackend(device=0, seed=seed)
    acc = pdp.NaiveBudgetAccountant(eps, delta)
    eng = pdp.DPEngine(acc, backend)
    cols = pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                            value=None if value is None else torch.as_tensor(value),
                            n_partitions=n_partitions)
    res = eng.aggregate(cols, params, pdp.DataExtractors("pid", "pk", "value"),
                        public_partitions=public)
    acc.compute_budgets()
    res.noise_enabled = noise
    if nonce is not None:
        res.nonce = nonce
    out = res.materialize()
    return res, out


@pytest.mark.parametrize("meta", gc.cases(), ids=lambda m: m["name"])
def test_gpu_matches_reference_fixture(built, meta):
    d = gc.load(meta)
    params = gc.params_of(meta)
    public = d["public_partitions"].tolist() if "public_partitions" in d else None
    if public is None:
        # the stub keeps every partition; with noise off, use the observed
        # partitions as public so selection does not drop any
        public = sorted(set(d["pk"].tolist()))
        params.partition_selection_strategy = pdp.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC
    res, out = run_engine(d["pid"], d["pk"], d["value"], params, public=public)
    keys = np.asarray(out.keys())
    order = np.argsort(keys)
    assert list(out.fields) == meta["fields"]
    assert np.array_equal(keys[order], d["out_keys"])
    vals = out.values.cpu().numpy()[order]
    for j, f in enumerate(out.fields):
        assert gc.tolerance_ok(f, vals[:, j], d["out_" + f]), f


def _dataset(seed, n, n_pid, P, zipf=1.2, vlo=-2.0, vhi=12.0, dup_values=False):
    rng = np.random.default_rng(seed)
    pid = rng.integers(0, n_pid, n)
    pk = (rng.zipf(zipf, n) - 1) % P
    val = rng.uniform(vlo, vhi, n)
    if dup_values:
        val = np.round(val)
    return pid.astype(np.int64), pk.astype(np.int64), val


MODES = [
    ("cross_and_per", dict(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                    pdp.Metrics.PRIVACY_ID_COUNT],
                           max_partitions_contributed=3, max_contributions_per_partition=2,
                           min_value=0.0, max_value=10.0)),
    ("mean_var", dict(metrics=[pdp.Metrics.MEAN, pdp.Metrics.VARIANCE, pdp.Metrics.COUNT],
                      max_partitions_contributed=4, max_contributions_per_partition=1,
                      min_value=-1.0, max_value=5.0)),
    ("per_pid", dict(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN],
                     max_contributions=5, min_value=0.0, max_value=10.0)),
    ("cross_sum_pp", dict(metrics=[pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
                          max_partitions_contributed=2, max_contributions_per_partition=1,
                          min_sum_per_partition=-5.0, max_sum_per_partition=20.0)),
    ("count_only", dict(metrics=[pdp.Metrics.COUNT], max_partitions_contributed=2,
                        max_contributions_per_partition=3)),
]


@pytest.mark.parametrize("name,kw", MODES, ids=[m[0] for m in MODES])
@pytest.mark.parametrize("dup", [False, True], ids=["distinct", "dupvalues"])
def test_gpu_bounding_matches_oracle_exactly(built, name, kw, dup):
    """Bounding triggers: the GPU's keyed sampler must pick exactly the
    oracle's records, so partials agree bit for bit (sums to 1e-9)."""
    P = 3000
    pid, pk, val = _dataset(11, 300_000, 8_000, P, dup_values=dup)
    params = pdp.AggregateParams(**kw)
    res, _ = run_engine(pid, pk, val, params, public=list(range(P)), n_partitions=P)
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val if plan.needs_values() else None,
                                 res.last_bound_fields, SEED, public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


def test_gpu_selection_and_noise_match_oracle(built):
    """Private selection (truncated geometric) + Laplace noise: keep flags
    identical, noisy values equal up to one granule."""
    P = 20_000
    pid, pk, val = _dataset(5, 400_000, 50_000, P, zipf=1.1)
    params = pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        max_partitions_contributed=2, max_contributions_per_partition=1,
        min_value=0.0, max_value=10.0)
    res, out = run_engine(pid, pk, val, params, noise=True, n_partitions=P)
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    sel = res.last_select_fields
    keep, o = oracle.select_and_noise(ref, sel, plan.noise_fields(True), SEED,
                                      keep_table=res._table)
    ids = np.nonzero(keep)[0]
    got_ids = out.partition_ids.cpu().numpy()
    assert np.array_equal(np.sort(got_ids), ids)
    assert np.allclose(out.values.cpu().numpy(), o[ids], rtol=1e-12, atol=1e-6)


@pytest.mark.parametrize("target,cap", [(1024, 2048), (16, 2048), (1024, 64), (8, 48)],
                         ids=["default", "3levels", "global_path", "mixed"])
def test_gpu_partition_levels_and_fallback(built, target, cap):
    """Multi-level partitioning and the global-memory path for oversize
    buckets give exactly the oracle's partials (tuning hook dpg_set_tuning)."""
    P = 5000
    pid, pk, val = _dataset(21, 250_000, 2_500, P, zipf=1.1)   # ~100 records / pid
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=8, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    backend.ctx.set_tuning(target, cap)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED,
                                 public_mask=oracle.bitmap(range(P), P))
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


GLOBAL_MODES = [
    # MEAN + VARIANCE without SUM: 24-byte ItemV items
    ("itemv", dict(metrics=[pdp.Metrics.MEAN, pdp.Metrics.VARIANCE, pdp.Metrics.COUNT],
                   max_partitions_contributed=4, max_contributions_per_partition=2,
                   min_value=-1.0, max_value=5.0)),
    # MEAN with SUM: 32-byte Item32 items
    ("item32", dict(metrics=[pdp.Metrics.MEAN, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
                    max_partitions_contributed=3, max_contributions_per_partition=2,
                    min_value=0.0, max_value=10.0)),
    # PER_PRIVACY_ID bounding with MEAN (Item32)
    ("per_pid", dict(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.MEAN],
                     max_contributions=5, min_value=0.0, max_value=10.0)),
]


@pytest.mark.parametrize("name,kw", GLOBAL_MODES, ids=[m[0] for m in GLOBAL_MODES])
def test_gpu_global_path_item_types(built, monkeypatch, name, kw):
    """The global-memory bounding kernel (k_bound_big) for the MEAN/VARIANCE
    item layouts and PER_PRIVACY_ID bounding: every bucket over a 64-record
    capacity (dpg_set_tuning) and the heavy-id filter off (DPG_NO_HEAVY), so
    all records take that kernel; partials equal the oracle's
    (contribution_bounders.py:66-195, combiners.py:382-529)."""
    monkeypatch.setenv("DPG_NO_HEAVY", "1")
    P = 3000
    pid, pk, val = _dataset(31, 200_000, 2_000, P, zipf=1.1)   # ~100 records / pid
    params = pdp.AggregateParams(**kw)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    backend.ctx.set_tuning(1024, 64)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED,
                                 public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


def test_gpu_4096_digit_level(built, monkeypatch):
    """A 12-bit second partition level (4096 digits: the scatter variant
    with 48 KB of digit arrays, 4 digits per thread in the digit bases),
    forced by the level-split hook: partials equal the oracle's."""
    monkeypatch.setenv("DPG_DEBUG_B1", "1")
    P = 3000
    pid, pk, val = _dataset(23, 2_000_000, 1 << 20, P, zipf=1.1)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=2, max_contributions_per_partition=1,
                                 min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, public=list(range(P)), n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED,
                                 public_mask=oracle.bitmap(range(P), P))
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


def test_gpu_empty_and_single_record(built):
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM],
                                 max_partitions_contributed=1, max_contributions_per_partition=1,
                                 min_value=0.0, max_value=1.0)
    _, out = run_engine(np.array([7]), np.array([3]), np.array([0.5]), params, public=[3, 4])
    keys = out.keys()
    vals = out.values.cpu().numpy()
    got = dict(zip(keys, vals.tolist()))
    assert got == {3: [1.0, 0.5], 4: [0.0, 0.0]}


def test_gpu_key_range_error(built):
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT], max_partitions_contributed=1,
                                 max_contributions_per_partition=1)
    with pytest.raises(ValueError, match="outside"):
        run_engine(np.array([1, 2]), np.array([0, 10]), None, params, n_partitions=5)


def test_gpu_determinism_same_seed_and_nonce(built):
    """A release is a pure function of (seed, nonce): the same pair
    reproduces it bit for bit; another nonce (the default: fresh per
    release) draws independent selection and noise."""
    P = 2000
    pid, pk, val = _dataset(3, 200_000, 5_000, P)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=2, max_contributions_per_partition=1,
                                 min_value=0.0, max_value=10.0)
    a = run_engine(pid, pk, val, params, noise=True, n_partitions=P, nonce=42)[1]
    b = run_engine(pid, pk, val, params, noise=True, n_partitions=P, nonce=42)[1]
    assert np.array_equal(a.partition_ids.cpu().numpy(), b.partition_ids.cpu().numpy())
    assert np.allclose(a.values.cpu().numpy(), b.values.cpu().numpy(), rtol=1e-12, atol=1e-6)
    c = run_engine(pid, pk, val, params, noise=True, n_partitions=P, nonce=43)[1]
    ka, kc = a.partition_ids.cpu().numpy(), c.partition_ids.cpu().numpy()
    common = np.intersect1d(ka, kc)
    va = a.values.cpu().numpy()[np.searchsorted(ka, common)]
    vc = c.values.cpu().numpy()[np.searchsorted(kc, common)]
    assert not np.array_equal(ka, kc) or not np.array_equal(va, vc)
    assert (va != vc).all(axis=1).mean() > 0.9


_NO_NOISE = dict(noise_kind=0, family=0, slot_mask=0, n_outputs=0, out_src=[0] * 8,
                 scale=[0.0] * 4, mid=0.0, mean_const=0, msq_const=0,
                 mean_const_value=0.0, msq_const_value=0.0)


@pytest.mark.parametrize("strategy", [pdp.PartitionSelectionStrategy.TRUNCATED_GEOMETRIC,
                                      pdp.PartitionSelectionStrategy.LAPLACE_THRESHOLDING,
                                      pdp.PartitionSelectionStrategy.GAUSSIAN_THRESHOLDING],
                         ids=["tg", "laplace", "gaussian"])
def test_gpu_select_partitions_matches_oracle(built, strategy):
    """DPEngine.select_partitions (dp_engine.py:201-278): cross-partition
    bounding of distinct partitions per privacy id, then private selection;
    the kept set equals the oracle's for the same seed."""
    P = 20_000
    pid, pk, _ = _dataset(21, 300_000, 40_000, P, zipf=1.1)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-5)
    eng = pdp.DPEngine(acc, backend)
    params = pdp.SelectPartitionsParams(max_partitions_contributed=3,
                                        partition_selection_strategy=strategy)
    cols = pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk), n_partitions=P)
    res = eng.select_partitions(cols, params, pdp.DataExtractors("pid", "pk"))
    acc.compute_budgets()
    out = res.materialize()
    ref = oracle.bound_aggregate(pid, pk, None, res.last_bound_fields, SEED)
    got_rows = res.last_partials["rows"].cpu().numpy()
    assert np.array_equal(got_rows, ref["rows"])
    keep, _ = oracle.select_and_noise(ref, res.last_select_fields, _NO_NOISE, SEED,
                                      keep_table=getattr(res, "_table", None))
    want = np.nonzero(keep)[0]
    assert 0 < len(want) < P
    assert np.array_equal(np.sort(out.partition_ids.cpu().numpy()), want)
    assert sorted(res) == want.tolist()


def test_gpu_heavy_privacy_ids(built):
    """A few privacy ids with thousands of records: their buckets overflow the
    LDS chunk capacity, are refined by further hash bits, and the heaviest go
    to the global-memory path; results stay identical to the oracle."""
    rng = np.random.default_rng(77)
    P = 5_000
    light_pid = rng.integers(0, 200_000, 1_500_000)
    heavy = np.repeat(np.arange(10**6, 10**6 + 12), [3000, 2500, 2200, 5000, 9000, 2100,
                                                     1500, 1200, 4000, 2049, 2047, 7000])
    pid = np.concatenate([light_pid, heavy]).astype(np.int64)
    rng.shuffle(pid)
    pk = ((rng.zipf(1.2, len(pid)) - 1) % P).astype(np.int64)
    val = rng.uniform(-1.0, 11.0, len(pid))
    params = pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        max_partitions_contributed=40, max_contributions_per_partition=3,
        min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, public=list(range(P)), n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED,
                                 public_mask=oracle.bitmap(range(P), P))
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("P", [6_000_000, 12_000_000], ids=["P6e6", "P1.2e7"])
def test_gpu_large_partition_space(built, P):
    """More than 1024 ranges of 4096 partitions: the kept pairs are merged
    through two partition-key levels (dpg_api.hip bound_and_reduce); partials
    equal the oracle's."""
    rng = np.random.default_rng(31)
    n = 300_000
    pid = rng.integers(0, 20_000, n).astype(np.int64)
    pk = rng.integers(0, P, n).astype(np.int64)
    pk[: n // 3] = (rng.zipf(1.2, n // 3) - 1) % P   # some heavy partitions too
    val = rng.uniform(0.0, 10.0, n)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=4, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


def test_gpu_wide_records(built):
    """Privacy ids spread over 2^31 values and 4e7 partitions: the packed key
    no longer fits 64 bits, so records travel as R16; more than 7 hash bits
    stay below a fine bucket, so every bucket takes the 256-thread chunk
    kernel (and the refine level).  Partials equal the oracle's."""
    rng = np.random.default_rng(77)
    n, P = 300_000, 40_000_000
    ids = rng.choice(np.int64(2) ** 31, 20_000, replace=False)
    pid = ids[rng.integers(0, ids.size, n)]
    pk = rng.integers(0, P, n).astype(np.int64)
    pk[: n // 2] = (rng.zipf(1.3, n // 2) - 1) % 5000
    val = rng.uniform(-2.0, 12.0, n)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=3, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("mpc", [1, 4, 9])
def test_gpu_candidate_prefilter_and_restart(built, mpc):
    """The wave kernel inserts only records whose pair priority is below a
    per-pid bound; a pid left with fewer than mpc candidate pairs restarts
    the chunk with every record.  Privacy ids here put many records into few
    partitions (bound far too tight: restarts) or spread them over many
    (no restart); partials equal the oracle's either way."""
    rng = np.random.default_rng(90 + mpc)
    P = 4000
    n_pid = 6000
    recs = rng.integers(1, 60, n_pid)                 # records per pid
    parts = np.where(rng.random(n_pid) < 0.5, rng.integers(1, 4, n_pid),
                     rng.integers(10, 50, n_pid))     # distinct partitions per pid
    pid = np.repeat(np.arange(n_pid), recs)
    base = rng.integers(0, P, n_pid)
    off = np.concatenate([rng.integers(0, p, r) for p, r in zip(parts, recs)])
    pk = (np.repeat(base, recs) + off * 37) % P
    order = rng.permutation(len(pid))
    pid, pk = pid[order].astype(np.int64), pk[order].astype(np.int64)
    val = rng.uniform(-1.0, 11.0, len(pid))
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=mpc, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, public=list(range(P)), n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED,
                                 public_mask=oracle.bitmap(range(P), P))
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("name,kw", MODES, ids=[m[0] for m in MODES])
@pytest.mark.parametrize("kernel", ["sort", "hash"])
def test_gpu_small_chunk_kernels_match_oracle(built, monkeypatch, name, kw, kernel):
    """Both small-chunk bounding kernels -- the sort-based default of the
    cross-partition modes (dpg_sortb.h) and the hash-table kernel
    (dpg_wave.h; DPG_BOUND_HASH forces it) -- keep exactly the oracle's
    records, with bounding triggered (mpc 3 over ~40 partitions per id,
    mcpp 2 over hot partitions).  PER_PRIVACY_ID always takes the hash
    kernel; the stage marker says which one ran."""
    if kernel == "hash":
        monkeypatch.setenv("DPG_BOUND_HASH", "1")
    else:
        monkeypatch.delenv("DPG_BOUND_HASH", raising=False)
    P = 3000
    pid, pk, val = _dataset(41, 400_000, 10_000, P, zipf=1.1)
    params = pdp.AggregateParams(**kw)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    ran = [k for k in backend.ctx.stage_times() if k.startswith("bound.kernel=")]
    want = "hash" if (kernel == "hash" or name == "per_pid") else "sort"
    assert ran == ["bound.kernel=" + want]
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val if plan.needs_values() else None,
                                 res.last_bound_fields, SEED, public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


MW_MODES = [m for m in MODES if m[0] in ("cross_and_per", "mean_var", "count_only")]


@pytest.mark.parametrize("name,kw", MW_MODES, ids=[m[0] for m in MW_MODES])
@pytest.mark.parametrize("mw", ["multiwave", "default", "single", "hash_medium"])
def test_gpu_wide_and_medium_chunks_match_oracle(built, monkeypatch, name, kw, mw):
    """Chunks of more than 256 candidate records (two 200-record privacy ids
    per chunk, mpc 100: the pre-filter passes almost everything) and medium
    chunks (one 700-record privacy id per fine bucket) through the
    multi-wave sort kernels (dpg_sortmw.h: 2 waves per wide chunk, 4 per
    medium chunk) -- and, DPG_MW_OFF, through the single-wave 8-element
    kernel -- keep exactly the oracle's records.  The default is the 2-wave
    wide kernel with the streamed single-wave medium pass (dpg_sortb.h tier
    3), whose chunks of too many candidates (here: most, at mpc 100) go to
    the hash-table medium kernel; DPG_MEDIUM_STREAM=0 gives every medium
    chunk to the hash-table kernel, DPG_MW_MEDIUM=1 to the 4-wave one."""
    monkeypatch.delenv("DPG_MW_OFF", raising=False)
    monkeypatch.delenv("DPG_MW_MEDIUM", raising=False)
    monkeypatch.delenv("DPG_MEDIUM_STREAM", raising=False)
    if mw == "single":
        monkeypatch.setenv("DPG_MW_OFF", "1")
    elif mw == "multiwave":
        monkeypatch.setenv("DPG_MW_MEDIUM", "1")
    elif mw == "hash_medium":
        monkeypatch.setenv("DPG_MEDIUM_STREAM", "0")
    rng = np.random.default_rng(77)
    P = 2000
    pid = np.concatenate([np.repeat(np.arange(6000), 200), np.repeat(np.arange(6000, 6300), 700)])
    pid = rng.permutation(pid).astype(np.int64)
    pk = ((rng.zipf(1.1, pid.size) - 1) % P).astype(np.int64)
    val = rng.uniform(-2.0, 12.0, pid.size)
    kw = dict(kw, max_partitions_contributed=100, max_contributions_per_partition=2)
    params = pdp.AggregateParams(**kw)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    st = backend.ctx.stage_times()
    assert ("bound.multiwave" in st) == (mw != "single")
    assert ("bound.medium_deferred" in st) == (mw in ("default", "single"))
    assert st["bound.wide"] > 0.0 and st["bound.medium"] > 0.0
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val if plan.needs_values() else None,
                                 res.last_bound_fields, SEED, public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


@pytest.mark.parametrize("name,kw", MW_MODES, ids=[m[0] for m in MW_MODES])
@pytest.mark.parametrize("size", [600, 1000])
def test_gpu_streamed_medium_chunks_match_oracle(built, monkeypatch, name, kw, size):
    """Medium chunks streamed by single waves (dpg_sortb.h tier 3): one
    privacy id of `size` records per fine bucket, mpc 8, so ~84 candidate
    records each; one id in ten puts its records into three partitions (its
    candidates show fewer than mpc pairs: a restart with the bound lifted,
    then more candidates than the working set holds, so the chunk goes to
    the hash-table kernel).  Partials equal the oracle's."""
    monkeypatch.delenv("DPG_MW_MEDIUM", raising=False)
    monkeypatch.delenv("DPG_MEDIUM_STREAM", raising=False)
    rng = np.random.default_rng(size)
    P = 20_000
    n_pid = 1500
    pid = np.repeat(np.arange(n_pid), size)
    pk = ((rng.zipf(1.1, pid.size) - 1) % P).astype(np.int64)
    few = np.isin(pid, np.arange(0, n_pid, 10))
    pk[few] = rng.integers(0, 3, int(few.sum())) * 7
    perm = rng.permutation(pid.size)
    pid, pk = pid[perm].astype(np.int64), pk[perm]
    val = rng.uniform(-2.0, 12.0, pid.size)
    kw = dict(kw, max_partitions_contributed=8, max_contributions_per_partition=2)
    params = pdp.AggregateParams(**kw)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    st = backend.ctx.stage_times()
    assert "bound.medium_deferred" in st
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val if plan.needs_values() else None,
                                 res.last_bound_fields, SEED, public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


@pytest.mark.parametrize("name,kw", MW_MODES, ids=[m[0] for m in MW_MODES])
@pytest.mark.parametrize("over", ["stream", "heavy_filter"])
def test_gpu_oversize_buckets_match_oracle(built, monkeypatch, name, kw, over):
    """Oversize buckets (a 64-record bucket capacity, dpg_set_tuning; one
    privacy id of ~100 records per bucket): streamed by the sort pass's
    tier 3 from the medium list (default) or cut by the heavy filter into
    heavy chunks (DPG_STREAM_OVER=0).  One id in ten puts its records into
    three partitions: the streamed pass hands its bucket back to the
    global-memory kernel.  Partials equal the oracle's."""
    monkeypatch.delenv("DPG_NO_HEAVY", raising=False)
    monkeypatch.delenv("DPG_MEDIUM_STREAM", raising=False)
    monkeypatch.delenv("DPG_MW_MEDIUM", raising=False)
    monkeypatch.setenv("DPG_STREAM_OVER", "1" if over == "stream" else "0")
    rng = np.random.default_rng(404)
    P = 3000
    n_pid = 2000
    pid = rng.integers(0, n_pid, 200_000)
    pk = ((rng.zipf(1.1, pid.size) - 1) % P).astype(np.int64)
    few = pid % 10 == 3
    pk[few] = rng.integers(0, 3, int(few.sum())) * 11
    pid = pid.astype(np.int64)
    val = rng.uniform(-2.0, 12.0, pid.size)
    kw = dict(kw, max_partitions_contributed=4, max_contributions_per_partition=2)
    params = pdp.AggregateParams(**kw)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    backend.ctx.set_tuning(1024, 64)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"), public_partitions=list(range(P)))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    st = backend.ctx.stage_times()
    assert ("heavy" in st) == (over == "heavy_filter")
    assert "bound.medium" in st
    plan = res.plan
    ref = oracle.bound_aggregate(pid, pk, val if plan.needs_values() else None,
                                 res.last_bound_fields, SEED, public_mask=oracle.bitmap(range(P), P))
    got = {k: (v.cpu().numpy() if v is not None else None) for k, v in res.last_partials.items()}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    for k in ("sum", "nsum", "nsq"):
        if got[k] is not None:
            assert np.allclose(got[k], ref[k], rtol=1e-9, atol=1e-9), k


def test_gpu_wide_packed_sort_and_its_fallback(built):
    """The 2-wave sort kernel's float64-packed keys keep the top 45 - 24 =
    21 bits of a pair priority at 24-bit partition keys: privacy ids of 300
    pairs each (mpc 200: every record a candidate, so every chunk goes to
    the 2-wave pass) collide in those bits in ~2 % of the ids, whose chunks
    re-sort with full keys.  Partials equal the oracle's either way."""
    rng = np.random.default_rng(2424)
    P = 1 << 24
    n_pid, per = 600, 300
    pid = np.repeat(np.arange(n_pid), per)
    pk = rng.integers(0, P, pid.size).astype(np.int64)
    perm = rng.permutation(pid.size)
    pid, pk = pid[perm].astype(np.int64), pk[perm]
    val = rng.uniform(-2.0, 12.0, pid.size)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=200, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    res, _ = run_engine(pid, pk, val, params, n_partitions=P)
    ref = oracle.bound_aggregate(pid, pk, val, res.last_bound_fields, SEED)
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    assert np.array_equal(got["rows"], ref["rows"])
    assert np.array_equal(got["count"], ref["count"])
    assert np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9)
