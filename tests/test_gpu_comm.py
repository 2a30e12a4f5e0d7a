"""The C-ABI RCCL communicator (dpg_comm_unique_id / dpg_ctx_create_comm /
dpg_reduce_scatter_partials): the partial merge a host without PyTorch uses
across GPUs.  One GPU here, so one rank: the pack -> ncclReduceScatter ->
unpack round trip must return the partials unchanged (integer arrays exact
through float64).  Several ranks go through the same calls with one
communicator per GPU; RCCL refuses two ranks on one device, so that case
is covered by the torch.distributed path's tests (test_gpu_multirank.py),
and the pack / unpack layout for several ranks by dpg_pack_partials /
dpg_unpack_partials (the same kernels, host-summed) below."""
import os

import numpy as np
import pytest
import torch

SEED = 0xC033

pytestmark = pytest.mark.gpu


def _aggregate():
    import pipelinedp_amd as pdp
    rng = np.random.default_rng(31)
    P = 7_001
    pid = rng.integers(0, 30_000, 400_000).astype(np.int64)
    pk = ((rng.zipf(1.1, pid.size) - 1) % P).astype(np.int64)
    val = rng.uniform(-1.0, 11.0, pid.size)
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                          pdp.Metrics.PRIVACY_ID_COUNT],
                                 max_partitions_contributed=4, max_contributions_per_partition=2,
                                 min_value=0.0, max_value=10.0)
    res = pdp.DPEngine(acc, backend).aggregate(
        pdp.ColumnarData(pid=torch.as_tensor(pid), pk=torch.as_tensor(pk),
                         value=torch.as_tensor(val), n_partitions=P),
        params, pdp.DataExtractors("pid", "pk", "value"))
    acc.compute_budgets()
    res.noise_enabled = False
    res.materialize()
    return backend, res.last_partials, P


def test_rccl_reduce_scatter_partials_one_rank(built):
    from pipelinedp_amd import _native
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    backend, parts, P = _aggregate()
    ctx = backend.ctx
    uid = ctx.comm_unique_id()
    assert len(uid) == _native.COMM_ID_BYTES
    ctx.create_comm(uid, 0, 1)
    dev = parts["rows"].device
    out = {k: torch.full_like(v, -7) for k, v in parts.items() if v is not None}
    ptr = lambda d, k: d[k].data_ptr() if d.get(k) is not None else None  # noqa: E731
    full = _native.Partials(P, *(ptr(parts, k) for k in ("rows", "count", "sum", "nsum", "nsq")))
    sl = _native.Partials(P, *(ptr(out, k) for k in ("rows", "count", "sum", "nsum", "nsq")))
    stream = torch.cuda.current_stream(dev)
    lo, n = ctx.reduce_scatter_partials(full, sl, stream.cuda_stream)
    torch.cuda.synchronize()
    assert (lo, n) == (0, P)   # one rank owns every partition
    for k, v in out.items():
        assert torch.equal(v, parts[k]), k
    assert int(out["rows"].sum()) > 0


def test_reduce_scatter_without_communicator_fails(built):
    import pipelinedp_amd as pdp
    from pipelinedp_amd import _native
    backend = pdp.MI355XBackend(device=0, seed=SEED)
    t = torch.zeros(16, dtype=torch.int64, device="cuda:0")
    p = _native.Partials(16, t.data_ptr(), t.data_ptr(), None, None, None)
    with pytest.raises(_native.NativeError):
        backend.ctx.reduce_scatter_partials(p, p, None)


@pytest.mark.parametrize("R", [2, 3])
def test_pack_unpack_layout_for_several_ranks(built, R):
    """The C-ABI pack layout equals the torch path's
    (distributed.reduce_scatter_partials): rank r's block is [array][S] with
    element i = partition i * R + r (interleaved ownership), zero padded past
    P, then the sender's error flag; R emulated ranks' packs summed on the
    host and unpacked per rank give every rank its partitions of the sum."""
    from pipelinedp_amd import _native
    backend, parts, P = _aggregate()
    ctx = backend.ctx
    dev = parts["rows"].device
    names = [k for k in ("rows", "count", "sum", "nsum", "nsq") if parts.get(k) is not None]
    A = len(names)
    S = (P + R - 1) // R
    stream = torch.cuda.current_stream(dev).cuda_stream
    ptr = lambda d, k: d[k].data_ptr() if d.get(k) is not None else None  # noqa: E731
    # rank r holds the partials scaled by r + 1 (integers stay integers)
    ranks = [{k: (v * (r + 1)) for k, v in parts.items() if v is not None} for r in range(R)]
    packs = []
    for r in range(R):
        full = _native.Partials(P, *(ptr(ranks[r], k) for k in ("rows", "count", "sum", "nsum",
                                                                  "nsq")))
        pack = torch.full((R, A * S + 1), -5.0, dtype=torch.float64, device=dev)
        ctx.pack_partials(full, R, pack.data_ptr(), stream)
        torch.cuda.synchronize()
        expect = torch.zeros((R, A * S + 1), dtype=torch.float64, device=dev)
        for j, k in enumerate(names):
            x = torch.zeros(R * S, dtype=torch.float64, device=dev)
            x[:P] = ranks[r][k].to(torch.float64)
            expect[:, j * S:(j + 1) * S] = x.view(S, R).t()
        assert torch.equal(pack, expect), r      # error slot 0.0: no bounding error
        packs.append(pack)
    total = sum(packs)
    scale = R * (R + 1) // 2
    for r in range(R):
        part = total[r].contiguous()
        out = {k: torch.full((S,), -7, dtype=parts[k].dtype, device=dev) for k in names}
        sl = _native.Partials(S, *(ptr(out, k) for k in ("rows", "count", "sum", "nsum", "nsq")))
        lo, n = ctx.unpack_partials(part.data_ptr(), P, R, r, sl, stream)
        torch.cuda.synchronize()
        own = torch.arange(r, P, R, device=dev)
        assert lo == r and n == own.numel()
        for k in names:
            want = parts[k][own] * scale
            if parts[k].dtype == torch.int64:
                assert torch.equal(out[k][:n], want), (r, k)
            else:
                assert torch.allclose(out[k][:n], want, rtol=1e-12, atol=1e-9), (r, k)


def test_error_flag_travels_and_fails_compaction(built):
    """a rank whose bounding latched an internal error must fail
    every rank's release.  The flag of a sender travels in the exchange
    (dpg_unpack_partials / dpg_import_error latch it) and the receiver's
    dpg_compact_kept then fails; a clean block leaves it unharmed."""
    from pipelinedp_amd import _native
    backend, parts, P = _aggregate()
    ctx = backend.ctx
    dev = parts["rows"].device
    stream = torch.cuda.current_stream(dev).cuda_stream
    flag = torch.full((1,), -1.0, dtype=torch.float64, device=dev)
    ctx.export_error(flag.data_ptr(), stream)
    torch.cuda.synchronize()
    assert float(flag) == 0.0                     # the aggregate above was clean
    keep = torch.ones(8, dtype=torch.uint8, device=dev)
    ids = torch.empty(8, dtype=torch.int64, device=dev)
    zero = torch.zeros(2, dtype=torch.float64, device=dev)
    ctx.import_error(zero.data_ptr(), 2, stream)
    assert ctx.compact(keep.data_ptr(), None, 8, 0, ids.data_ptr(), None, stream) == 8
    # an unpacked block whose error slot is set (another rank's flag)
    names = [k for k in ("rows", "count", "sum") if parts.get(k) is not None]
    part = torch.zeros(len(names) * P + 1, dtype=torch.float64, device=dev)
    part[-1] = 1.0
    out = {k: torch.empty(P, dtype=parts[k].dtype, device=dev) for k in names}
    sl = _native.Partials(P, *(out[k].data_ptr() if k in out else None
                               for k in ("rows", "count", "sum", "nsum", "nsq")))
    ctx.unpack_partials(part.data_ptr(), P, 1, 0, sl, stream)
    with pytest.raises(_native.NativeError, match="internal"):
        ctx.compact(keep.data_ptr(), None, 8, 0, ids.data_ptr(), None, stream)


def test_async_compaction_matches_and_latches_error(built):
    """dpg_compact_kept_async: the same ids and rows as the synchronising
    compaction, the count and the bounding's error bits in a device word;
    DeviceResult reads them on first use and raises the internal error
    there (what the synchronising call raises at once)."""
    from pipelinedp_amd import _native
    from pipelinedp_amd.device_aggregate import DeviceResult
    backend, parts, P = _aggregate()
    ctx = backend.ctx
    dev = parts["rows"].device
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device="cpu").manual_seed(7)
    n, n_out = 5000, 3
    keep = (torch.rand(n, generator=g) < 0.3).to(torch.uint8).to(dev)
    out = torch.randn(n * n_out, generator=g, dtype=torch.float64).to(dev)
    ids_s = torch.empty(n, dtype=torch.int64, device=dev)
    vals_s = torch.empty(n * n_out, dtype=torch.float64, device=dev)
    k = ctx.compact(keep.data_ptr(), out.data_ptr(), n, n_out, ids_s.data_ptr(),
                    vals_s.data_ptr(), stream)
    ids_a = torch.empty(n, dtype=torch.int64, device=dev)
    vals_a = torch.empty(n * n_out, dtype=torch.float64, device=dev)
    info = torch.full((2,), -1, dtype=torch.int64, device=dev)
    ctx.compact_async(keep.data_ptr(), out.data_ptr(), n, n_out, ids_a.data_ptr(),
                      vals_a.data_ptr(), info.data_ptr(), stream)
    res = DeviceResult(ids_a, vals_a, ("a", "b", "c"), None, pending=(info, n_out, 1, 0))
    assert k == int(keep.sum())
    assert torch.equal(res.partition_ids, ids_s[:k])
    assert torch.equal(res.values, vals_s[:k * n_out].view(k, n_out))
    assert torch.equal(res.partition_ids, torch.nonzero(keep).flatten())
    # a latched internal error (as an exchanged block carries it) is raised
    # when the result is first read
    names = [k for k in ("rows", "count", "sum") if parts.get(k) is not None]
    part = torch.zeros(len(names) * P + 1, dtype=torch.float64, device=dev)
    part[-1] = 1.0
    tgt = {k: torch.empty(P, dtype=parts[k].dtype, device=dev) for k in names}
    sl = _native.Partials(P, *(tgt[k].data_ptr() if k in tgt else None
                               for k in ("rows", "count", "sum", "nsum", "nsq")))
    ctx.unpack_partials(part.data_ptr(), P, 1, 0, sl, stream)
    info2 = torch.empty(2, dtype=torch.int64, device=dev)
    ctx.compact_async(keep.data_ptr(), out.data_ptr(), n, n_out, ids_a.data_ptr(),
                      vals_a.data_ptr(), info2.data_ptr(), stream)
    bad = DeviceResult(ids_a, vals_a, ("a", "b", "c"), None, pending=(info2, n_out, 1, 0))
    with pytest.raises(_native.NativeError, match="internal"):
        bad.partition_ids
