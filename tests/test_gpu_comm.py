"""The C-ABI RCCL communicator (dpg_comm_unique_id / dpg_ctx_create_comm /
dpg_reduce_scatter_partials): the partial merge a host without PyTorch uses
across GPUs.  One GPU here, so one rank: the pack -> ncclReduceScatter ->
unpack round trip must return the partials unchanged (integer arrays exact
through float64).  Several ranks go through the same calls with one
communicator per GPU; RCCL refuses two ranks on one device, so that case
is covered by the torch.distributed path's tests (test_gpu_multirank.py)."""
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
    assert (lo, n) == (0, P)
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
