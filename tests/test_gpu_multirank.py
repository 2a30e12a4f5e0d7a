"""Two ranks on GPU 0 (gloo process group, since RCCL refuses two ranks on
one device) run DPEngine.aggregate through DeviceAggregation with the
process group set.  For the same seed and nonce the merged partials, the
selected-partition set and the noised values equal the one-rank release of
the same dataset (north star: "same selected-partition set as the 1-GPU run
given the same RNG seed")."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SEED, NONCE, P = 0xAB5EED, 0x1234ABCD, 30_000
WORLD = 2


def _dataset():
    """Privacy-id-sharded dataset: records ordered shard by shard, so rank r
    holds one contiguous block and its global record ids are offset + i."""
    from pipelinedp_amd import distributed
    rng = np.random.default_rng(12)
    n = 600_000
    pid = rng.integers(0, 40_000, n).astype(np.int64)
    pk = ((rng.zipf(1.1, n) - 1) % P).astype(np.int64)
    val = rng.uniform(-1.0, 11.0, n)
    shard = distributed.shard_of(torch.as_tensor(pid), WORLD).numpy()
    order = np.argsort(shard, kind="stable")
    starts = np.searchsorted(shard[order], np.arange(WORLD + 1))
    return pid[order], pk[order], val[order], starts


def _params():
    import pipelinedp_amd as pdp
    return pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        max_partitions_contributed=3, max_contributions_per_partition=2,
        min_value=0.0, max_value=10.0)


def _release(pid, pk, val, offset, group):
    import pipelinedp_amd as pdp
    backend = pdp.MI355XBackend(device=0, seed=SEED, process_group=group)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    cols = pdp.ColumnarData(pid=torch.from_numpy(pid).cuda(), pk=torch.from_numpy(pk).cuda(),
                            value=torch.from_numpy(val).cuda(), n_partitions=P,
                            record_id_offset=int(offset))
    res = pdp.DPEngine(acc, backend).aggregate(cols, _params(),
                                               pdp.DataExtractors("pid", "pk", "value"))
    acc.compute_budgets()
    res.nonce = NONCE
    out = res.materialize()
    part, lo, stride, n = res.last_slice
    return (lo, stride, n, {k: v.cpu().numpy() for k, v in part.items() if v is not None},
            out.partition_ids.cpu().numpy(), out.values.cpu().numpy(), res.nonce)


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        pid, pk, val, starts = _dataset()
        a, b = starts[rank], starts[rank + 1]
        q.put((rank,) + _release(pid[a:b], pk[a:b], val[a:b], a, dist.group.WORLD))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_equal_one_rank(built):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=100) for _ in range(WORLD)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    pid, pk, val, _ = _dataset()
    lo1, s1, n1, full, ids1, vals1, nonce1 = _release(pid, pk, val, 0, None)
    assert (lo1, s1, n1) == (0, 1, P)
    for rank, lo, stride, n, part, ids, vals, nonce in res:
        assert nonce == NONCE
        # interleaved ownership: rank r owns r, r + WORLD, ...
        assert lo == rank and stride == WORLD and n == P // WORLD
        own = np.arange(rank, P, WORLD)
        assert np.array_equal(part["rows"], full["rows"][own])
        assert np.array_equal(part["count"], full["count"][own])
        assert np.allclose(part["sum"], full["sum"][own], rtol=1e-12, atol=1e-9)
        # every rank holds the gathered release: same set, same values
        assert np.array_equal(np.sort(ids), np.sort(ids1))
        o, o1 = np.argsort(ids), np.argsort(ids1)
        assert np.allclose(vals[o], vals1[o1], rtol=1e-12, atol=1e-6)
    assert 0 < len(ids1) < P
