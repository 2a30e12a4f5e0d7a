"""Multi-rank exchange logic on CPU (gloo, world size 2): the merge of the
dense per-partition partials (reduce-scatter semantics), the ownership
slices, the bitmap re-basing and the all-gather of the kept results.  The
per-rank partials come from the oracle on a privacy-id-sharded dataset, so
the merged slices must equal the single-process oracle exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle
from pipelinedp_amd import distributed

P = 1000


def _data():
    rng = np.random.default_rng(4)
    n = 20000
    pid = rng.integers(0, 3000, n)
    pk = (rng.zipf(1.2, n) - 1) % P
    val = rng.uniform(0, 5, n)
    return pid, pk, val


FIELDS = dict(mode=0, sum_mode=1, metric_mask=7, max_partitions_contributed=3,
              max_contributions_per_partition=2, max_contributions=0, min_value=0.0,
              max_value=5.0, min_sum_per_partition=0.0, max_sum_per_partition=0.0,
              n_partitions=P)


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pid, pk, val = _data()
    shard = distributed.shard_of(torch.as_tensor(pid), world).numpy()
    m = shard == rank
    # global record ids keep the record sampler identical to the whole run
    part = oracle.bound_aggregate(pid[m], pk[m], val[m], FIELDS, 99, rec_ids=np.nonzero(m)[0])
    tens = {k: torch.as_tensor(part[k]) for k in ("rows", "count", "sum")}
    tens.update(nsum=None, nsq=None)
    if mode == "reduce_scatter":
        out, lo, n = distributed.reduce_scatter_partials(tens, P, dist.group.WORLD)
    else:
        out, lo, n, info = distributed.exchange_partials(tens, P, dist.group.WORLD, mode)
        assert info["mode"] == "all_to_all" and info["world_size"] == world
    # kept results: partitions of this slice with rows > 0, values = counts
    ids = torch.nonzero(out["rows"] > 0).flatten() + lo
    vals = out["count"][ids - lo].to(torch.float64).view(-1, 1)
    g_ids, g_vals = distributed.all_gather_results(ids, vals, dist.group.WORLD)
    bm = torch.as_tensor(oracle.bitmap(np.arange(0, P, 3), P))
    sl = distributed.slice_bitmap(bm, lo, n)
    q.put((rank, lo, n, {k: v.numpy() for k, v in out.items() if v is not None},
           g_ids.numpy(), g_vals.numpy(), sl.numpy()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,mode", [(2, "reduce_scatter"), (2, "all_to_all"),
                                        (3, "all_to_all")])
def test_rank_merge_equals_single_process(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pid, pk, val = _data()
    ref = oracle.bound_aggregate(pid, pk, val, FIELDS, 99)
    for rank, lo, n, out, g_ids, g_vals, sl in res:
        assert np.array_equal(out["rows"], ref["rows"][lo:lo + n])
        assert np.array_equal(out["count"], ref["count"][lo:lo + n])
        assert np.allclose(out["sum"], ref["sum"][lo:lo + n], rtol=1e-12)
        want_ids = np.nonzero(ref["rows"] > 0)[0]
        assert np.array_equal(np.sort(g_ids), want_ids)
        bits = np.unpackbits(sl, bitorder="little")[:n]
        assert np.array_equal(np.nonzero(bits)[0] + lo, np.arange(0, P, 3)[(np.arange(0, P, 3) >= lo) & (np.arange(0, P, 3) < lo + n)])
    chunk = (P + world - 1) // world
    assert sorted(r[1] for r in res) == [r * chunk for r in range(world)]


def _choose_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Pbig = 1_000_000
    rows = torch.zeros(Pbig, dtype=torch.int64)
    # rank 1 is the fuller one: the choice must follow the largest occupancy
    nnz = 1000 if rank == 0 else (50_000 if q is not None and world == 2 else 1000)
    rows[torch.arange(nnz) * 7] = 1
    sparse = distributed.choose_exchange(rows, Pbig, 3, dist.group.WORLD)
    rows[:] = 1
    dense = distributed.choose_exchange(rows, Pbig, 3, dist.group.WORLD)
    forced = distributed.choose_exchange(rows, Pbig, 3, dist.group.WORLD, "all_to_all")
    q.put((rank, sparse, dense, forced))
    dist.destroy_process_group()


def test_exchange_choice_is_global_and_by_occupancy():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_choose_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sparse, dense, forced in res:
        assert sparse == ("all_to_all", 50_000)   # max over ranks, same on both
        assert dense == ("reduce_scatter", 1_000_000)
        assert forced == ("all_to_all", 1_000_000)
    b = distributed.exchange_bytes(100_000_000, 10_000_000, 5)
    assert b["all_to_all"] * 6 < b["reduce_scatter"]


def test_shard_is_deterministic_and_balanced():
    pid = torch.arange(100000)
    s = distributed.shard_of(pid, 8)
    assert s.min() >= 0 and s.max() < 8
    counts = torch.bincount(s, minlength=8).numpy()
    assert counts.min() > 0.9 * counts.mean()
    assert torch.equal(s, distributed.shard_of(pid, 8))
