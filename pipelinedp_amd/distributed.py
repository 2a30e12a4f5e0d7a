"""Multi-GPU exchange of the per-partition partials (one process per GPU).

Records are sharded by privacy id before they reach a rank (each privacy id
lives on exactly one GPU), so contribution bounding is shard-local and the
only exchange is the merge of the per-partition partials.  Every rank owns
an equal, contiguous slice of the partition space; the owner runs
selection + noise for its slice, and the kept results are all-gathered.
Two exchanges reach that slice:

* dense -- ONE `reduce_scatter` (sum) of all accumulator arrays packed
  together: 8 B x P x A per rank (A = accumulator arrays; P = 1e6,
  COUNT+SUM+PID: 24 MB), whatever the occupancy;
* sparse -- ONE `all_to_all` of the occupied partitions only, as rows
  (pk, partial_1..A) routed to the rank owning pk: 8 B x (1 + A) x nnz per
  rank (nnz = partitions with a kept pair on that rank), after a
  world-sized count exchange.  Config 4 (P = 1e8, ~1e7 occupied) moves
  ~0.5 GB instead of 4 GB per rank.

`exchange_partials` picks the cheaper one from the largest nnz over ranks
(one all_reduce of a scalar, so every rank takes the same branch).  The
integer accumulators travel as float64, which is exact below 2^53 (a rank
holds < 2^32 records, so no count comes near it).  With gloo (CPU tests,
and several ranks sharing one GPU) the collectives are staged through host
memory and the reduce-scatter is an all_reduce + slice.

Every random draw is keyed by (stream seed, pid, pk) or (stream seed, pk)
with global partition ids -- never by rank -- and the release nonce is
broadcast from rank 0, so the selected-partition set is identical for any
world size.
"""
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

_PACK_ORDER = ("rows", "count", "sum", "nsum", "nsq")


def shard_of(pid: torch.Tensor, world_size: int) -> torch.Tensor:
    """Rank owning each privacy id (multiplicative hash, independent of the
    bits the kernels bucket by)."""
    h = (pid.to(torch.int64) * 0x9E3779B1) & 0xFFFFFFFF
    return ((h * world_size) >> 32).to(torch.int64)


def slice_bounds(P: int, world_size: int, rank: int) -> Tuple[int, int]:
    chunk = (P + world_size - 1) // world_size
    lo = min(P, rank * chunk)
    return lo, min(P, lo + chunk) - lo


def _is_nccl(group) -> bool:
    return dist.get_backend(group) == "nccl"


def broadcast_u64(x: int, group, device) -> int:
    """Rank 0's 64-bit value on every rank (the release nonce)."""
    signed = x - (1 << 64) if x >= (1 << 63) else x
    dev = device if _is_nccl(group) else torch.device("cpu")
    t = torch.tensor([signed], dtype=torch.int64, device=dev)
    dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0,
                   group=group)
    return int(t.item()) & ((1 << 64) - 1)


def reduce_scatter_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group
                            ) -> Tuple[Dict[str, Optional[torch.Tensor]], int, int]:
    """Sums the dense partials over ranks and returns this rank's slice
    [lo, lo + n) of every array, with one collective for all of them."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    chunk = (P + world - 1) // world
    padded = chunk * world
    lo, n_local = slice_bounds(P, world, rank)
    names = [k for k in _PACK_ORDER if tensors.get(k) is not None]
    like = tensors[names[0]]
    dev = like.device
    # layout [world][array][chunk]: rank r's reduce-scatter block is the
    # contiguous [array][chunk] slab of its partition slice
    pack = torch.zeros((len(names), padded), dtype=torch.float64, device=dev)
    for j, k in enumerate(names):
        pack[j, :P] = tensors[k].to(torch.float64)
    pack = pack.view(len(names), world, chunk).transpose(0, 1).contiguous()
    if _is_nccl(group):
        part = torch.empty((len(names), chunk), dtype=torch.float64, device=dev)
        dist.reduce_scatter_tensor(part, pack, op=dist.ReduceOp.SUM, group=group)
    else:
        host = pack.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        part = host[rank].to(dev)
    out: Dict[str, Optional[torch.Tensor]] = {k: None for k in _PACK_ORDER}
    for j, k in enumerate(names):
        col = part[j, :n_local]
        out[k] = (col.round().to(torch.int64) if tensors[k].dtype == torch.int64
                  else col).contiguous()
    return out, lo, n_local


def _names(tensors) -> list:
    return [k for k in _PACK_ORDER if tensors.get(k) is not None]


def exchange_bytes(P: int, nnz: int, n_arrays: int) -> Dict[str, int]:
    """Bytes one rank contributes to each exchange (the send side)."""
    return {"reduce_scatter": 8 * n_arrays * P, "all_to_all": 8 * (1 + n_arrays) * nnz}


def choose_exchange(rows: torch.Tensor, P: int, n_arrays: int, group, mode: str = "auto"
                    ) -> Tuple[str, int]:
    """The exchange every rank of `group` uses, and the largest occupancy
    over ranks.  'auto' takes the sparse all-to-all when its rows are at
    most half the dense reduce-scatter's bytes (the count exchange and the
    host round trip for the split sizes cost latency the dense path does
    not pay)."""
    if mode not in ("auto", "reduce_scatter", "all_to_all"):
        raise ValueError(f"unknown exchange {mode!r}")
    nnz = int(torch.count_nonzero(rows).item())
    dev = rows.device if _is_nccl(group) else torch.device("cpu")
    t = torch.tensor([nnz], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    nnz_max = int(t.item())
    if mode != "auto":
        return mode, nnz_max
    b = exchange_bytes(P, nnz_max, n_arrays)
    return ("all_to_all" if 2 * b["all_to_all"] <= b["reduce_scatter"] else "reduce_scatter",
            nnz_max)


def all_to_all_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group
                        ) -> Tuple[Dict[str, Optional[torch.Tensor]], int, int]:
    """Sparse merge: the occupied partitions (rows > 0) of every rank travel
    as (pk, partials...) rows to the rank owning pk's slice; the owner adds
    them into its dense slice, source rank by source rank (pks are unique
    within one source, so every add is conflict-free and the merge is
    deterministic).  Same result as reduce_scatter_partials."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    chunk = (P + world - 1) // world
    lo, n_local = slice_bounds(P, world, rank)
    names = _names(tensors)
    dev = tensors[names[0]].device
    nccl = _is_nccl(group)
    cdev = dev if nccl else torch.device("cpu")
    idx = torch.nonzero(tensors["rows"]).flatten()  # ascending, so grouped by owner
    send = torch.empty((idx.numel(), 1 + len(names)), dtype=torch.float64, device=dev)
    send[:, 0] = idx.to(torch.float64)
    for j, k in enumerate(names):
        send[:, 1 + j] = tensors[k][idx].to(torch.float64)
    send_counts = torch.bincount(idx // chunk, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts, device=cdev)
    dist.all_to_all_single(recv_counts, send_counts.to(cdev), group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    recv = torch.empty((sum(rc), 1 + len(names)), dtype=torch.float64, device=cdev)
    dist.all_to_all_single(recv, send.to(cdev), output_split_sizes=rc, input_split_sizes=sc,
                           group=group)
    recv = recv.to(dev)
    acc = torch.zeros((len(names), n_local), dtype=torch.float64, device=dev)
    o = 0
    for c in rc:  # source rank order
        if c:
            blk = recv[o:o + c]
            li = blk[:, 0].round().to(torch.int64) - lo
            acc[:, li] += blk[:, 1:].t()
        o += c
    out: Dict[str, Optional[torch.Tensor]] = {k: None for k in _PACK_ORDER}
    for j, k in enumerate(names):
        col = acc[j]
        out[k] = (col.round().to(torch.int64) if tensors[k].dtype == torch.int64
                  else col).contiguous()
    return out, lo, n_local


def exchange_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group,
                      mode: str = "auto"):
    """Merges the partials of every rank into this rank's slice with the
    exchange `choose_exchange` picks.  Returns (slice tensors, lo, n,
    info) where info names the exchange and its per-rank send bytes."""
    names = _names(tensors)
    chosen, nnz_max = choose_exchange(tensors["rows"], P, len(names), group, mode)
    if chosen == "all_to_all":
        out, lo, n = all_to_all_partials(tensors, P, group)
    else:
        out, lo, n = reduce_scatter_partials(tensors, P, group)
    info = {"mode": chosen, "backend": dist.get_backend(group),
            "world_size": dist.get_world_size(group), "nnz_max": nnz_max,
            "send_bytes": exchange_bytes(P, nnz_max, len(names))[chosen]}
    return out, lo, n, info


def slice_bitmap(mask: torch.Tensor, lo: int, n: int) -> torch.Tensor:
    """Bitmap of partitions [lo, lo + n) re-based to bit 0."""
    ids = torch.arange(lo, lo + n, device=mask.device)
    bits = ((mask[ids >> 3].to(torch.int64) >> (ids & 7)) & 1).to(torch.uint8)
    padded = torch.zeros(((n + 7) // 8) * 8, dtype=torch.uint8, device=mask.device)
    padded[:n] = bits
    weights = (1 << torch.arange(8, device=mask.device)).to(torch.int64)
    return (padded.view(-1, 8).to(torch.int64) * weights).sum(1).to(torch.uint8)


def all_gather_results(ids: torch.Tensor, vals: torch.Tensor, group):
    """Concatenates every rank's kept (ids, values) in rank order: one size
    exchange, then one all_gather of ids and values packed as float64 rows
    (ids < 2^32 are exact)."""
    world = dist.get_world_size(group)
    nccl = _is_nccl(group)
    dev = ids.device
    cdev = dev if nccl else torch.device("cpu")
    n = torch.tensor([ids.numel()], dtype=torch.int64, device=cdev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    cols = vals.shape[1] if vals.dim() == 2 else 0
    buf = torch.zeros((m, 1 + cols), dtype=torch.float64, device=cdev)
    buf[:ids.numel(), 0] = ids.to(torch.float64).to(cdev)
    if cols:
        buf[:ids.numel(), 1:] = vals.to(cdev)
    got = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(got, buf, group=group)
    rows = torch.cat([g[:s] for g, s in zip(got, sizes)]).to(dev)
    return rows[:, 0].round().to(torch.int64), rows[:, 1:].to(vals.dtype).contiguous()
