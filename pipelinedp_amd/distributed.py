"""Multi-GPU exchange of the per-partition partials (one process per GPU).

Records are sharded by privacy id before they reach a rank (each privacy id
lives on exactly one GPU), so contribution bounding is shard-local and the
only exchange is the merge of the per-partition partials.

Ownership is by partition key: rank r owns partitions r, r + R, r + 2R, ...
(R ranks; `pk mod R`, the identity hash of the dense ids), at local index
pk // R.  Interleaving spreads hot low ids -- an unpermuted Zipf key space
puts most of its occupied partitions at the bottom -- over every rank, so the
sparse exchange's receive volume and every rank's selection work stay
balanced whatever the key order.  The owner runs selection + noise for its
partitions and the kept results are all-gathered (SURVEY.md 8(e);
DESIGN.md section 5).  Two exchanges reach the owner:

* dense -- ONE `reduce_scatter` (sum) of all accumulator arrays packed
  together: 8 B x (A x S + 1) per destination, S = ceil(P / R) (A =
  accumulator arrays; P = 1e6, COUNT+SUM+PID: 24 MB per rank), whatever
  the occupancy;
* sparse -- ONE `all_to_all` with equal splits: every destination gets a
  fixed block of `cap` rows (pk, partial_1..A) (padding rows pk = -1), cap =
  min(S, an upper bound on the partitions one rank can occupy), so no count
  exchange and no host round trip of split sizes is needed.

Neither exchange synchronises the host: the choice between them is made
from host-known sizes only (`choose_exchange`: P, A, R and the occupancy
bound min(P, records, privacy ids x l0), maximised over ranks in the one
collective that already carries the release nonce, `release_header`), and
the split sizes are static.  Every block also carries its sender's
internal-error flag (a bounding whose table overflowed); the owner latches
the sum (`dpg_import_error`), so an error on any rank fails every rank's
`dpg_compact_kept` instead of releasing partials of a mis-bounded shard.

The integer accumulators travel as float64, exact below 2^53 (a rank holds
< 2^32 records).  With gloo (CPU tests, and several ranks sharing one GPU)
the collectives are staged through host memory and the reduce-scatter is an
all_reduce + slice.

Every random draw is keyed by (stream seed, pid, pk) or (stream seed, pk)
with global partition ids -- never by rank -- and the release nonce comes
from rank 0, so the selected-partition set is identical for any world size
(SURVEY.md 8(e)).
"""
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

_PACK_ORDER = ("rows", "count", "sum", "nsum", "nsq")
_PACK_DTYPE = {"rows": torch.int64, "count": torch.int64, "sum": torch.float64,
               "nsum": torch.float64, "nsq": torch.float64}
_I64_MIN = -(1 << 63)


def shard_of(pid: torch.Tensor, world_size: int) -> torch.Tensor:
    """Rank owning each privacy id (multiplicative hash, independent of the
    bits the kernels bucket by)."""
    h = (pid.to(torch.int64) * 0x9E3779B1) & 0xFFFFFFFF
    return ((h * world_size) >> 32).to(torch.int64)


def owned(P: int, world_size: int, rank: int) -> Tuple[int, int, int]:
    """(lo, stride, n): this rank owns partitions lo + i * stride, i < n."""
    n = (P - rank + world_size - 1) // world_size if rank < P else 0
    return rank, world_size, n


def owner_of(pk: torch.Tensor, world_size: int) -> torch.Tensor:
    return pk.to(torch.int64) % world_size


def _is_nccl(group) -> bool:
    return dist.get_backend(group) == "nccl"


def _coll_device(group, device):
    return device if _is_nccl(group) else torch.device("cpu")


def broadcast_u64(x: int, group, device) -> int:
    """Rank 0's 64-bit value on every rank."""
    return release_header(x, 0, group, device)[0]


def release_header(nonce: int, nnz_bound: int, group, device) -> Tuple[int, int]:
    """ONE all_reduce (max) before a release: rank 0's nonce (the others
    contribute INT64_MIN) and the largest occupancy bound over ranks, so
    every rank draws the same streams and takes the same exchange."""
    signed = nonce - (1 << 64) if nonce >= (1 << 63) else nonce
    root = dist.get_global_rank(group, 0) if group is not None else 0
    mine = signed if dist.get_rank() == root else _I64_MIN
    t = torch.tensor([mine, int(nnz_bound)], dtype=torch.int64,
                     device=_coll_device(group, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    got = t.tolist()
    return got[0] & ((1 << 64) - 1), got[1]


def _names(tensors) -> list:
    return [k for k in _PACK_ORDER if tensors.get(k) is not None]


def _interleaved(t: torch.Tensor, P: int, world: int, S: int) -> torch.Tensor:
    """[world, S] float64 view of partition array t: element (r, i) is
    partition i * world + r (zero past P)."""
    x = torch.zeros(S * world, dtype=torch.float64, device=t.device)
    x[:P] = t.to(torch.float64)
    return x.view(S, world).t()


def _unpack_column(col: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    return (col.round().to(torch.int64) if like.dtype == torch.int64 else col).contiguous()


def reduce_scatter_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group,
                            err: Optional[torch.Tensor] = None, ctx=None, stream=None):
    """Sums the dense partials over ranks; returns this rank's partitions
    of every array, (lo, stride, n) and the summed error flags (a [1]
    float64 tensor on the partials' device), with one collective for all
    of them.  Layout [rank][array][S] + one error slot per rank block --
    the C ABI's dpg_pack_partials layout.

    Device partials with the library context `ctx` (the product path): ONE
    pack kernel (dpg_pack_partials: every array interleaved into its rank
    blocks, int64 -> float64, zero past P, the context's error flag in each
    block's last slot) and ONE unpack kernel (dpg_unpack_partials: this
    rank's block back into int64 / float64 slices, a nonzero error sum
    latched for dpg_compact_kept), stream-ordered on `stream` (torch's
    current stream, which the collective waits on) -- one pass over the
    partials each way.  Host partials (the gloo CPU tests, no context): the
    same layout built with torch ops."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = (P + world - 1) // world
    lo, stride, n_local = owned(P, world, rank)
    names = _names(tensors)
    A = len(names)
    dev = tensors[names[0]].device
    # the library's pack / unpack kernels read and write the partials
    # through raw pointers: only contiguous arrays of the layout they assume
    # (int64 rows / count, float64 sums) take them; anything else takes the
    # torch path, which handles any dtype
    fused = (ctx is not None and dev.type == "cuda" and
             all(tensors[k].is_contiguous() and tensors[k].dtype == _PACK_DTYPE[k]
                 and tensors[k].numel() >= P for k in names))
    pack = torch.empty((world, A * S + 1), dtype=torch.float64, device=dev)
    if fused:
        from pipelinedp_amd import _native
        full = _native.Partials(P, *(tensors[k].data_ptr() if tensors.get(k) is not None else None
                                     for k in _PACK_ORDER))
        ctx.pack_partials(full, world, pack.data_ptr(), stream)
    else:
        for j, k in enumerate(names):
            pack[:, j * S:(j + 1) * S] = _interleaved(tensors[k], P, world, S)
        pack[:, A * S] = err.to(dev).reshape(()) if err is not None else 0.0
    if _is_nccl(group):
        part = torch.empty(A * S + 1, dtype=torch.float64, device=dev)
        dist.reduce_scatter_tensor(part, pack.view(-1), op=dist.ReduceOp.SUM, group=group)
    else:
        host = pack.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        part = host[rank].to(dev)
    del pack
    out: Dict[str, Optional[torch.Tensor]] = {k: None for k in _PACK_ORDER}
    if fused:
        from pipelinedp_amd import _native
        for k in names:
            out[k] = torch.empty(max(n_local, 1), dtype=tensors[k].dtype, device=dev)
        sl = _native.Partials(n_local, *(out[k].data_ptr() if out.get(k) is not None else None
                                         for k in _PACK_ORDER))
        lo_k, n_k = ctx.unpack_partials(part.data_ptr(), P, world, rank, sl, stream)
        assert (lo_k, n_k) == (lo, n_local), (lo_k, n_k, lo, n_local)
        for k in names:
            out[k] = out[k][:n_local]
    else:
        for j, k in enumerate(names):
            out[k] = _unpack_column(part[j * S:j * S + n_local], tensors[k])
    return out, (lo, stride, n_local), part[A * S:A * S + 1]


def occupancy_bound(P: int, n_records: int, pid_count: int, l0: int) -> int:
    """Upper bound on the partitions one rank's kept pairs can reach: at
    most one per record, at most l0 per privacy id, at most P."""
    b = min(P, max(0, n_records))
    if pid_count > 0 and l0 > 0:
        b = min(b, pid_count * l0)
    return max(1, b)


def exchange_bytes(P: int, nnz_bound: int, n_arrays: int, world: int = 1) -> Dict[str, int]:
    """Bytes one rank sends in each exchange."""
    S = (P + world - 1) // world
    cap = min(S, nnz_bound)
    return {"reduce_scatter": 8 * world * (n_arrays * S + 1),
            "all_to_all": 8 * world * (cap + 1) * (1 + n_arrays)}


def choose_exchange(P: int, n_arrays: int, world: int, nnz_bound: int, mode: str = "auto") -> str:
    """The exchange of one release, from sizes every rank agrees on (no
    device data): 'auto' takes the sparse all-to-all when its fixed blocks
    are at most half the dense reduce-scatter's bytes."""
    if mode not in ("auto", "reduce_scatter", "all_to_all"):
        raise ValueError(f"unknown exchange {mode!r}")
    if mode != "auto":
        return mode
    b = exchange_bytes(P, nnz_bound, n_arrays, world)
    return "all_to_all" if 2 * b["all_to_all"] <= b["reduce_scatter"] else "reduce_scatter"


def all_to_all_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group,
                        nnz_bound: int, err: Optional[torch.Tensor] = None):
    """Sparse merge: the occupied partitions (rows > 0) of every rank travel
    as (pk, partials...) rows to their owner in fixed blocks of cap rows per
    destination (equal splits: nothing about the occupancy reaches the
    host).  The owner adds them into its dense slice source rank by source
    rank (pks are unique within one source, so every add is conflict-free
    and the merge is deterministic).  Same result as
    reduce_scatter_partials.  A block with more occupied partitions than cap
    (impossible when nnz_bound bounds the occupancy) raises the error flag.

    The send side works on the occupied partitions only: at most K =
    min(P, nnz_bound) of them, taken by one fixed-size nonzero (no host
    sync), ordered by owner with a stable sort, so its temporaries are
    K-sized (the sparse exchange is chosen exactly when K is far below P
    / R: ADVICE r4)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = (P + world - 1) // world
    cap = max(1, min(S, int(nnz_bound)))
    lo, stride, n_local = owned(P, world, rank)
    names = _names(tensors)
    A = len(names)
    dev = tensors[names[0]].device
    K = max(1, min(P, int(nnz_bound)))
    occ = tensors["rows"] > 0
    n_occ = occ.sum()
    idx = torch.nonzero_static(occ, size=K, fill_value=P).view(-1)   # ascending, pad P
    valid = idx < P
    own = torch.where(valid, idx % world, torch.full_like(idx, world))
    order = torch.argsort(own, stable=True)                          # by owner, pk ascending
    idx, own, valid = idx[order], own[order], valid[order]
    cnt = torch.bincount(own, minlength=world + 1)
    start = torch.cumsum(cnt, 0) - cnt
    pos = torch.arange(K, device=dev) - start[own]
    fits = valid & (pos < cap)
    over = ((n_occ > K) | (valid & ~fits).any()).to(torch.float64)
    blk = cap + 1                                                  # header row + cap rows
    sink = world * blk                                             # rows past the cap, padding
    dst = torch.where(fits, own * blk + 1 + pos, torch.full_like(pos, sink))
    safe = torch.where(valid, idx, torch.zeros_like(idx))
    rows = torch.stack([idx.to(torch.float64)] +
                       [tensors[k][safe].to(torch.float64) for k in names], -1)
    send = torch.zeros((sink + 1, 1 + A), dtype=torch.float64, device=dev)
    send[:, 0] = -1.0
    send.index_copy_(0, dst, rows)
    hdr = torch.arange(world, device=dev) * blk
    send[hdr, 0] = -2.0
    send[hdr, 1] = (err.to(dev).reshape(()) if err is not None else 0.0) + over
    send = send[:sink].contiguous()
    nccl = _is_nccl(group)
    if nccl:
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=group)
    else:
        recv = torch.empty_like(send, device="cpu")
        dist.all_to_all_single(recv, send.cpu(), group=group)
        recv = recv.to(dev)
    recv = recv.view(world, blk, 1 + A)
    flags = recv[:, 0, 1].sum().reshape(1)
    acc = torch.zeros((A, n_local + 1), dtype=torch.float64, device=dev)
    for src in range(world):  # source rank order: deterministic sums
        body = recv[src, 1:]
        pk = body[:, 0]
        li = torch.where(pk >= 0, (pk.round().to(torch.int64) - lo) // stride,
                         torch.full_like(pk, n_local, dtype=torch.int64))
        acc.index_add_(1, li, body[:, 1:].t().contiguous())
    out: Dict[str, Optional[torch.Tensor]] = {k: None for k in _PACK_ORDER}
    for j, k in enumerate(names):
        out[k] = _unpack_column(acc[j, :n_local], tensors[k])
    return out, (lo, stride, n_local), flags


def exchange_partials(tensors: Dict[str, Optional[torch.Tensor]], P: int, group,
                      mode: str = "auto", nnz_bound: Optional[int] = None,
                      err: Optional[torch.Tensor] = None, ctx=None, stream=None):
    """Merges the partials of every rank into this rank's partitions with
    the exchange `choose_exchange` picks.  nnz_bound must be the same on
    every rank (release_header); None = P.  ctx / stream: the library
    context and its stream, for the fused pack / unpack kernels of the
    dense exchange.  Returns (tensors, (lo, stride, n), info, error flags)
    where info names the exchange and its per-rank send bytes."""
    names = _names(tensors)
    world = dist.get_world_size(group)
    bound = P if nnz_bound is None else int(nnz_bound)
    chosen = choose_exchange(P, len(names), world, bound, mode)
    if chosen == "all_to_all":
        out, own, flags = all_to_all_partials(tensors, P, group, bound, err)
    else:
        out, own, flags = reduce_scatter_partials(tensors, P, group, err, ctx, stream)
    info = {"mode": chosen, "backend": dist.get_backend(group), "world_size": world,
            "nnz_bound": bound,
            "send_bytes": exchange_bytes(P, bound, len(names), world)[chosen]}
    return out, own, info, flags


def slice_bitmap(mask: torch.Tensor, lo: int, stride: int, n: int) -> torch.Tensor:
    """Bitmap of partitions lo + i * stride (i < n) re-based to bit i."""
    ids = lo + torch.arange(n, device=mask.device) * stride
    bits = ((mask[ids >> 3].to(torch.int64) >> (ids & 7)) & 1).to(torch.uint8)
    padded = torch.zeros(((n + 7) // 8) * 8, dtype=torch.uint8, device=mask.device)
    padded[:n] = bits
    weights = (1 << torch.arange(8, device=mask.device)).to(torch.int64)
    return (padded.view(-1, 8).to(torch.int64) * weights).sum(1).to(torch.uint8)


def all_gather_results(ids: torch.Tensor, vals: torch.Tensor, group):
    """Concatenates every rank's kept (ids, values) in rank order: one size
    exchange, then one all_gather of ids and values packed as float64 rows
    (ids < 2^53 are exact).  Runs after dpg_compact_kept, which has already
    synchronised the host."""
    world = dist.get_world_size(group)
    dev = ids.device
    cdev = _coll_device(group, dev)
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
