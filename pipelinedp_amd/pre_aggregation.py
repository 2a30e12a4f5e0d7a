"""The per-(privacy id, partition) pre-aggregate on the device.

One entry per distinct (privacy id, partition) pair -- (pk, count, sum,
n_partitions, n_contributions | leader << 31), 24 bytes (dpg_pair_entry) -- sorted
by partition key, with partition_start[P + 1] delimiting each partition's
pairs.  Utility analysis and the dataset histograms both start from it:

  raw rows       analysis/pre_aggregation.py:19-61 and
                 analysis/contribution_bounders.py:37-77, computed by
                 dpg_preaggregate (no bounding, values summed unclipped);
                 the leader bit marks one pair per privacy id
  pre-aggregated PreAggregateExtractors rows (partition key, (count, sum,
                 n_partitions, n_contributions)) as the reference takes them
                 (pipeline_dp/data_extractors.py PreAggregateExtractors),
                 dictionary-encoded and sorted by key on ingest
"""
import ctypes
import dataclasses
from typing import Any, Optional

import numpy as np
import torch

from pipelinedp_amd import _native
from pipelinedp_amd import columnar

PAIR_DTYPE = np.dtype([("pk", "<u4"), ("count", "<u4"), ("sum", "<f8"), ("np", "<u4"),
                       ("ncl", "<u4")])
assert PAIR_DTYPE.itemsize == ctypes.sizeof(_native.PairEntry) == 24
PAIR_WORDS = PAIR_DTYPE.itemsize // 8   # float64 words per pair (device tensors)
NC_MASK = 0x7FFFFFFF                    # n_contributions bits of "ncl"


@dataclasses.dataclass
class PairSet:
    pairs: torch.Tensor             # device float64[cap, 3] viewed as dpg_pair_entry
    starts: torch.Tensor            # device int64[P + 1]
    n_partitions: int
    n_pairs: int
    key_table: Any                  # dense id -> user key (columnar.decode_keys)
    public_mask: Optional[torch.Tensor]  # device bitmap of public partitions


def device_pairs(col, extractors, backend, public_partitions, dev) -> PairSet:
    """Raw rows -> the pre-aggregate, through dpg_preaggregate."""
    enc = columnar.encode(col, extractors, dev,
                          need_values=extractors.value_extractor is not None,
                          public_partitions=public_partitions)
    P = enc.n_partitions
    bound = _native.BoundParams()
    bound.n_partitions = P
    bound.pid_min, bound.pid_count = enc.pid_min, enc.pid_count
    bound.rec_id_offset = enc.rec_id_offset
    if enc.public_mask is not None:
        bound.public_mask = enc.public_mask.data_ptr()
    cap = max(enc.n, 1)
    pairs = torch.empty((cap, PAIR_WORDS), dtype=torch.float64, device=dev)
    starts = torch.empty(P + 1, dtype=torch.int64, device=dev)
    with torch.cuda.device(dev):
        sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        n_pairs = backend.ctx.preaggregate(
            ctypes.c_void_p(enc.pid.data_ptr()), ctypes.c_void_p(enc.pk.data_ptr()),
            ctypes.c_void_p(enc.value.data_ptr()) if enc.value is not None else None,
            enc.n, bound, ctypes.c_void_p(pairs.data_ptr()), cap,
            ctypes.c_void_p(starts.data_ptr()), sptr)
    return PairSet(pairs, starts, P, n_pairs, enc.key_table, enc.public_mask)


def host_preaggregated_pairs(col, extractors, public_partitions, dev) -> PairSet:
    """PreAggregateExtractors rows -> the pre-aggregate (ingest: the rows
    are host objects; the encoding is the same dictionary encoding as raw
    keys)."""
    rows = col if isinstance(col, list) else list(col)
    keys = [extractors.partition_extractor(r) for r in rows]
    pre = [extractors.preaggregate_extractor(r) for r in rows]
    ids, table, pub_ids = columnar._encode_keys(
        keys, torch.device("cpu"), None if public_partitions is None else list(public_partitions))
    ids = ids.numpy()
    P = max(len(table), 1)
    pub_mask = None
    if public_partitions is not None:
        pub = np.zeros(P, bool)
        pub[np.asarray(pub_ids, np.int64)] = True
        keep = pub[ids]
        ids, pre = ids[keep], [x for x, k in zip(pre, keep) if k]
        pub_mask = torch.from_numpy(np.packbits(pub, bitorder="little")).to(dev)
    order = np.argsort(ids, kind="stable")
    n = len(order)
    arr = np.zeros(max(n, 1), dtype=PAIR_DTYPE)
    if n:
        pre_a = np.asarray(pre, dtype=np.float64).reshape(n, -1)[order]
        arr["pk"][:n] = ids[order]
        arr["count"][:n] = pre_a[:, 0]
        arr["sum"][:n] = pre_a[:, 1]
        arr["np"][:n] = pre_a[:, 2]
        if pre_a.shape[1] > 3:
            # the word's top bit is the leader flag (unused for these rows):
            # n_contributions must fit the remaining 31 bits, as in
            # dpg_preaggregate (a clamp would bin L0 / L1 silently wrong)
            if pre_a[:, 3].max() > NC_MASK or pre_a[:, 3].min() < 0:
                raise ValueError(f"n_contributions must lie in [0, {NC_MASK}] (31 bits)")
            arr["ncl"][:n] = pre_a[:, 3]
    starts = np.searchsorted(ids[order], np.arange(P + 1)).astype(np.int64)
    pairs = torch.from_numpy(arr.view(np.float64).reshape(-1, PAIR_WORDS).copy()).to(dev)
    return PairSet(pairs, torch.from_numpy(starts).to(dev), P, n, table, pub_mask)


def to_numpy(ps: PairSet) -> np.ndarray:
    """The pairs as a structured host array (tests, reports)."""
    a = ps.pairs[:ps.n_pairs].cpu().numpy()
    return a.view(PAIR_DTYPE).reshape(-1)
