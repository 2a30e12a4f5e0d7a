"""Ingest: turn the user's collection into device columns for the kernels.

The reference extracts `(privacy_id, partition_key, value)` per row with the
DataExtractors callables (dp_engine.py:384-397).  The MI355X path keeps the
same extractors but prefers columnar input:

* `ColumnarData` / a mapping of columns (numpy arrays or torch tensors,
  ideally already on the GPU).  An extractor is then a column name or a
  callable applied to the whole container.
* Any other iterable is treated as rows; the extractors run per row on the
  host (reference behaviour, slow, meant for small inputs).

Keys: the kernels need integer privacy ids spanning at most 2^32 values and
dense partition ids in [0, P).  Integer keys that already satisfy this are
used as they are; anything else (strings, tuples, ints spread wider) is
dictionary-encoded (`unique` + inverse), and the partition dictionary maps
results back.  Encoding is ingest, not part of the DP computation.
"""
import dataclasses
from collections.abc import Mapping
from typing import Any, Optional, Sequence, Tuple

import numpy as np
import torch

_PID_SPAN = 1 << 32  # privacy ids of one call must span at most 2^32 values


@dataclasses.dataclass
class ColumnarData:
    """Columnar collection for DPEngine.aggregate on the MI355X backend.

    `n_partitions`: if given, `pk` must already hold dense ids in
    [0, n_partitions) and is passed to the device unchecked (the kernel still
    rejects out-of-range keys with ValueError).

    `privacy_id_range`: optional (lo, hi) with every privacy id in [lo, hi),
    hi - lo <= 2^32; saves the device a min/max pass (out-of-range ids raise
    ValueError).  `record_id_offset`: global id of record 0 -- the record
    sampler is keyed by (pid, pk, record id), so the shards of one dataset,
    each given its offset, sample exactly like the whole."""
    pid: Any = None
    pk: Any = None
    value: Any = None
    n_partitions: Optional[int] = None
    privacy_id_range: Optional[Tuple[int, int]] = None
    record_id_offset: int = 0

    def __getitem__(self, name):
        return getattr(self, name)

    def __len__(self):
        return len(self.pk)

    def __bool__(self):
        return self.pk is not None and len(self.pk) > 0


@dataclasses.dataclass
class EncodedInput:
    pid: Optional[torch.Tensor]
    pk: torch.Tensor
    value: Optional[torch.Tensor]
    n: int
    n_partitions: int
    key_table: Optional[Sequence]  # dense id -> original key (None: identity)
    public_mask: Optional[torch.Tensor] = None  # uint8 bitmap on the device
    public_count: int = 0
    pid_min: int = 0
    pid_count: int = 0        # 0: unknown (the device reduces min / max)
    rec_id_offset: int = 0
    partitions_declared: bool = False  # dense ids in [0, n_partitions) given by the caller


def _extract(col, extractor):
    if extractor is None:
        return None
    if isinstance(extractor, str):
        return col[extractor]
    return extractor(col)


def _is_columnar(col) -> bool:
    return isinstance(col, (ColumnarData, Mapping))


def _to_tensor(x, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device) if x.device != device else x
    a = np.asarray(x)
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _integer_like(x) -> bool:
    if isinstance(x, torch.Tensor):
        return not x.is_floating_point() and not x.is_complex() and x.dtype != torch.bool
    return np.asarray(x).dtype.kind in "iu"


def _is_int_key(k) -> bool:
    return isinstance(k, (int, np.integer)) and not isinstance(k, bool)


def _encode_keys(values, device, extra=None):
    """Dictionary-encodes arbitrary keys; returns (ids tensor, key table,
    ids of `extra`)."""
    if isinstance(values, torch.Tensor) and _integer_like(values):
        extra_i = None
        if extra is not None:
            extra = list(extra)
            if not all(_is_int_key(k) for k in extra):
                # integer data keys, public partitions with other keys: the
                # general (object) encoding; those partitions come out empty
                return _encode_keys(values.cpu().numpy().astype(object), device, extra)
            extra_i = torch.as_tensor(np.asarray(extra, dtype=np.int64), device=values.device)
        both = values if extra is None else torch.cat([values, extra_i])
        uniq, inv = torch.unique(both, return_inverse=True)
        n = values.numel()
        return (inv[:n].to(torch.int64).to(device), uniq.cpu().numpy(),
                None if extra is None else inv[n:].cpu().numpy())
    arr = np.asarray(values, dtype=object) if not isinstance(values, np.ndarray) else values
    if extra is not None:
        arr = np.concatenate([np.asarray(arr, dtype=object),
                              np.asarray(list(extra), dtype=object)])
    try:
        uniq, inv = np.unique(arr, return_inverse=True)
        table = list(uniq)
    except TypeError:  # unorderable keys: first-seen order
        index = {}
        inv = np.empty(len(arr), dtype=np.int64)
        for i, k in enumerate(arr.tolist()):
            inv[i] = index.setdefault(k, len(index))
        table = list(index)
    n = len(values)
    ids = torch.from_numpy(np.ascontiguousarray(inv[:n].astype(np.int64))).to(device)
    return ids, table, (None if extra is None else inv[n:])


def _public_id_tensor(public_partitions, device) -> Optional[torch.Tensor]:
    """Integer public partitions given as a range, ndarray or tensor, as a
    device int64 tensor (None for other containers, which are listed)."""
    if isinstance(public_partitions, range):
        r = public_partitions
        return torch.arange(r.start, r.stop, r.step, dtype=torch.int64, device=device)
    if isinstance(public_partitions, (torch.Tensor, np.ndarray)) and _integer_like(public_partitions):
        return _to_tensor(public_partitions, device).to(torch.int64).reshape(-1)
    return None


def _check_public_range(lo: int, hi: int, P: int) -> None:
    if lo < 0 or hi >= P:
        raise ValueError(
            f"public partition id {lo if lo < 0 else hi} is outside [0, n_partitions={P}): with "
            f"ColumnarData(n_partitions=P) every partition key, public ones included, must be a "
            f"dense id in [0, P)")


def _device_bitmap(ids: torch.Tensor, P: int, device) -> Tuple[torch.Tensor, int]:
    """Bitmap of P bits (bit i of byte i >> 3 = partition i public) built on
    the device, and the number of distinct ids (all must lie in [0, P))."""
    if ids.numel():
        _check_public_range(*_range(ids), P)
    flags = torch.zeros(((P + 7) // 8) * 8, dtype=torch.uint8, device=device)
    flags[ids] = 1
    count = int(flags.sum(dtype=torch.int64).item())
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=device)
    mask = (flags.view(-1, 8) * w).sum(1, dtype=torch.uint8)
    return mask.contiguous(), count


def _range_bitmap(lo: int, hi: int, P: int, device) -> Tuple[torch.Tensor, int]:
    """The _device_bitmap of range(lo, hi) without materialising the ids
    (config 4's public_partitions = range(1e8): 800 MB of ids, a scatter
    and two reductions per release otherwise)."""
    mask = torch.zeros((P + 7) // 8, dtype=torch.uint8, device=device)
    if hi <= lo:
        return mask, 0
    _check_public_range(lo, hi - 1, P)
    b0, b1 = lo >> 3, (hi - 1) >> 3
    head = (0xFF << (lo & 7)) & 0xFF
    tail = 0xFF >> (7 - ((hi - 1) & 7))
    if b0 == b1:
        mask[b0] = head & tail
    else:
        mask[b0] = head
        mask[b0 + 1:b1] = 0xFF
        mask[b1] = tail
    return mask, hi - lo


def _range(t: torch.Tensor):
    if t.numel() == 0:
        return 0, -1
    return int(t.min().item()), int(t.max().item())


def encode(col, extractors, device: torch.device, need_values: bool,
           public_partitions=None, need_pid: bool = True) -> EncodedInput:
    pid_range, rec_off = None, 0
    if _is_columnar(col):
        pid = _extract(col, extractors.privacy_id_extractor) if need_pid else None
        pk = _extract(col, extractors.partition_extractor)
        value = _extract(col, extractors.value_extractor) if need_values else None
        hint = col.n_partitions if isinstance(col, ColumnarData) else col.get("n_partitions")
        if isinstance(col, ColumnarData):
            pid_range, rec_off = col.privacy_id_range, int(col.record_id_offset)
    else:
        rows = col if isinstance(col, list) else list(col)
        ex = extractors
        pid = [ex.privacy_id_extractor(r) for r in rows] if need_pid else None
        pk = [ex.partition_extractor(r) for r in rows]
        value = ([ex.value_extractor(r) for r in rows]
                 if need_values and ex.value_extractor is not None else None)
        hint = None
    if pk is None:
        raise ValueError("partition_extractor must be set")
    n = len(pk)
    if need_values and value is None:
        raise ValueError("value_extractor must be set for SUM, MEAN and VARIANCE")

    # ---- partition keys -> dense ids
    # dense integer keys with a declared P and array-like public partitions:
    # the public bitmap is built on the device (config 4: 1e8 public ids)
    pub_dense = None
    pub_range = None  # a unit-step range: its bitmap is two partial bytes and a fill
    if public_partitions is not None and hint is not None and _integer_like(pk):
        if isinstance(public_partitions, range) and public_partitions.step == 1:
            pub_range = (public_partitions.start, public_partitions.stop)
        else:
            pub_dense = _public_id_tensor(public_partitions, device)
    public_list = (None if public_partitions is None or pub_dense is not None
                   or pub_range is not None else list(public_partitions))
    key_table = None
    pk_ids = None
    public_ids = None
    # rows whose partition keys are numpy scalars keep those objects as the
    # key table: results and the utility analysis' partition sampler then see
    # the user's own keys (repr np.int64(5), as the reference's rows print).
    # Only without an n_partitions hint: with one, the keys are the caller's
    # dense ids, and the public bitmap above (pub_range / pub_dense) was
    # built over those ids, so they must not be re-encoded
    np_row_keys = (hint is None and isinstance(pk, list)
                   and any(isinstance(k, np.generic) for k in pk))
    if _integer_like(pk) and not np_row_keys:
        pk_t = _to_tensor(pk, device).to(torch.int64)
        if hint is not None:
            P = int(hint)
            pk_ids = pk_t
            if public_list is not None:
                public_ids = np.asarray(public_list, dtype=np.int64)
        else:
            lo, hi = _range(pk_t)
            pub_arr = None
            if public_list is not None:
                try:
                    pub_arr = np.asarray(public_list, dtype=np.int64)
                except (TypeError, ValueError, OverflowError):
                    pub_arr = None
                if pub_arr is not None and pub_arr.size:
                    lo, hi = min(lo, int(pub_arr.min())), max(hi, int(pub_arr.max()))
            dense_ok = lo >= 0 and hi + 1 <= max(1 << 20, 4 * max(n, 1)) and (
                public_list is None or pub_arr is not None)
            if dense_ok:
                pk_ids, P = pk_t, max(hi + 1, 1)
                public_ids = pub_arr
            else:
                pk_ids, key_table, public_ids = _encode_keys(pk_t, device, public_list)
                P = max(len(key_table), 1)
    else:
        pk_ids, key_table, public_ids = _encode_keys(pk, device, public_list)
        P = max(len(key_table), 1)

    # ---- privacy ids -> integers spanning <= 2^32 values, with their range
    # when known (else the device reduces it)
    pid_ids = None
    pid_min, pid_count = 0, 0
    if need_pid:
        if pid is None:
            raise ValueError("privacy_id_extractor must be set")
        if _integer_like(pid):
            pid_t = _to_tensor(pid, device).to(torch.int64)
            if pid_range is not None:
                lo, hi = int(pid_range[0]), int(pid_range[1])
                if not 0 < hi - lo <= _PID_SPAN:
                    raise ValueError("privacy_id_range must be (lo, hi) with 0 < hi - lo <= 2^32")
                pid_min, pid_count = lo, hi - lo
            elif hint is None and n > 0:
                lo, hi = _range(pid_t)
                if hi - lo >= _PID_SPAN:
                    pid_t, uniq, _ = _encode_keys(pid_t, device)
                    pid_min, pid_count = 0, max(1, len(uniq))
                else:
                    pid_min, pid_count = lo, hi - lo + 1
            pid_ids = pid_t
        else:
            pid_ids, table, _ = _encode_keys(pid, device)
            pid_min, pid_count = 0, max(1, len(table))

    val = None
    if need_values:
        val = _to_tensor(value, device).to(torch.float64)

    enc = EncodedInput(pid=pid_ids, pk=pk_ids.contiguous(), value=val, n=n,
                       n_partitions=int(P), key_table=key_table, pid_min=pid_min,
                       pid_count=pid_count, rec_id_offset=rec_off,
                       partitions_declared=hint is not None and key_table is None)
    if pub_range is not None:
        enc.public_mask, enc.public_count = _range_bitmap(*pub_range, int(P), device)
    elif pub_dense is not None:
        enc.public_mask, enc.public_count = _device_bitmap(pub_dense, int(P), device)
    elif public_ids is not None:
        mask = np.zeros((P + 7) // 8, dtype=np.uint8)
        ids = np.unique(np.asarray(public_ids, dtype=np.int64))
        if ids.size and key_table is None:
            _check_public_range(int(ids[0]), int(ids[-1]), P)
        np.bitwise_or.at(mask, ids >> 3, (1 << (ids & 7)).astype(np.uint8))
        enc.public_mask = torch.from_numpy(mask).to(device)
        enc.public_count = int(ids.size)
    if enc.pid is not None:
        enc.pid = enc.pid.contiguous()
    return enc


def decode_keys(ids: np.ndarray, key_table) -> list:
    """Dense ids -> the user's keys, as Python objects: a numpy key table
    (integer tensor / array columns) yields Python scalars, so a key prints
    and hashes as the reference's row keys do (e.g. repr 5, not
    np.int64(5), which the utility analysis' partition sampler hashes)."""
    if key_table is None:
        return ids.tolist()
    if isinstance(key_table, np.ndarray):
        return key_table[ids].tolist()
    return [key_table[i] for i in ids.tolist()]
