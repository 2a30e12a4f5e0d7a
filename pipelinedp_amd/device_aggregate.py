"""Lazy device execution of one DPEngine.aggregate / select_partitions call.

The reference returns a lazy collection whose generators run when the user
iterates it, after `BudgetAccountant.compute_budgets()` (SURVEY.md 3.4;
pinned by the reference's tests/pipeline_backend_test.py:564-591).  This
object keeps that contract: nothing touches the GPU until the first
`__iter__` / `materialize()`, and budgets are read at that moment.

Device pipeline per call (include/dpg.h):
  dpg_bound_aggregate -> [multi-GPU: reduce-scatter of the dense partials,
  or a fixed-block all-to-all of the occupied ones, with every rank's error
  flag: distributed.exchange_partials] -> dpg_select_and_noise ->
  dpg_compact_kept_async.  The kept count reaches the host when the result's
  ids or values are first read (the one host synchronisation after the
  bounding), so a caller can enqueue the next release first.
"""
import ctypes
import os
import warnings
from typing import Optional, Sequence

import numpy as np
import torch

from pipelinedp_amd import _native
from pipelinedp_amd import columnar
from pipelinedp_amd import combiners
from pipelinedp_amd import distributed
from pipelinedp_amd import partition_selection


# experiments: DPG_SYNC_COMPACT=1 synchronises at the compaction, as before
# round 5 (same-box A/B of the asynchronous result)
_SYNC_COMPACT = os.environ.get("DPG_SYNC_COMPACT", "0") == "1"


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


# Results dropped before their device info word was read: their
# bounding error bits are checked when the release has finished, at the
# latest by the next release on any backend, and reported as a warning.
_DROPPED = []


def check_dropped(block: bool = False) -> None:
    """Warns about dropped, never-read results whose bounding latched an
    internal error; block=True waits for the unfinished ones."""
    keep = []
    for info, ev in _DROPPED:
        if ev is not None and not block and not ev.query():
            keep.append((info, ev))
            continue
        if ev is not None:
            ev.synchronize()
        if int(info[1].item()) & 2:
            warnings.warn("a DeviceResult dropped without being read had an internal bounding "
                          "error (hash-table overflow); its release was invalid", RuntimeWarning)
    _DROPPED[:] = keep


class DeviceResult:
    """Materialised result: kept partition ids (int64 [K], global dense ids)
    and their metric columns (float64 [K, len(fields)]), on the device.
    `keys()` maps ids back to the user's partition keys.

    Built from the compaction's full-size outputs and its device info word
    (kept count, bounding error bits): the count is read -- and an internal
    bounding error raised -- when `partition_ids` or `values` is first used."""

    def __init__(self, partition_ids: torch.Tensor, values: torch.Tensor, fields: tuple,
                 key_table: Optional[Sequence], stage_ms: Optional[dict] = None,
                 pending: Optional[tuple] = None):
        self._ids, self._vals = partition_ids, values
        self.fields = fields
        self.key_table = key_table
        self.stage_ms = stage_ms if stage_ms is not None else {}
        # (info int64[2] on the device, outputs per row, id stride, id offset
        # [, event recorded behind the compaction on the release's stream])
        self._pending = pending

    def _resolve(self):
        if self._pending is None:
            return
        info, n_out, stride, offset = self._pending[:4]
        if len(self._pending) > 4 and self._pending[4] is not None:
            # the release ran on the stream current at materialize(); the
            # reader's current stream may be another one
            self._pending[4].synchronize()
        k, err = (int(x) for x in info.tolist())
        if err & 2:
            self._pending = None  # reported here, not again when dropped
            raise _native.NativeError(
                "dpg_compact_kept failed (HIP error): internal hash-table error in bounding")
        ids = self._ids[:k]
        if stride != 1 or offset:  # several ranks: this rank's slice
            ids = ids * stride + offset
        vals = (self._vals[:k * n_out].view(k, n_out) if n_out
                else torch.empty((k, 0), dtype=torch.float64, device=self._vals.device))
        # a small kept set does not pin the partition-sized compaction
        # buffers: compact copies
        if 2 * k < self._ids.numel():
            ids = ids.clone() if ids.data_ptr() == self._ids.data_ptr() else ids
            vals = vals.clone()
        self._ids, self._vals = ids, vals
        self._pending = None

    def __del__(self):
        p = getattr(self, "_pending", None)
        if p is not None:
            _DROPPED.append((p[0], p[4] if len(p) > 4 else None))

    @property
    def partition_ids(self) -> torch.Tensor:
        self._resolve()
        return self._ids

    @property
    def values(self) -> torch.Tensor:
        self._resolve()
        return self._vals

    def keys(self) -> list:
        return columnar.decode_keys(self.partition_ids.cpu().numpy(), self.key_table)


class DeviceAggregation:
    """Lazy collection of (partition_key, MetricsTuple) -- or of partition
    keys for select_partitions."""

    def __init__(self, backend, col, extractors, plan: Optional[combiners.CompoundPlan],
                 public_partitions=None, selection_spec=None, strategy=None,
                 max_partitions_contributed: int = 1, pre_threshold=None,
                 max_rows_per_privacy_id: int = 1, drop_non_public: bool = True,
                 bounds_already_enforced: bool = False, keys_only: bool = False):
        self.backend = backend
        self.col = col
        self.extractors = extractors
        self.plan = plan
        self.public_partitions = public_partitions
        self.selection_spec = selection_spec
        self.strategy = strategy
        self.max_partitions_contributed = max_partitions_contributed
        self.pre_threshold = pre_threshold
        self.max_rows = max_rows_per_privacy_id
        self.drop_non_public = drop_non_public
        self.bounds_already_enforced = bounds_already_enforced
        self.keys_only = keys_only
        self._result: Optional[DeviceResult] = None
        self.last_partials = None
        self.noise_enabled = True
        # Per-release nonce of every keyed random stream (include/dpg.h
        # dpg_stream_seed).  None: drawn from os.urandom when the release is
        # materialised, so two releases on one backend draw independent
        # sampling, selection and noise, like the reference's fresh PyDP /
        # numpy randomness per call (dp_computations.py:131-133, 151-152;
        # pipeline_backend.py:540-544).  Tests inject it to reproduce a
        # release; multi-GPU releases broadcast rank 0's.
        self.nonce: Optional[int] = None
        self.last_bound_fields: Optional[dict] = None
        self.last_exchange: Optional[dict] = None
        self.last_select_fields: Optional[dict] = None

    # ------------------------------------------------------------ public
    def __iter__(self):
        res = self.materialize()
        keys = res.keys()
        if self.keys_only:
            return iter(keys)
        vals = res.values.cpu().numpy()
        T = self.plan.MetricsTuple
        return iter([(k, T(*map(float, row))) for k, row in zip(keys, vals)])

    def materialize(self, gather: bool = True) -> DeviceResult:
        if self._result is None:
            self._result = self._run(gather)
        return self._result

    # ------------------------------------------------------------ device
    def _bound_fields(self, P: int) -> dict:
        if self.plan is not None:
            f = self.plan.bound_fields(P)
        else:  # select_partitions: cross-partition bounding, keys only
            f = dict(mode=combiners.MODE_CROSS, sum_mode=combiners.SUM_NONE, metric_mask=0,
                     max_partitions_contributed=self.max_partitions_contributed,
                     max_contributions_per_partition=1, max_contributions=0,
                     min_value=0.0, max_value=0.0, min_sum_per_partition=0.0,
                     max_sum_per_partition=0.0, n_partitions=P)
        if self.bounds_already_enforced:
            # every row is its own privacy unit: bounding never samples
            f.update(mode=combiners.MODE_CROSS_AND_PER if f["mode"] != combiners.MODE_CROSS
                     else combiners.MODE_CROSS,
                     max_partitions_contributed=max(1, f["max_partitions_contributed"]),
                     max_contributions_per_partition=max(1, f["max_contributions_per_partition"]))
            if f["mode"] == combiners.MODE_PER_PID:
                f["mode"] = combiners.MODE_CROSS_AND_PER
        return f

    def _select_fields(self, pk_offset: int, public_mask_local, pk_stride: int = 1) -> dict:
        nonce = self.nonce or 0
        if self.public_partitions is not None:
            return dict(strategy=0, table_len=0, keep_table=None, threshold=0.0,
                        noise_scale=0.0, pre_threshold=0, max_rows_per_privacy_id=1,
                        pk_offset=pk_offset, pk_stride=pk_stride, public_mask=public_mask_local,
                        nonce=nonce)
        spec = self.selection_spec
        sp = partition_selection.create_partition_selection_strategy(
            self.strategy, spec.eps, spec.delta, self.max_partitions_contributed,
            self.pre_threshold)
        self._selection_plan = sp
        f = dict(strategy=sp.native_strategy, table_len=0, keep_table=None,
                 threshold=sp.threshold, noise_scale=sp.noise_scale,
                 pre_threshold=int(self.pre_threshold or 0),
                 max_rows_per_privacy_id=int(self.max_rows), pk_offset=pk_offset,
                 pk_stride=pk_stride, public_mask=None, nonce=nonce)
        if sp.table is not None:
            self._table = np.ascontiguousarray(np.asarray(sp.table, dtype=np.float64))
            f["table_len"] = len(self._table)
            f["keep_table"] = self._table.ctypes.data
        return f

    def _release_header(self, nnz_bound: int):
        """The release nonce (rank 0's) and, with several ranks, the
        occupancy bound maximised over ranks: one collective, before any
        device work of the release."""
        if self.nonce is None:
            self.nonce = int.from_bytes(os.urandom(8), "little")
        if self.backend.world_size > 1:
            self.nonce, nnz_bound = distributed.release_header(
                self.nonce, nnz_bound, self.backend.process_group, self.backend.device)
        return self.nonce, nnz_bound

    def _run(self, gather: bool) -> DeviceResult:
        if _DROPPED:
            check_dropped()
        backend = self.backend
        ctx = backend.ctx
        dev = backend.device
        need_values = self.plan is not None and self.plan.needs_values()
        enc = columnar.encode(self.col, self.extractors, dev, need_values,
                              self.public_partitions,
                              need_pid=not self.bounds_already_enforced)
        if self.bounds_already_enforced:
            enc.pid = torch.arange(enc.n, dtype=torch.int64, device=dev)
            enc.pid_min, enc.pid_count = 0, max(1, enc.n)
        # noise / selection parameters are resolved now (after compute_budgets)
        noise = (self.plan.noise_fields(self.noise_enabled) if self.plan is not None else
                 dict(noise_kind=0, family=0, slot_mask=0, n_outputs=0, out_src=[0] * 8,
                      scale=[0.0] * 4, mid=0.0, mean_const=0, msq_const=0,
                      mean_const_value=0.0, msq_const_value=0.0))
        P = enc.n_partitions
        if backend.world_size > 1 and not enc.partitions_declared:
            # every rank must use the same dense partition ids and P, or the
            # exchange sums partials of different keys (or hangs)
            raise ValueError(
                "multi-GPU aggregation needs globally dense integer partition ids: "
                "pass ColumnarData(..., n_partitions=P) with pk in [0, P) on every rank")
        bfields = self._bound_fields(P)
        l0 = (bfields["max_contributions"] if bfields["mode"] == combiners.MODE_PER_PID
              else bfields["max_partitions_contributed"])
        nonce, nnz_bound = self._release_header(distributed.occupancy_bound(
            P, enc.n, enc.pid_count, int(l0)))
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            sptr = ctypes.c_void_p(stream.cuda_stream)
            f64 = dict(dtype=torch.float64, device=dev)
            rows = torch.empty(P, dtype=torch.int64, device=dev)
            count = torch.empty(P, dtype=torch.int64, device=dev)
            mask = self.plan.mask if self.plan is not None else 0
            sum_ = torch.empty(P, **f64) if mask & combiners.M_SUM else None
            var = mask & (combiners.M_MEAN | combiners.M_VARIANCE)
            nsum = torch.empty(P, **f64) if var else None
            nsq = torch.empty(P, **f64) if var else None
            bound = _native.fill(_native.BoundParams, bfields)
            bound.pid_min, bound.pid_count = enc.pid_min, enc.pid_count
            bound.rec_id_offset = enc.rec_id_offset
            bound.nonce = nonce
            self.last_bound_fields = dict(bfields, pid_min=enc.pid_min, pid_count=enc.pid_count,
                                          rec_id_offset=enc.rec_id_offset, nonce=nonce)
            # _drop_partitions (dp_engine.py:280-286) in the level-1 pass; a
            # public set that covers every partition id drops nothing, so
            # the per-record bitmap lookups are skipped
            if (enc.public_mask is not None and self.drop_non_public
                    and enc.public_count < enc.n_partitions):
                bound.public_mask = enc.public_mask.data_ptr()
            partials = _native.Partials(P, rows.data_ptr(), count.data_ptr(),
                                        sum_.data_ptr() if sum_ is not None else None,
                                        nsum.data_ptr() if nsum is not None else None,
                                        nsq.data_ptr() if nsq is not None else None)
            ctx.bound_aggregate(_ptr(enc.pid), _ptr(enc.pk),
                                _ptr(enc.value) if need_values else None,
                                enc.n, bound, partials, sptr)
            stage_ms = {}
            tensors = dict(rows=rows, count=count, sum=sum_, nsum=nsum, nsq=nsq)
            self.last_partials = tensors
            pk_offset, pk_stride, local_P = 0, 1, P
            public_mask_local = enc.public_mask
            self.last_exchange = None
            if backend.world_size > 1:
                err = torch.empty(1, **f64)
                ctx.export_error(err.data_ptr(), sptr)
                tensors, (pk_offset, pk_stride, local_P), self.last_exchange, flags = \
                    distributed.exchange_partials(tensors, P, backend.process_group,
                                                  backend.exchange, nnz_bound, err, ctx, sptr)
                # any rank's bounding error fails this rank's compaction
                flags = flags.to(dev).contiguous()
                ctx.import_error(flags.data_ptr(), flags.numel(), sptr)
                if public_mask_local is not None:
                    public_mask_local = distributed.slice_bitmap(
                        enc.public_mask, pk_offset, pk_stride, local_P)
            # this rank's merged partitions pk_offset + i * pk_stride, i < local_P
            self.last_slice = (tensors, pk_offset, pk_stride, local_P)
            lp = _native.Partials(local_P, tensors["rows"].data_ptr(),
                                  tensors["count"].data_ptr(),
                                  *(tensors[k].data_ptr() if tensors[k] is not None else None
                                    for k in ("sum", "nsum", "nsq")))
            sfields = self._select_fields(
                pk_offset, public_mask_local.data_ptr() if public_mask_local is not None else None,
                pk_stride)
            self.last_select_fields = sfields
            sel = _native.fill(_native.SelectParams, sfields)
            nz = _native.fill(_native.NoiseParams, noise)
            n_out = noise["n_outputs"]
            keep = torch.empty(local_P, dtype=torch.uint8, device=dev)
            out = torch.empty(max(local_P * n_out, 1), **f64)
            ctx.select_and_noise(lp, sel, nz, keep.data_ptr(), out.data_ptr(), sptr)
            ids = torch.empty(local_P, dtype=torch.int64, device=dev)
            kept_out = torch.empty(max(local_P * n_out, 1), **f64)
            fields = self.plan.fields if self.plan is not None else ()
            if _SYNC_COMPACT:  # A/B switch: the synchronising compaction
                k = ctx.compact(keep.data_ptr(), out.data_ptr(), local_P, n_out,
                                ids.data_ptr(), kept_out.data_ptr(), sptr)
                info = torch.tensor([k, 0], dtype=torch.int64, device=dev)
            else:
                info = torch.empty(2, dtype=torch.int64, device=dev)
                ctx.compact_async(keep.data_ptr(), out.data_ptr(), local_P, n_out,
                                  ids.data_ptr(), kept_out.data_ptr(), info.data_ptr(), sptr)
            done = torch.cuda.Event()
            done.record(stream)
            res = DeviceResult(ids, kept_out, fields, enc.key_table, stage_ms,
                               pending=(info, n_out, pk_stride, pk_offset, done))
            if backend.world_size > 1 and gather:
                ids, vals = distributed.all_gather_results(res.partition_ids, res.values,
                                                           backend.process_group)
                res = DeviceResult(ids, vals, fields, enc.key_table, stage_ms)
        return res
