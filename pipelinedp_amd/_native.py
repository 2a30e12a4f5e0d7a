"""ctypes binding of libdpg.so (include/dpg.h).

The library is built in-tree by __graft_entry__.build() into
pipelinedp_amd/lib/libdpg.so.  There is no CPU fallback: if the library or a
GPU is missing, every device entry point raises.
"""
import ctypes
import os
import threading

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libdpg.so")

DPG_OK = 0
ERRORS = {1: "invalid argument", 2: "key out of range", 3: "HIP error",
          4: "out of device memory", 5: "unsupported"}

EXPORTED = ("dpg_ctx_create", "dpg_ctx_destroy", "dpg_last_error", "dpg_set_seed",
            "dpg_set_tuning",
            "dpg_bound_aggregate", "dpg_select_and_noise", "dpg_compact_kept",
            "dpg_compact_kept_async", "dpg_last_stage_times", "dpg_stream_seed",
            "dpg_preaggregate",
            "dpg_utility_analysis", "dpg_dataset_histograms",
            "dpg_comm_unique_id", "dpg_ctx_create_comm", "dpg_reduce_scatter_partials",
            "dpg_pack_partials", "dpg_unpack_partials", "dpg_export_error",
            "dpg_import_error")

COMM_ID_BYTES = 128  # DPG_COMM_ID_BYTES

HIST_INT_BINS = 16300  # DPG_HIST_INT_BINS
HIST_SUM_BINS = 10000  # DPG_HIST_SUM_BINS


class BoundParams(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("sum_mode", ctypes.c_int32),
                ("metric_mask", ctypes.c_uint32), ("reserved0", ctypes.c_int32),
                ("max_partitions_contributed", ctypes.c_int64),
                ("max_contributions_per_partition", ctypes.c_int64),
                ("max_contributions", ctypes.c_int64),
                ("min_value", ctypes.c_double), ("max_value", ctypes.c_double),
                ("min_sum_per_partition", ctypes.c_double),
                ("max_sum_per_partition", ctypes.c_double),
                ("n_partitions", ctypes.c_int64), ("public_mask", ctypes.c_void_p),
                ("pid_min", ctypes.c_int64), ("pid_count", ctypes.c_int64),
                ("rec_id_offset", ctypes.c_int64), ("nonce", ctypes.c_uint64)]


class Partials(ctypes.Structure):
    _fields_ = [("n_partitions", ctypes.c_int64), ("rows", ctypes.c_void_p),
                ("count", ctypes.c_void_p), ("sum", ctypes.c_void_p),
                ("nsum", ctypes.c_void_p), ("nsq", ctypes.c_void_p)]


class SelectParams(ctypes.Structure):
    _fields_ = [("strategy", ctypes.c_int32), ("table_len", ctypes.c_int32),
                ("keep_table", ctypes.c_void_p), ("threshold", ctypes.c_double),
                ("noise_scale", ctypes.c_double), ("pre_threshold", ctypes.c_int64),
                ("max_rows_per_privacy_id", ctypes.c_int64),
                ("pk_offset", ctypes.c_int64), ("public_mask", ctypes.c_void_p),
                ("nonce", ctypes.c_uint64), ("pk_stride", ctypes.c_int64)]


class NoiseParams(ctypes.Structure):
    _fields_ = [("noise_kind", ctypes.c_int32), ("family", ctypes.c_int32),
                ("slot_mask", ctypes.c_uint32), ("n_outputs", ctypes.c_int32),
                ("out_src", ctypes.c_int32 * 8), ("scale", ctypes.c_double * 4),
                ("mid", ctypes.c_double), ("mean_const", ctypes.c_int32),
                ("msq_const", ctypes.c_int32), ("mean_const_value", ctypes.c_double),
                ("msq_const_value", ctypes.c_double)]


class PairEntry(ctypes.Structure):
    """dpg_pair_entry: one (privacy id, partition) pair of the pre-aggregate."""
    _fields_ = [("pk", ctypes.c_uint32), ("count", ctypes.c_uint32), ("sum", ctypes.c_double),
                ("n_partitions", ctypes.c_uint32),
                ("contributions_leader", ctypes.c_uint32)]  # n_contributions | leader << 31


class HistOut(ctypes.Structure):
    """dpg_hist_out: device outputs of dpg_dataset_histograms."""
    _fields_ = [("int_bins", ctypes.c_void_p), ("sum_count", ctypes.c_void_p),
                ("sum_sum", ctypes.c_void_p), ("sum_max", ctypes.c_void_p),
                ("lowers", ctypes.c_void_p)]


class UaConfig(ctypes.Structure):
    _fields_ = [("max_partitions_contributed", ctypes.c_int64),
                ("max_contributions_per_partition", ctypes.c_int64),
                ("min_sum_per_partition", ctypes.c_double),
                ("max_sum_per_partition", ctypes.c_double),
                ("selection_strategy", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("pre_threshold", ctypes.c_int64), ("keep_table", ctypes.c_void_p),
                ("table_len", ctypes.c_int64), ("threshold", ctypes.c_double),
                ("noise_scale", ctypes.c_double), ("noise_std", ctypes.c_double * 3)]


class UaParams(ctypes.Structure):
    _fields_ = [("n_configs", ctypes.c_int32), ("metric_mask", ctypes.c_uint32),
                ("public_partitions", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("configs", ctypes.c_void_p), ("sample_mask", ctypes.c_void_p),
                ("public_mask", ctypes.c_void_p)]


def fill(struct_type, fields: dict):
    s = struct_type()
    for k, v in fields.items():
        if k in ("out_src", "scale"):
            arr = getattr(s, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(s, k, v)
    return s


_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def library_path() -> str:
    return _LIB_PATH


def load():
    """Loads libdpg.so; raises NativeError if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("DPG_LIB_PATH") or _LIB_PATH  # debug: A/B builds
        if os.environ.get("DPG_PHASE_TIMING"):
            # debug build with per-phase cycle counters (tools/gpu_phase.sh)
            path = _LIB_PATH.replace("libdpg.so", "libdpg_timing.so")
        if not os.path.exists(path):
            raise NativeError(
                f"{path} is missing: build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'`. "
                f"There is no CPU fallback for the MI355X hot path.")
        lib = ctypes.CDLL(path)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.dpg_ctx_create.argtypes = [ctypes.c_int, ctypes.c_uint64]
        lib.dpg_ctx_create.restype = vp
        lib.dpg_ctx_destroy.argtypes = [vp]
        lib.dpg_ctx_destroy.restype = None
        lib.dpg_last_error.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
        lib.dpg_last_error.restype = ctypes.c_int
        lib.dpg_set_seed.argtypes = [vp, ctypes.c_uint64]
        lib.dpg_set_seed.restype = ctypes.c_int
        lib.dpg_stream_seed.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        lib.dpg_stream_seed.restype = ctypes.c_uint64
        lib.dpg_set_tuning.argtypes = [vp, i32, i32]
        lib.dpg_set_tuning.restype = ctypes.c_int
        lib.dpg_bound_aggregate.argtypes = [vp, vp, vp, vp, i64,
                                            ctypes.POINTER(BoundParams),
                                            ctypes.POINTER(Partials), vp]
        lib.dpg_bound_aggregate.restype = ctypes.c_int
        lib.dpg_select_and_noise.argtypes = [vp, ctypes.POINTER(Partials),
                                             ctypes.POINTER(SelectParams),
                                             ctypes.POINTER(NoiseParams), vp, vp, vp]
        lib.dpg_select_and_noise.restype = ctypes.c_int
        lib.dpg_compact_kept.argtypes = [vp, vp, vp, i64, i32, vp, vp,
                                         ctypes.POINTER(ctypes.c_int64), vp]
        lib.dpg_compact_kept.restype = ctypes.c_int
        lib.dpg_compact_kept_async.argtypes = [vp, vp, vp, i64, i32, vp, vp, vp, vp]
        lib.dpg_compact_kept_async.restype = ctypes.c_int
        lib.dpg_preaggregate.argtypes = [vp, vp, vp, vp, i64, ctypes.POINTER(BoundParams), vp,
                                         i64, vp, ctypes.POINTER(ctypes.c_int64), vp]
        lib.dpg_preaggregate.restype = ctypes.c_int
        lib.dpg_utility_analysis.argtypes = [vp, vp, vp, i64, ctypes.POINTER(UaParams), vp, vp,
                                             vp, vp, ctypes.POINTER(ctypes.c_int64), vp]
        lib.dpg_utility_analysis.restype = ctypes.c_int
        lib.dpg_dataset_histograms.argtypes = [vp, vp, i64, vp, i64, i32,
                                               ctypes.POINTER(HistOut), vp]
        lib.dpg_dataset_histograms.restype = ctypes.c_int
        lib.dpg_last_stage_times.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_double), i32,
                                             ctypes.POINTER(ctypes.c_int32)]
        lib.dpg_last_stage_times.restype = ctypes.c_int
        lib.dpg_comm_unique_id.argtypes = [ctypes.c_char_p]
        lib.dpg_comm_unique_id.restype = ctypes.c_int
        lib.dpg_ctx_create_comm.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        lib.dpg_ctx_create_comm.restype = ctypes.c_int
        lib.dpg_reduce_scatter_partials.argtypes = [vp, ctypes.POINTER(Partials),
                                                    ctypes.POINTER(Partials),
                                                    ctypes.POINTER(ctypes.c_int64),
                                                    ctypes.POINTER(ctypes.c_int64), vp]
        lib.dpg_reduce_scatter_partials.restype = ctypes.c_int
        lib.dpg_pack_partials.argtypes = [vp, ctypes.POINTER(Partials), ctypes.c_int, vp, vp]
        lib.dpg_pack_partials.restype = ctypes.c_int
        lib.dpg_unpack_partials.argtypes = [vp, vp, i64, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(Partials),
                                            ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_int64), vp]
        lib.dpg_unpack_partials.restype = ctypes.c_int
        lib.dpg_export_error.argtypes = [vp, vp, vp]
        lib.dpg_export_error.restype = ctypes.c_int
        lib.dpg_import_error.argtypes = [vp, vp, i64, vp]
        lib.dpg_import_error.restype = ctypes.c_int
        _lib = lib
        return lib


def stream_seed(seed: int, nonce: int) -> int:
    """dpg_stream_seed: the key of every random stream of one release."""
    return int(load().dpg_stream_seed(ctypes.c_uint64(seed & (2**64 - 1)),
                                      ctypes.c_uint64(nonce & (2**64 - 1))))


class Context:
    """Owns one dpg_ctx (one device, one seed)."""

    def __init__(self, device: int, seed: int):
        self.lib = load()
        self.device = device
        self.handle = self.lib.dpg_ctx_create(int(device), ctypes.c_uint64(seed & (2**64 - 1)))
        if not self.handle:
            raise NativeError(f"dpg_ctx_create failed on device {device}")

    def close(self):
        if self.handle:
            self.lib.dpg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, status: int, what: str):
        if status == DPG_OK:
            return
        buf = ctypes.create_string_buffer(1024)
        self.lib.dpg_last_error(self.handle, buf, 1024)
        msg = buf.value.decode(errors="replace")
        if status == 2:
            raise ValueError(f"{what}: {msg}")
        raise NativeError(f"{what} failed ({ERRORS.get(status, status)}): {msg}")

    def set_seed(self, seed: int):
        self.check(self.lib.dpg_set_seed(self.handle, ctypes.c_uint64(seed & (2**64 - 1))),
                   "dpg_set_seed")

    def set_tuning(self, bucket_target: int = 0, bucket_cap: int = 0):
        self.check(self.lib.dpg_set_tuning(self.handle, int(bucket_target), int(bucket_cap)),
                   "dpg_set_tuning")

    def bound_aggregate(self, pid_ptr, pk_ptr, value_ptr, n, bound: BoundParams,
                        partials: Partials, stream):
        st = self.lib.dpg_bound_aggregate(self.handle, pid_ptr, pk_ptr, value_ptr, n,
                                          ctypes.byref(bound), ctypes.byref(partials), stream)
        self.check(st, "dpg_bound_aggregate")

    def comm_unique_id(self) -> bytes:
        """RCCL unique id (rank 0), DPG_COMM_ID_BYTES opaque bytes."""
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        self.check(self.lib.dpg_comm_unique_id(buf), "dpg_comm_unique_id")
        return buf.raw

    def create_comm(self, uid: bytes, rank: int, nranks: int):
        self.check(self.lib.dpg_ctx_create_comm(self.handle, uid, rank, nranks),
                   "dpg_ctx_create_comm")

    def reduce_scatter_partials(self, full: Partials, slice_: Partials, stream):
        """Sums every rank's partials; this rank's slice (lo, n) lands in
        slice_ (see dpg.h)."""
        lo, n = ctypes.c_int64(0), ctypes.c_int64(0)
        st = self.lib.dpg_reduce_scatter_partials(self.handle, ctypes.byref(full),
                                                  ctypes.byref(slice_), ctypes.byref(lo),
                                                  ctypes.byref(n), stream)
        self.check(st, "dpg_reduce_scatter_partials")
        return lo.value, n.value

    def pack_partials(self, full: Partials, nranks: int, pack_ptr, stream):
        st = self.lib.dpg_pack_partials(self.handle, ctypes.byref(full), nranks, pack_ptr, stream)
        self.check(st, "dpg_pack_partials")

    def unpack_partials(self, part_ptr, n_partitions: int, nranks: int, rank: int,
                        slice_: Partials, stream):
        lo, n = ctypes.c_int64(0), ctypes.c_int64(0)
        st = self.lib.dpg_unpack_partials(self.handle, part_ptr, n_partitions, nranks, rank,
                                          ctypes.byref(slice_), ctypes.byref(lo),
                                          ctypes.byref(n), stream)
        self.check(st, "dpg_unpack_partials")
        return lo.value, n.value

    def export_error(self, dst_ptr, stream):
        """1.0 at device dst if the last bounding latched an internal error."""
        self.check(self.lib.dpg_export_error(self.handle, dst_ptr, stream), "dpg_export_error")

    def import_error(self, src_ptr, n: int, stream):
        """Latches the internal error if any of n device doubles is nonzero
        (the next compact then fails)."""
        self.check(self.lib.dpg_import_error(self.handle, src_ptr, n, stream), "dpg_import_error")

    def select_and_noise(self, partials: Partials, sel: SelectParams, noise: NoiseParams,
                         keep_ptr, out_ptr, stream):
        st = self.lib.dpg_select_and_noise(self.handle, ctypes.byref(partials),
                                           ctypes.byref(sel), ctypes.byref(noise),
                                           keep_ptr, out_ptr, stream)
        self.check(st, "dpg_select_and_noise")

    def compact(self, keep_ptr, out_ptr, n_partitions, n_out, ids_ptr, kept_out_ptr, stream) -> int:
        n = ctypes.c_int64(0)
        st = self.lib.dpg_compact_kept(self.handle, keep_ptr, out_ptr, n_partitions, n_out,
                                       ids_ptr, kept_out_ptr, ctypes.byref(n), stream)
        self.check(st, "dpg_compact_kept")
        return n.value

    def compact_async(self, keep_ptr, out_ptr, n_partitions, n_out, ids_ptr, kept_out_ptr,
                      info_ptr, stream) -> None:
        """dpg_compact_kept without the host synchronisation: the kept count
        and the bounding's error bits land in the device int64[2] at
        info_ptr in stream order."""
        st = self.lib.dpg_compact_kept_async(self.handle, keep_ptr, out_ptr, n_partitions, n_out,
                                             ids_ptr, kept_out_ptr, info_ptr, stream)
        self.check(st, "dpg_compact_kept_async")

    def preaggregate(self, pid_ptr, pk_ptr, value_ptr, n, bound: BoundParams, pairs_ptr,
                     capacity, starts_ptr, stream) -> int:
        n_pairs = ctypes.c_int64(0)
        st = self.lib.dpg_preaggregate(self.handle, pid_ptr, pk_ptr, value_ptr, n,
                                       ctypes.byref(bound), pairs_ptr, capacity, starts_ptr,
                                       ctypes.byref(n_pairs), stream)
        self.check(st, "dpg_preaggregate")
        return n_pairs.value

    def utility_analysis(self, pairs_ptr, starts_ptr, n_partitions, params: UaParams, raw_ptr,
                         err_ptr, keep_ptr, report_ptr, stream) -> int:
        n_out = ctypes.c_int64(0)
        st = self.lib.dpg_utility_analysis(self.handle, pairs_ptr, starts_ptr, n_partitions,
                                           ctypes.byref(params), raw_ptr, err_ptr, keep_ptr,
                                           report_ptr, ctypes.byref(n_out), stream)
        self.check(st, "dpg_utility_analysis")
        return n_out.value

    def dataset_histograms(self, pairs_ptr, n_pairs, starts_ptr, n_partitions,
                           pre_aggregated: bool, out: HistOut, stream):
        st = self.lib.dpg_dataset_histograms(self.handle, pairs_ptr, n_pairs, starts_ptr,
                                             n_partitions, int(bool(pre_aggregated)),
                                             ctypes.byref(out), stream)
        self.check(st, "dpg_dataset_histograms")

    def stage_times(self):
        names = ctypes.create_string_buffer(4096)
        ms = (ctypes.c_double * 64)()
        ns = ctypes.c_int32(0)
        self.check(self.lib.dpg_last_stage_times(self.handle, names, 4096, ms, 64,
                                                 ctypes.byref(ns)), "stage_times")
        keys = names.value.decode().split(",") if ns.value else []
        return dict(zip(keys, [ms[i] for i in range(ns.value)]))
