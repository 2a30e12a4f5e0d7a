"""ctypes front-end of the C oracle (oracle/dp_oracle.c).  TEST INFRASTRUCTURE.

Mirrors the C-ABI structs of include/dpg.h with its own ctypes definitions
(the oracle does not import the product).  Arrays are numpy, on the host.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DPO_LIB_PATH: an instrumented build of the same source (tests/test_asan_host.py)
_LIB = os.environ.get("DPO_LIB_PATH") or os.path.join(_HERE, "_build", "libdporacle.so")


class _Bound(ctypes.Structure):
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


class _Partials(ctypes.Structure):
    _fields_ = [("n_partitions", ctypes.c_int64), ("rows", ctypes.c_void_p),
                ("count", ctypes.c_void_p), ("sum", ctypes.c_void_p),
                ("nsum", ctypes.c_void_p), ("nsq", ctypes.c_void_p)]


class _Select(ctypes.Structure):
    _fields_ = [("strategy", ctypes.c_int32), ("table_len", ctypes.c_int32),
                ("keep_table", ctypes.c_void_p), ("threshold", ctypes.c_double),
                ("noise_scale", ctypes.c_double), ("pre_threshold", ctypes.c_int64),
                ("max_rows_per_privacy_id", ctypes.c_int64),
                ("pk_offset", ctypes.c_int64), ("public_mask", ctypes.c_void_p),
                ("nonce", ctypes.c_uint64), ("pk_stride", ctypes.c_int64)]


class _Noise(ctypes.Structure):
    _fields_ = [("noise_kind", ctypes.c_int32), ("family", ctypes.c_int32),
                ("slot_mask", ctypes.c_uint32), ("n_outputs", ctypes.c_int32),
                ("out_src", ctypes.c_int32 * 8), ("scale", ctypes.c_double * 4),
                ("mid", ctypes.c_double), ("mean_const", ctypes.c_int32),
                ("msq_const", ctypes.c_int32), ("mean_const_value", ctypes.c_double),
                ("msq_const_value", ctypes.c_double)]


def _fill(t, fields):
    s = t()
    for k, v in fields.items():
        if v is None:
            continue
        if k in ("out_src", "scale"):
            arr = getattr(s, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(s, k, v)
    return s


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        vp = ctypes.c_void_p
        L.dpo_bound_aggregate.argtypes = [ctypes.c_uint64, vp, vp, vp, ctypes.c_int64,
                                          ctypes.POINTER(_Bound), ctypes.POINTER(_Partials)]
        L.dpo_bound_aggregate.restype = ctypes.c_int
        L.dpo_bound_aggregate_ids.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int64,
                                              ctypes.POINTER(_Bound), ctypes.POINTER(_Partials)]
        L.dpo_bound_aggregate_ids.restype = ctypes.c_int
        L.dpo_select_and_noise.argtypes = [ctypes.c_uint64, ctypes.POINTER(_Partials),
                                           ctypes.POINTER(_Select), ctypes.POINTER(_Noise),
                                           vp, vp]
        L.dpo_select_and_noise.restype = ctypes.c_int
        L.dpo_stream_seed.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.dpo_stream_seed.restype = ctypes.c_uint64
        L.dpo_pair_prio.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.dpo_pair_prio.restype = ctypes.c_uint32
        L.dpo_rec_prio.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint64]
        L.dpo_rec_prio.restype = ctypes.c_uint64
        L.dpo_noise_sample.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.dpo_noise_sample.restype = ctypes.c_double
        L.dpo_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32 * 4),
                                 ctypes.POINTER(ctypes.c_uint32 * 2),
                                 ctypes.POINTER(ctypes.c_uint32 * 4)]
        L.dpo_philox.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


def bound_aggregate(pid, pk, value, fields: dict, seed: int, public_mask=None, rec_ids=None):
    """Dense partials (numpy) of the bounded aggregation.  The record sampler
    is keyed by the global record id: rec_ids[i] if given, else
    fields['rec_id_offset'] (default 0) + i."""
    pid = np.ascontiguousarray(pid, dtype=np.int64)
    rid = None if rec_ids is None else np.ascontiguousarray(rec_ids, dtype=np.int64)
    pk = np.ascontiguousarray(pk, dtype=np.int64)
    v = None if value is None else np.ascontiguousarray(value, dtype=np.float64)
    P = int(fields["n_partitions"])
    out = dict(rows=np.zeros(P, np.int64), count=np.zeros(P, np.int64),
               sum=np.zeros(P), nsum=np.zeros(P), nsq=np.zeros(P))
    b = _fill(_Bound, {k: fields[k] for k in fields if k != "public_mask"})
    pm = None
    if public_mask is not None:
        pm = np.ascontiguousarray(public_mask, dtype=np.uint8)
        b.public_mask = pm.ctypes.data
    part = _Partials(P, _p(out["rows"]), _p(out["count"]), _p(out["sum"]),
                     _p(out["nsum"]), _p(out["nsq"]))
    st = lib().dpo_bound_aggregate_ids(ctypes.c_uint64(seed), _p(pid), _p(pk), _p(v), _p(rid),
                                       len(pid), ctypes.byref(b), ctypes.byref(part))
    if st != 0:
        raise ValueError(f"oracle bound_aggregate failed with status {st}")
    return out


def select_and_noise(partials: dict, select: dict, noise: dict, seed: int,
                     keep_table=None, public_mask=None):
    P = len(partials["rows"])
    arrs = {k: np.ascontiguousarray(partials[k]) for k in ("rows", "count", "sum", "nsum", "nsq")
            if partials.get(k) is not None}
    part = _Partials(P, _p(arrs["rows"]), _p(arrs["count"]), _p(arrs.get("sum")),
                     _p(arrs.get("nsum")), _p(arrs.get("nsq")))
    s = _fill(_Select, {k: v for k, v in select.items() if k not in ("keep_table", "public_mask")})
    tab = None
    if keep_table is not None:
        tab = np.ascontiguousarray(keep_table, dtype=np.float64)
        s.keep_table = tab.ctypes.data
        s.table_len = len(tab)
    pm = None
    if public_mask is not None:
        pm = np.ascontiguousarray(public_mask, dtype=np.uint8)
        s.public_mask = pm.ctypes.data
    z = _fill(_Noise, noise)
    keep = np.zeros(P, np.uint8)
    out = np.zeros(max(P * z.n_outputs, 1))
    st = lib().dpo_select_and_noise(ctypes.c_uint64(seed), ctypes.byref(part), ctypes.byref(s),
                                    ctypes.byref(z), _p(keep), _p(out))
    if st != 0:
        raise ValueError(f"oracle select_and_noise failed with status {st}")
    return keep, out[:P * z.n_outputs].reshape(P, z.n_outputs)


def stream_seed(seed, nonce):
    return int(lib().dpo_stream_seed(ctypes.c_uint64(seed & (2**64 - 1)),
                                     ctypes.c_uint64(nonce & (2**64 - 1))))


def pair_prio(seed, pid, pk):
    return lib().dpo_pair_prio(ctypes.c_uint64(seed), pid, pk)


def rec_prio(seed, pid, pk, gidx):
    return lib().dpo_rec_prio(ctypes.c_uint64(seed), ctypes.c_uint64(pid), pk,
                              ctypes.c_uint64(gidx))


def noise_sample(kind, x, scale, seed, pk, slot):
    return lib().dpo_noise_sample(kind, x, scale, ctypes.c_uint64(seed), ctypes.c_uint64(pk), slot)


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().dpo_philox(ctypes.byref(c), ctypes.byref(k), ctypes.byref(o))
    return list(o)


def bitmap(ids, P):
    m = np.zeros((P + 7) // 8, np.uint8)
    ids = np.unique(np.asarray(ids, np.int64))
    ids = ids[(ids >= 0) & (ids < P)]
    np.bitwise_or.at(m, ids >> 3, (1 << (ids & 7)).astype(np.uint8))
    return m
