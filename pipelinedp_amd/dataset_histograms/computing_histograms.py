"""Dataset contribution histograms on MI355X (API mirror of
pipeline_dp/dataset_histograms/computing_histograms.py).

compute_dataset_histograms (:420-474) builds six histograms from the rows:
L0 / L1 contributions per privacy id, LINF records and LINF_SUM value sum
per (privacy id, partition) pair, and records / privacy ids per partition.
The reference runs a dozen backend group-bys over the rows.  Here it is two
C-ABI calls: dpg_preaggregate (one 24-byte entry per pair, one pair per
privacy id marked as its leader) and dpg_dataset_histograms (csrc/
dpg_hist.h: streaming passes over the pairs and the partitions into
LDS-privatised bins).  The host only turns the few thousand non-empty bins
into FrequencyBin objects.

compute_dataset_histograms_on_preaggregated_data (:642-684) takes
PreAggregateExtractors rows instead; L0 / L1 are then weighted by
1 / n_partitions per exact value and rounded (:81-102, 482-529).
"""
import ctypes
from typing import List

import numpy as np
import torch

from pipelinedp_amd import _native
from pipelinedp_amd import data_extractors as dex
from pipelinedp_amd import pipeline_backend
from pipelinedp_amd import pre_aggregation
from pipelinedp_amd.dataset_histograms import histograms as hist

NUMBER_OF_BUCKETS_IN_LINF_SUM_CONTRIBUTIONS_HISTOGRAM = _native.HIST_SUM_BINS

# order of the integer histograms in dpg_hist_out.int_bins (DPG_HIST_*)
_INT_TYPES = (hist.HistogramType.L0_CONTRIBUTIONS, hist.HistogramType.L1_CONTRIBUTIONS,
              hist.HistogramType.LINF_CONTRIBUTIONS, hist.HistogramType.COUNT_PER_PARTITION,
              hist.HistogramType.COUNT_PRIVACY_ID_PER_PARTITION)


def _to_bin_lower_upper_logarithmic(value: int):
    """Bin of an integer: 3 significant digits (computing_histograms.py
    :28-47; private_contribution_bounds.generate_possible_contribution_bounds
    enumerates the same lowers)."""
    bound = 1000
    while value > bound:
        bound *= 10
    base = bound // 1000
    lower = value // base * base
    return lower, lower + (base if value != bound else base * 10)


def int_bin_bounds(idx):
    """(lower, upper) lists of the dense integer bin indices of dpg_hist.h
    (Python ints: the top bins exceed int64)."""
    lower, upper = [], []
    for i in np.asarray(idx, dtype=np.int64).tolist():
        if i < 1000:
            lower.append(i)
            upper.append(i + 1)
        else:
            e, m = divmod(i - 1000, 900)
            p = 10 ** (e + 1)
            lower.append((100 + m) * p)
            upper.append((101 + m) * p)
    return lower, upper


def _int_histogram(name, b: np.ndarray) -> hist.Histogram:
    """b: uint64[bins][3] (count, sum, max) -> Histogram of existing bins."""
    idx = np.nonzero((b[:, 0] > 0) | (b[:, 2] > 0))[0]
    lower, upper = int_bin_bounds(idx)
    bins = [hist.FrequencyBin(lower=int(lo), upper=int(up), count=int(c), sum=int(s), max=int(m))
            for lo, up, (c, s, m) in zip(lower, upper, b[idx].tolist())]
    return hist.Histogram(name, bins)


def _float_histogram(count, sums, maxes, lowers) -> hist.Histogram:
    idx = np.nonzero(count > 0)[0]
    bins = [hist.FrequencyBin(lower=float(lowers[i]), upper=float(lowers[i + 1]),
                              count=int(count[i]), sum=float(sums[i]), max=float(maxes[i]))
            for i in idx]
    return hist.Histogram(hist.HistogramType.LINF_SUM_CONTRIBUTIONS, bins)


def histograms_from_pairs(ps: pre_aggregation.PairSet, backend,
                          pre_aggregated: bool) -> hist.DatasetHistograms:
    """dpg_dataset_histograms over a pre-aggregate, bins to the host."""
    dev = ps.pairs.device
    nb, ns = _native.HIST_INT_BINS, _native.HIST_SUM_BINS
    u64 = dict(dtype=torch.int64, device=dev)
    f64 = dict(dtype=torch.float64, device=dev)
    ib = torch.empty((len(_INT_TYPES), nb, 3), **u64)
    sc = torch.empty(ns, **u64)
    ss, sm = torch.empty(ns, **f64), torch.empty(ns, **f64)
    lowers = torch.empty(ns + 1, **f64)
    out = _native.HistOut(ib.data_ptr(), sc.data_ptr(), ss.data_ptr(), sm.data_ptr(),
                          lowers.data_ptr())
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        backend.ctx.dataset_histograms(ctypes.c_void_p(ps.pairs.data_ptr()), ps.n_pairs,
                                       ctypes.c_void_p(ps.starts.data_ptr()), ps.n_partitions,
                                       pre_aggregated, out, ctypes.c_void_p(stream.cuda_stream))
        stream.synchronize()
    ib_h = ib.cpu().numpy().view(np.uint64)
    hs = {t: _int_histogram(t, ib_h[i]) for i, t in enumerate(_INT_TYPES)}
    lin_sum = _float_histogram(sc.cpu().numpy(), ss.cpu().numpy(), sm.cpu().numpy(),
                               lowers.cpu().numpy())
    T = hist.HistogramType
    return hist.DatasetHistograms(hs[T.L0_CONTRIBUTIONS], hs[T.L1_CONTRIBUTIONS],
                                  hs[T.LINF_CONTRIBUTIONS], lin_sum,
                                  hs[T.COUNT_PER_PARTITION],
                                  hs[T.COUNT_PRIVACY_ID_PER_PARTITION])


class _OneElement:
    """Lazy 1-element collection (the reference returns one from the
    backend); computed on first iteration."""

    def __init__(self, fn):
        self._fn = fn
        self._value = None
        self._done = False

    def __iter__(self):
        if not self._done:
            self._value = self._fn()
            self._done = True
        return iter([self._value])


def _require_device_backend(backend):
    if not isinstance(backend, pipeline_backend.MI355XBackend):
        raise NotImplementedError("dataset histograms run on MI355XBackend")


def compute_dataset_histograms(col, data_extractors: dex.DataExtractors, backend):
    """1-element collection with the DatasetHistograms of the rows
    (computing_histograms.py:420-474)."""
    _require_device_backend(backend)

    def run():
        ps = pre_aggregation.device_pairs(col, data_extractors, backend, None, backend.device)
        return histograms_from_pairs(ps, backend, pre_aggregated=False)

    return _OneElement(run)


def compute_dataset_histograms_on_preaggregated_data(
        col, data_extractors: dex.PreAggregateExtractors, backend):
    """1-element collection with the DatasetHistograms of pre-aggregated rows
    (partition key, (count, sum, n_partitions, n_contributions))
    (computing_histograms.py:642-684)."""
    _require_device_backend(backend)

    def run():
        ps = pre_aggregation.host_preaggregated_pairs(col, data_extractors, None, backend.device)
        return histograms_from_pairs(ps, backend, pre_aggregated=True)

    return _OneElement(run)
