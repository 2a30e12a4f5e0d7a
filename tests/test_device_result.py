"""Host logic of the lazily resolved release (device_aggregate.DeviceResult):
the compaction leaves the kept count and the bounding's error bits in a
device word; the result slices its full-size outputs, maps a rank's local
ids to global ones and raises a latched internal error on first use.  CPU
tensors stand in for the device buffers (no GPU needed)."""
import pytest
import torch

from pipelinedp_amd import _native
from pipelinedp_amd.device_aggregate import DeviceResult


def _full(k, n_out, cap=10):
    ids = torch.arange(cap, dtype=torch.int64) * 3
    vals = torch.arange(cap * n_out, dtype=torch.float64)
    return ids, vals


def test_resolves_count_and_shapes_on_first_use():
    ids, vals = _full(4, 2)
    info = torch.tensor([4, 0], dtype=torch.int64)
    r = DeviceResult(ids, vals, ("count", "sum"), None, pending=(info, 2, 1, 0))
    assert r._pending is not None                  # nothing read yet
    assert r.partition_ids.tolist() == [0, 3, 6, 9]
    assert r.values.shape == (4, 2)
    assert r.values[1].tolist() == [2.0, 3.0]
    assert r._pending is None
    assert r.keys() == [0, 3, 6, 9]


def test_rank_slice_maps_local_ids():
    ids, vals = _full(3, 1)
    info = torch.tensor([3, 0], dtype=torch.int64)
    r = DeviceResult(ids, vals, ("count",), None, pending=(info, 1, 4, 2))
    assert r.partition_ids.tolist() == [2, 14, 26]  # local i -> 2 + 4 i


def test_no_outputs_and_empty():
    ids, vals = _full(0, 0)
    r = DeviceResult(ids, vals, (), None, pending=(torch.tensor([0, 0]), 0, 1, 0))
    assert r.partition_ids.numel() == 0 and r.values.shape == (0, 0)


def test_latched_internal_error_raises_on_first_use():
    ids, vals = _full(2, 1)
    r = DeviceResult(ids, vals, ("count",), None, pending=(torch.tensor([2, 2]), 1, 1, 0))
    with pytest.raises(_native.NativeError, match="internal"):
        r.values
    # other error bits (key range is reported by the bounding call itself)
    ok = DeviceResult(ids, vals, ("count",), None, pending=(torch.tensor([2, 1]), 1, 1, 0))
    assert ok.partition_ids.tolist() == [0, 3]


def test_resolved_result_passes_through():
    r = DeviceResult(torch.tensor([5, 7]), torch.ones(2, 1, dtype=torch.float64), ("count",), None)
    assert r.partition_ids.tolist() == [5, 7] and r.values.shape == (2, 1)
