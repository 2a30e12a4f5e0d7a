"""Host-side key handling: distinct-partition counts and key decoding must
treat tensor / numpy keys by value, as the reference's hashable row keys
are (private_contribution_bounds.py:93 len(set(partitions));
sampling_utils.py:32-51 ValueSampler hashes repr(key))."""
import numpy as np
import torch

from pipelinedp_amd import aggregate_params as agg
from pipelinedp_amd import columnar
from pipelinedp_amd import private_contribution_bounds as pcb
from pipelinedp_amd.analysis import utility_analysis as ua


def _calc(partitions):
    params = agg.CalculatePrivateContributionBoundsParams(
        aggregation_eps=1.0, aggregation_delta=1e-6, calculation_eps=0.1,
        aggregation_noise_kind=agg.NoiseKind.LAPLACE, max_partitions_contributed_upper_bound=10)
    return pcb.PrivateL0Calculator(params, partitions, None, None)


def test_distinct_partitions_by_value_for_every_container():
    keys = [3, 1, 3, 7, 1, 1]
    want = 3
    assert _calc(keys)._number_of_partitions() == want
    assert _calc(np.array(keys))._number_of_partitions() == want
    assert _calc(torch.tensor(keys))._number_of_partitions() == want
    assert _calc(range(5))._number_of_partitions() == 5
    assert _calc(iter(keys))._number_of_partitions() == want


def test_decoded_keys_are_python_scalars_and_sample_like_row_keys():
    table = np.array([5, 9, 11], dtype=np.int64)
    keys = columnar.decode_keys(np.array([2, 0]), table)
    assert keys == [11, 5] and all(type(k) is int for k in keys)
    assert repr(keys[1]) == "5"
    for bound in (ua._sample_bound(0.3), ua._sample_bound(0.7)):
        for k in (0, 5, 123456789):
            assert ua._keep_by_hash(np.int64(k), bound) == ua._keep_by_hash(k, bound)
    # object key tables (strings) pass through unchanged
    assert columnar.decode_keys(np.array([1]), ["a", "b"]) == ["b"]
