"""Host-side key handling: distinct-partition counts and key decoding must
treat tensor / numpy keys by value, as the reference's hashable row keys
are (private_contribution_bounds.py:93 len(set(partitions));
sampling_utils.py:32-51 ValueSampler hashes repr(key))."""
import hashlib

import numpy as np
import pytest
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


def _ref_keep(v, rate):
    """The reference ValueSampler (sampling_utils.py:30-51), restated."""
    return int(hashlib.sha1(repr(v).encode()).hexdigest()[:16], 16) < int(round(2**64 * rate))


def test_decoded_keys_are_python_scalars_and_sample_like_row_keys():
    table = np.array([5, 9, 11], dtype=np.int64)
    keys = columnar.decode_keys(np.array([2, 0]), table)
    assert keys == [11, 5] and all(type(k) is int for k in keys)
    assert repr(keys[1]) == "5"
    for rate in (0.3, 0.7):
        bound = ua._sample_bound(rate)
        for k in (0, 5, 123456789, "pk7", np.int64(5), np.int32(123456789)):
            # keys are hashed exactly as given, like the reference's row keys
            assert ua._keep_by_hash(k, bound) == _ref_keep(k, rate)
    # object key tables (strings) pass through unchanged
    assert columnar.decode_keys(np.array([1]), ["a", "b"]) == ["b"]


def test_numpy_scalar_row_keys_come_back_as_given():
    """rows whose partition keys are numpy scalars keep those
    objects, so the partition sampler hashes repr(np.int64(5)) as the
    reference does and the results carry the user's key objects."""
    rows = [(1, np.int64(5), 1.0), (2, np.int64(9), 2.0), (3, np.int64(5), 3.0)]
    ex = type("Ex", (), dict(privacy_id_extractor=staticmethod(lambda r: r[0]),
                             partition_extractor=staticmethod(lambda r: r[1]),
                             value_extractor=staticmethod(lambda r: r[2])))
    enc = columnar.encode(rows, ex, torch.device("cpu"), True)
    keys = columnar.decode_keys(np.arange(enc.n_partitions), enc.key_table)
    assert keys == [np.int64(5), np.int64(9)] and all(type(k) is np.int64 for k in keys)
    assert [repr(k) for k in keys] == [repr(np.int64(5)), repr(np.int64(9))]
    # plain Python integer rows stay dense ids decoded as Python ints
    enc2 = columnar.encode([(1, 5, 1.0), (2, 9, 2.0)], ex, torch.device("cpu"), True)
    assert enc2.key_table is None


@pytest.mark.parametrize("lo,hi,P", [(0, 100, 100), (3, 4, 10), (5, 13, 20), (8, 16, 16),
                                     (0, 0, 9), (7, 9, 9), (1, 1000, 1003), (16, 17, 40)])
def test_range_bitmap_matches_ids_bitmap(lo, hi, P):
    """public_partitions = range(lo, hi) builds its bitmap without listing
    the ids; it must equal the bitmap of the listed ids bit for bit."""
    from pipelinedp_amd import columnar
    dev = torch.device("cpu")
    got, n = columnar._range_bitmap(lo, hi, P, dev)
    want, m = columnar._device_bitmap(torch.arange(lo, hi, dtype=torch.int64), P, dev)
    assert n == m == max(0, hi - lo)
    assert torch.equal(got, want)


def test_range_bitmap_rejects_out_of_range():
    from pipelinedp_amd import columnar
    with pytest.raises(ValueError, match="outside"):
        columnar._range_bitmap(0, 11, 10, torch.device("cpu"))


def test_preaggregated_rows_reject_n_contributions_past_31_bits():
    # the pair word shares its top bit with the leader flag; a
    # larger n_contributions must raise, not be clamped into wrong L0/L1 bins
    from pipelinedp_amd import pre_aggregation as pa
    import pipelinedp_amd as pdp
    ex = pdp.PreAggregateExtractors(partition_extractor=lambda r: r[0],
                                    preaggregate_extractor=lambda r: r[1])
    ok = pa.host_preaggregated_pairs([("a", (1, 2.0, 1, pa.NC_MASK))], ex, None,
                                     torch.device("cpu"))
    assert int(pa.to_numpy(ok)["ncl"][0]) == pa.NC_MASK
    for bad in (pa.NC_MASK + 1, 2**40, -1):
        with pytest.raises(ValueError, match="n_contributions"):
            pa.host_preaggregated_pairs([("a", (1, 2.0, 1, bad))], ex, None, torch.device("cpu"))
