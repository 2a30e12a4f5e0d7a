"""Keep rates of the GPU partition selection (k_select_noise through
dpg_select_and_noise) against the keep probability of each strategy, over
~1.2e6 partitions per case: a chi-square test of the kept counts per
privacy-id count n against

* the truncated-geometric pi(n) table (l0 = 1, whose values the reference's
  goldens pin: tests/test_mechanisms.py, and l0 = 3);
* the Laplace-thresholding CDF  P(n + Lap(b) > T);
* the Gaussian-thresholding CDF P(n + N(0, sigma^2) > T);
* a pre-threshold (n < pre dropped, else evaluated at n - pre + 1).

The reference's selection (pipeline_dp/dp_engine.py:305-361) calls PyDP's
`should_keep(n)` per partition; its keep decision is a Bernoulli(p(n)) draw,
so the GPU's per-partition Philox uniforms must reproduce those rates.
Partitions with p(n) in {0, 1} must be dropped / kept without exception."""
import ctypes
import math

import numpy as np
import pytest
import torch
from scipy import stats

pytestmark = pytest.mark.gpu

K = 24          # privacy-id counts n = 1..K
P = K * 50_000  # partitions (>= 1e6)


def _noise_off():
    return dict(noise_kind=0, family=0, slot_mask=0, n_outputs=0, out_src=[0] * 8,
                scale=[0.0] * 4, mid=0.0, mean_const=0, msq_const=0, mean_const_value=0.0,
                msq_const_value=0.0)


def _keep_rates(strategy, eps, delta, l0, pre=0, seed=0x5E1EC7, nonce=17):
    import pipelinedp_amd as pdp
    from pipelinedp_amd import _native, partition_selection as ps
    plan = ps.create_partition_selection_strategy(strategy, eps, delta, l0, pre or None)
    backend = pdp.MI355XBackend(device=0, seed=seed)
    dev = torch.device("cuda:0")
    n_of = (torch.arange(P, dtype=torch.int64, device=dev) % K) + 1
    rows = n_of.clone()
    count = n_of.clone()
    parts = _native.Partials(P, rows.data_ptr(), count.data_ptr(), None, None, None)
    table = None
    f = dict(strategy=plan.native_strategy, table_len=0, keep_table=None,
             threshold=plan.threshold, noise_scale=plan.noise_scale, pre_threshold=pre,
             max_rows_per_privacy_id=1, pk_offset=0, public_mask=None, nonce=nonce)
    if plan.table is not None:
        table = np.ascontiguousarray(np.asarray(plan.table, dtype=np.float64))
        f["table_len"] = len(table)
        f["keep_table"] = table.ctypes.data
    sel = _native.fill(_native.SelectParams, f)
    nz = _native.fill(_native.NoiseParams, _noise_off())
    keep = torch.empty(P, dtype=torch.uint8, device=dev)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    backend.ctx.select_and_noise(parts, sel, nz, keep.data_ptr(), out.data_ptr(),
                                 ctypes.c_void_p(stream.cuda_stream))
    torch.cuda.synchronize()
    kept = torch.zeros(K + 1, dtype=torch.int64, device=dev).index_add_(
        0, n_of, keep.to(torch.int64)).cpu().numpy()
    trials = np.bincount((np.arange(P) % K) + 1, minlength=K + 1)
    probs = np.array([ps.probability_of_keep(plan, n) for n in range(K + 1)])
    return kept, trials, probs


def _check(kept, trials, probs):
    stat, dof = 0.0, 0
    for n in range(1, K + 1):
        m, k, p = int(trials[n]), int(kept[n]), float(probs[n])
        if p <= 0.0:
            assert k == 0, (n, k)
        elif p >= 1.0:
            assert k == m, (n, k, m)
        else:
            var = m * p * (1.0 - p)
            if var < 5.0:  # too few expected events for the normal approximation
                assert abs(k - m * p) <= 6.0 * math.sqrt(var) + 3.0, (n, k, m * p)
                continue
            stat += (k - m * p) ** 2 / var
            dof += 1
    assert dof >= 3, "the case must have several informative counts"
    pval = stats.chi2.sf(stat, dof)
    assert pval > 1e-4, (stat, dof, pval)


def test_truncated_geometric_keep_rates(built):
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    _check(*_keep_rates(S.TRUNCATED_GEOMETRIC, 1.0, 1e-3, 1))


def test_truncated_geometric_keep_rates_l0_3(built):
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    _check(*_keep_rates(S.TRUNCATED_GEOMETRIC, 2.0, 1e-3, 3))


def test_laplace_thresholding_keep_rates(built):
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    _check(*_keep_rates(S.LAPLACE_THRESHOLDING, 1.0, 1e-3, 2))


def test_gaussian_thresholding_keep_rates(built):
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    _check(*_keep_rates(S.GAUSSIAN_THRESHOLDING, 1.0, 1e-3, 2))


def test_pre_threshold_keep_rates(built):
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    kept, trials, probs = _keep_rates(S.TRUNCATED_GEOMETRIC, 1.0, 1e-3, 1, pre=4)
    assert kept[1:4].sum() == 0
    _check(kept, trials, probs)


def test_keep_rates_change_with_the_nonce(built):
    """Two releases (nonces) draw independent keep decisions: their kept
    sets agree on about p^2 + (1-p)^2 of the partitions, not all of them."""
    from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy as S
    a = _keep_rates(S.TRUNCATED_GEOMETRIC, 1.0, 1e-3, 1, nonce=1)[0]
    b = _keep_rates(S.TRUNCATED_GEOMETRIC, 1.0, 1e-3, 1, nonce=2)[0]
    assert not np.array_equal(a, b)
