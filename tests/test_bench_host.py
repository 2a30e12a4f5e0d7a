"""Host-side logic of bench.py (no GPU): the PMC traffic of
profiles/hbm_traffic*.json is attached only to the workload its passes
measured (configs[1] / configs[3] private at their default sizes), never
to an envelope input or the public-partition line."""
import argparse

import bench


def _args(**kw):
    a = dict(records=1_000_000_000, pids=10_000_000, partitions=1_000_000, mpc=8, mcpp=2,
             public=False, pid_cap=1000.0)
    a.update(kw)
    return argparse.Namespace(**a)


def test_default_workloads_carry_traffic():
    assert bench._default_workload(_args(), c4=False)
    assert bench._default_workload(_args(partitions=100_000_000, mpc=50, mcpp=4), c4=True)


def test_envelope_and_public_lines_do_not():
    assert not bench._default_workload(_args(pids=1_000_000), c4=False)
    assert not bench._default_workload(_args(records=2_000_000_000, pids=20_000_000), c4=False)
    assert not bench._default_workload(
        _args(partitions=100_000_000, mpc=50, mcpp=4, public=True), c4=True)
    tj, why = bench._traffic(False, 1_000_000_000, default=False)
    assert tj is None and "default" in why
