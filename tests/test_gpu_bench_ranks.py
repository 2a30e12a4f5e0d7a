"""bench.py's own N-rank launcher (configs[2]'s path) on a one-GPU box: two
ranks share GPU 0 over gloo, at reduced size.  The printed line must show
what the collectives saw (2 ranks), every rank's timing, and -- for the same
seed and release nonce -- the same kept partition set and integer columns as
ONE rank over the union of both ranks' records, for both exchanges
(dense reduce-scatter and sparse all-to-all)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_line(*extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend",
           "gloo", "--records", "3000000", "--pids", "30000", "--partitions", "200000",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("exchange", ["reduce_scatter", "all_to_all"])
def test_two_rank_bench_line_and_single_rank_equality(built, exchange):
    d = _bench_line("--exchange", exchange)
    assert d["n_gpus"] == 2
    dd = d["distributed"]
    assert dd["backend"] == "gloo" and dd["world_size"] == 2
    assert dd["exchange"]["mode"] == exchange and dd["exchange"]["world_size"] == 2
    assert len(dd["rank_device_ms"]) == 2 and all(t > 0 for t in dd["rank_device_ms"])
    assert len(dd["rank_ms_per_step"]) == 2
    assert d["value"] > 0 and d["ms_per_step"] >= max(dd["rank_ms_per_step"]) - 1e-6
    # the one-rank check runs by default (no flag), on the whole of these
    # small shards
    c = dd["check_single"]
    assert c["records"] == 2 * 3_000_000 and c["records_per_rank"] == 3_000_000
    assert c["same_kept_set"] and c["integer_columns_equal"] and c["all_columns_close"], c
    assert 0 < c["kept_one_rank"] == c["kept_n_rank"]
    assert d["config"]["privacy_id_range_supplied"] is True
    assert d["kernels"]["pidrange_untimed"]["ms"] > 0


def test_two_rank_check_on_a_record_prefix(built):
    # --check-records: the check releases each rank's first m records (global
    # record ids rank * m + i) and their union as one rank
    d = _bench_line("--exchange", "reduce_scatter", "--check-records", "1000000")
    c = d["distributed"]["check_single"]
    assert c["records"] == 2 * 1_000_000 and c["records_per_rank"] == 1_000_000
    assert c["same_kept_set"] and c["integer_columns_equal"] and c["all_columns_close"], c
