"""Times the reference's CPU path (BUILD CONTAINER ONLY, test infrastructure).

Imports the read-only reference PipelineDP from /root/reference with the
no-noise PyDP stand-in of tests/golden/pydp_stub (noise and selection free:
the figures slightly OVERSTATE the reference's speed) and times
`DPEngine.aggregate` on `LocalBackend` -- engine + accountant construction,
aggregate(), compute_budgets(), list(result) -- on records of bench.py's own
generator (bench.host_sample: privacy ids uniform with 100 records each, 1e6
Zipf(1.1) partitions under the fixed permutation, values U[0, 10)), with
the bench's parameters (COUNT + SUM + PRIVACY_ID_COUNT, mpc 8, mcpp 2,
Laplace, eps 1, delta 1e-6, private partition selection).  LocalBackend is
single-threaded generators: one core.  Writes profiles/cpu_ref_r05.json,
which bench.py reports beside its C-port CPU baseline.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/time_reference_cpu.py [N ...]
"""
import datetime
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "pydp_stub"))
sys.path.insert(0, "/root/reference")

import pipeline_dp  # noqa: E402  (the reference, read-only)

import bench  # noqa: E402  (the generator only)

P = 1_000_000


def time_one(n: int) -> dict:
    pid, pk, val = bench.host_sample(n, max(1, n // 100), P, 20250202)
    rows = list(zip(pid.tolist(), pk.tolist(), val.tolist()))
    t0 = time.perf_counter()
    acc = pipeline_dp.NaiveBudgetAccountant(1.0, 1e-6)
    engine = pipeline_dp.DPEngine(acc, pipeline_dp.LocalBackend())
    params = pipeline_dp.AggregateParams(
        metrics=[pipeline_dp.Metrics.COUNT, pipeline_dp.Metrics.SUM,
                 pipeline_dp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pipeline_dp.NoiseKind.LAPLACE, max_partitions_contributed=8,
        max_contributions_per_partition=2, min_value=0.0, max_value=10.0)
    ex = pipeline_dp.DataExtractors(privacy_id_extractor=lambda r: r[0],
                                    partition_extractor=lambda r: r[1],
                                    value_extractor=lambda r: r[2])
    res = engine.aggregate(rows, params, ex)
    acc.compute_budgets()
    out = list(res)
    dt = time.perf_counter() - t0
    return {"records": n, "privacy_ids": max(1, n // 100), "partitions": P,
            "released_partitions": len(out), "seconds": round(dt, 3),
            "records_per_s": n / dt}


def main(sizes):
    runs = [time_one(n) for n in sizes]
    line = {
        "what": "reference LocalBackend DPEngine.aggregate (COUNT+SUM+PRIVACY_ID_COUNT, mpc 8, "
                "mcpp 2, Laplace, private selection) on bench.host_sample records",
        "kind": "reference", "cores": 1,
        "caveat": "no-noise / keep-all PyDP stand-in (tests/golden/pydp_stub): noise and "
                  "selection cost nothing, so the reference's true speed is somewhat lower",
        "host": {"nproc": os.cpu_count(), "python": platform.python_version(),
                 "machine": platform.machine()},
        "date": datetime.date.today().isoformat(),
        "script": "tools/time_reference_cpu.py",
        "runs": runs,
    }
    out = os.path.join(ROOT, "profiles", "cpu_ref_r05.json")
    with open(out, "w") as f:
        json.dump(line, f, indent=1)
    print(json.dumps(line))


if __name__ == "__main__":
    main([int(float(a)) for a in sys.argv[1:]] or [1_000_000, 10_000_000])
