"""Host-side (Python) cost of one config-2 release on the GPU: cProfile over
the same step bench.py times (aggregate -> compute_budgets -> materialize),
printed by own time, plus the wall time of each step against its device
time.  The GPU idles while the host prepares a step, so this time is part
of bench.py's per-step device time.  Usage: python tools/host_profile.py
[records] [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pipelinedp_amd as pdp  # noqa: E402


def main(n=1_000_000_000, steps=5):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    P, U = 1_000_000, 10_000_000
    pid, pk, val = bench.generate(n, U, P, 0, 1, dev)
    backend = pdp.MI355XBackend(device=0, seed=1)
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P, privacy_id_range=(0, U))
    ex = pdp.DataExtractors("pid", "pk", "value")
    params = pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=8,
        max_contributions_per_partition=2, min_value=0.0, max_value=10.0)

    def step():
        acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
        res = pdp.DPEngine(acc, backend).aggregate(cols, params, ex)
        acc.compute_budgets()
        return res.materialize(gather=False)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    prof = cProfile.Profile()
    for i in range(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        prof.enable()
        step()
        prof.disable()
        e1.record(stream)
        torch.cuda.synchronize()
        print(f"step {i}: wall {1e3 * (time.perf_counter() - t0):.2f} ms, device "
              f"{e0.elapsed_time(e1):.2f} ms", flush=True)
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000,
         int(sys.argv[2]) if len(sys.argv) > 2 else 5)
