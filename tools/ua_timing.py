"""Host / device time split of one config-5 utility-analysis step (GPU):
object setup, pre-aggregate call, sweep call, report assembly, each bracketed
by a stream synchronisation.  Usage: python tools/ua_timing.py [records]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pipelinedp_amd as pdp  # noqa: E402
from pipelinedp_amd.analysis import utility_analysis as ua  # noqa: E402


def main(n=1_000_000_000, pids=10_000_000, P=1_000_000):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pid, pk, val = bench.generate(n, pids, P, 0, 1, dev)
    backend = pdp.MI355XBackend(device=0, seed=1)
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P, privacy_id_range=(0, pids))
    opts, _, _ = bench._ua_options()
    ex = pdp.DataExtractors("pid", "pk", "value")
    for it in range(3):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        run = ua.UtilityAnalysis(cols, backend, opts, ex)
        t.append(time.perf_counter())
        ps = run._pairs(dev)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        run._pairs = lambda d, ps=ps: ps
        run.run()
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        reps = run.reports()
        t.append(time.perf_counter())
        st = run.stage_ms
        dt = [round((b - a) * 1e3, 1) for a, b in zip(t, t[1:])]
        print(f"step {it}: setup/preagg/sweep/reports ms {dt}; sweep stages "
              f"{ {k: round(v, 1) for k, v in st.items() if v > 0.5} }", flush=True)
        del run, reps, ps


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000)
