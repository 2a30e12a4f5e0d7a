"""GPU diagnostic: one aggregate at a given size / tuning, stage timings and
oracle parity of the partials.  Usage: diag_levels.py N PIDS P TARGET CAP [check]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import pipelinedp_amd as pdp  # noqa: E402

n, npid, P, target, cap = (int(x) for x in sys.argv[1:6])
check = len(sys.argv) > 6
rng = np.random.default_rng(3)
pid = rng.integers(0, npid, n)
pk = (rng.zipf(1.1, n) - 1) % P
val = rng.uniform(0, 10, n)
backend = pdp.MI355XBackend(device=0, seed=77)
backend.ctx.set_tuning(target, cap)
params = pdp.AggregateParams(metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM,
                                      pdp.Metrics.PRIVACY_ID_COUNT],
                             max_partitions_contributed=8, max_contributions_per_partition=2,
                             min_value=0.0, max_value=10.0)
cols = pdp.ColumnarData(pid=torch.from_numpy(pid).cuda(), pk=torch.from_numpy(pk).cuda(),
                        value=torch.from_numpy(val).cuda(), n_partitions=P)
for it in range(2):
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(cols, params, pdp.DataExtractors("pid", "pk", "value"))
    acc.compute_budgets()
    t = time.time()
    out = res.materialize()
    torch.cuda.synchronize()
    print(f"n={n} target={target} cap={cap} wall={time.time()-t:.3f}s kept={out.partition_ids.numel()} "
          f"stages={ {k: round(v, 3) for k, v in backend.ctx.stage_times().items()} }", flush=True)
if check:
    from oracle import oracle
    ref = oracle.bound_aggregate(pid, pk, val, res.plan.bound_fields(P), 77)
    got = {k: v.cpu().numpy() for k, v in res.last_partials.items() if v is not None}
    ok = (np.array_equal(got["rows"], ref["rows"]) and np.array_equal(got["count"], ref["count"])
          and np.allclose(got["sum"], ref["sum"], rtol=1e-9, atol=1e-9))
    print("parity", ok, int(got["rows"].sum()), int(ref["rows"].sum()), flush=True)
