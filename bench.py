"""Benchmark: DPEngine.aggregate COUNT+SUM+PRIVACY_ID_COUNT on MI355X.

Workload = BASELINE.json configs[1] per GPU: 1e9 records, 1e7 privacy ids,
1e6 Zipf(1.1) partitions (fixed permutation seeded 20250202), values
U[0, 10), mpc = 8, mcpp = 2 (bounding triggers), Laplace noise, eps = 1,
delta = 1e-6, truncated-geometric private partition selection.  With N GPUs
every rank holds its own privacy-id shard of the same size (weak scaling,
configs[2]); the partials are merged with one RCCL reduce-scatter.

A step = one full DPEngine.aggregate call on resident inputs: engine +
accountant construction, aggregate(), compute_budgets(), device execution
(bounding, merge, selection, noise, compaction) and the device sync.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--records R]
       python bench.py --workload config4 [--public]   (BASELINE configs[3]:
       MEAN+VARIANCE, Gaussian, Pareto(1.2) records per privacy id, mpc = 50,
       mcpp = 4, 1e8 partitions; --public: public_partitions = range(1e8))
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "records/sec DPEngine.aggregate COUNT+SUM at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0
ALGO_BYTES_PER_RECORD = 24  # pid int64 + pk int64 + value f64


def zipf_cdf(P: int, s: float, device) -> torch.Tensor:
    w = torch.arange(1, P + 1, dtype=torch.float64, device=device).pow(-s)
    c = torch.cumsum(w, 0)
    return c / c[-1]


def pareto_cdf(n_pid: int, alpha: float, cap: float, seed: int, device) -> torch.Tensor:
    """Heavy-tailed records per privacy id (config 4): pid i has weight
    min(Pareto(alpha, x_m = 1), cap), drawn once from a fixed seed."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    u = torch.rand(n_pid, dtype=torch.float64, generator=g, device=device)
    w = (1.0 - u).pow(-1.0 / alpha).clamp_(max=cap)
    c = torch.cumsum(w, 0)
    return c / c[-1]


def generate(n: int, n_pid: int, P: int, rank: int, seed: int, device, pid_cdf=None):
    """Synthetic Zipf-keyed records generated on the device (untimed).
    pid_cdf: sample privacy ids from this CDF instead of uniformly."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed * 1000 + rank)
    cdf = zipf_cdf(P, 1.1, device)
    perm = torch.randperm(P, generator=torch.Generator().manual_seed(20250202)).to(device)
    pid = torch.empty(n, dtype=torch.int64, device=device)
    pk = torch.empty(n, dtype=torch.int64, device=device)
    val = torch.empty(n, dtype=torch.float64, device=device)
    chunk = 1 << 27
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        if pid_cdf is None:
            pid[s:e] = torch.randint(0, n_pid, (e - s,), generator=gen, device=device)
        else:
            u = torch.rand(e - s, dtype=torch.float64, generator=gen, device=device)
            pid[s:e] = torch.searchsorted(pid_cdf, u).clamp_(max=n_pid - 1)
        pid[s:e] += rank * n_pid
        u = torch.rand(e - s, dtype=torch.float64, generator=gen, device=device)
        r = torch.searchsorted(cdf, u).clamp_(max=P - 1)
        pk[s:e] = perm[r]
        val[s:e] = torch.rand(e - s, dtype=torch.float64, generator=gen, device=device) * 10.0
    return pid, pk, val


def host_sample(n: int, n_pid: int, P: int, seed: int, pareto=None):
    rng = np.random.default_rng(seed)
    w = np.arange(1, P + 1, dtype=np.float64) ** -1.1
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    perm = np.random.default_rng(20250202).permutation(P)
    if pareto is None:
        pid = rng.integers(0, n_pid, n)
    else:
        alpha, cap = pareto
        pw = np.minimum((1.0 - rng.random(n_pid)) ** (-1.0 / alpha), cap)
        pc = np.cumsum(pw)
        pc /= pc[-1]
        pid = np.minimum(np.searchsorted(pc, rng.random(n)), n_pid - 1)
    pk = perm[np.minimum(np.searchsorted(cdf, rng.random(n)), P - 1)]
    val = rng.random(n) * 10.0
    return pid, pk, val


def cpu_baseline(args, P):
    """The C oracle (single core) on a bounded sample of the same workload."""
    from oracle import oracle
    import pipelinedp_amd as pdp
    from pipelinedp_amd import combiners
    n = args.cpu_records
    n_pid = max(1, int(round(args.pids * n / args.records)))
    pid, pk, val = host_sample(n, n_pid, P, 99,
                               (1.2, args.pid_cap) if args.workload == "config4" else None)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    plan = combiners.CompoundPlan(make_params(args), acc)
    fields = plan.bound_fields(P)
    t0 = time.perf_counter()
    oracle.bound_aggregate(pid, pk, val, fields, 5)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": f"{n} records, {n_pid} privacy ids, {P} partitions, same generator; "
                      f"C oracle bounding+merge only (selection/noise excluded), "
                      f"{dt:.1f} s on one host core"}


def make_params(args):
    import pipelinedp_amd as pdp
    if args.workload == "config4":
        return pdp.AggregateParams(
            metrics=[pdp.Metrics.MEAN, pdp.Metrics.VARIANCE],
            noise_kind=pdp.NoiseKind.GAUSSIAN, max_partitions_contributed=args.mpc,
            max_contributions_per_partition=args.mcpp, min_value=0.0, max_value=10.0)
    return pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=args.mpc,
        max_contributions_per_partition=args.mcpp, min_value=0.0, max_value=10.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["config2", "config4"], default="config2")
    ap.add_argument("--public", action="store_true",
                    help="config4: public_partitions = range(P) instead of private selection")
    ap.add_argument("--records", type=int, default=1_000_000_000)
    ap.add_argument("--pids", type=int, default=10_000_000)
    ap.add_argument("--partitions", type=int, default=None)
    ap.add_argument("--mpc", type=int, default=None)
    ap.add_argument("--mcpp", type=int, default=None)
    ap.add_argument("--pid-cap", type=float, default=1000.0,
                    help="config4: cap of the Pareto weight of one privacy id")
    ap.add_argument("--cpu-records", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    c4 = args.workload == "config4"
    if args.partitions is None:
        args.partitions = 100_000_000 if c4 else 1_000_000
    if args.mpc is None:
        args.mpc = 50 if c4 else 8
    if args.mcpp is None:
        args.mcpp = 4 if c4 else 2
    if args.cpu_records is None:
        args.cpu_records = 20_000_000 if c4 else 40_000_000

    import pipelinedp_amd as pdp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)
        group = torch.distributed.group.WORLD
    P = args.partitions
    pid_cdf = pareto_cdf(args.pids, 1.2, args.pid_cap, 4321, dev) if c4 else None
    pid, pk, val = generate(args.records, args.pids, P, rank, 1, dev, pid_cdf)
    del pid_cdf
    torch.cuda.synchronize()
    backend = pdp.MI355XBackend(device=local, seed=0xD1FF5EED, process_group=group)
    # the generator's privacy-id range and this rank's global record offset
    # are known metadata (like n_partitions): no device min/max pass
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P,
                            privacy_id_range=(rank * args.pids, (rank + 1) * args.pids),
                            record_id_offset=rank * args.records)
    ex = pdp.DataExtractors("pid", "pk", "value")
    params = make_params(args)
    public = range(P) if (c4 and args.public) else None

    def step():
        acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
        eng = pdp.DPEngine(acc, backend)
        res = eng.aggregate(cols, params, ex, public_partitions=public)
        acc.compute_budgets()
        out = res.materialize(gather=False)
        return res, out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if group is not None:
        torch.distributed.barrier()
    # device time of the hot path (HIP events on the stream the kernels use)
    stream = torch.cuda.current_stream(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    stage_tot = {}
    ev0.record(stream)
    kept = 0
    for _ in range(args.steps):
        res, out = step()
        kept = int(out.partition_ids.numel())
        for k, v in backend.ctx.stage_times().items():
            stage_tot[k] = stage_tot.get(k, 0.0) + v
    ev1.record(stream)
    torch.cuda.synchronize()
    if group is not None:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if group is not None:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    wall = float(t.item())
    ms_per_step = wall / args.steps * 1e3
    total_records = args.records * world
    value = total_records / (wall / args.steps)
    stage_ms = {k: v / args.steps for k, v in stage_tot.items()}
    path_ms = sum(stage_ms.values())
    algo_bytes = ALGO_BYTES_PER_RECORD * args.records
    # dominant kernel: the longest single-kernel stage (each of these stage
    # names brackets exactly one launch on the stream the kernels run on)
    kernels = {"bound": "k_bound_waves", "bound.medium": "k_bound_chunks",
               "partition1:scatter": "k_scatter<SrcSoAKey>",
               "partition2:scatter": "k_scatter<SrcAoS>",
               "bound.tail": "k_bound_big"}
    dom_stage = max(kernels, key=lambda k: stage_ms.get(k, 0.0))
    dom_kernel = kernels[dom_stage]
    dom_ms = stage_ms.get(dom_stage)
    achieved = algo_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms else None
    path_achieved = algo_bytes / (path_ms * 1e-3) / 1e9 if path_ms else None
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "hbm_traffic_c4.json" if c4 else "hbm_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            if tj.get("records") == args.records:
                traffic = tj.get("kernels", {}).get(dom_kernel)
        except Exception:
            traffic = None
    if c4:
        workload = (f"configs[3]: {args.records:.0e} records / {args.pids:.0e} privacy ids "
                    f"(Pareto(1.2) records per id, weight cap {args.pid_cap:g}) / {P:.0e} "
                    f"Zipf(1.1) partitions per GPU, MEAN+VARIANCE, Gaussian, "
                    + ("public partitions" if public is not None else "private selection"))
    else:
        workload = ("configs[1]: 1e9 records / 1e7 privacy ids / 1e6 Zipf(1.1) partitions "
                    "per GPU, COUNT+SUM+PRIVACY_ID_COUNT, private partition selection")
    line = {
        "metric": METRIC, "value": value, "unit": "records/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (device-generated Zipf keys, uniform values)",
        "config": {"workload": workload,
                   "records_per_gpu": args.records, "privacy_ids_per_gpu": args.pids,
                   "partitions": P, "max_partitions_contributed": args.mpc,
                   "max_contributions_per_partition": args.mcpp,
                   "noise": "gaussian" if c4 else "laplace",
                   "epsilon": 1.0, "delta": 1e-6,
                   "selection": "public" if public is not None else "truncated_geometric",
                   "parallelism": f"pid-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": traffic, "kernel": dom_kernel,
                     "kernel_ms": dom_ms,
                     "note": "achieved = 24 B/record x records / the dominant kernel's time "
                             "(HIP events on its stream); traffic = PMC HBM bytes per launch "
                             "of it (FETCH_SIZE x2 + WRITE_SIZE, profiles/hbm_traffic[_c4].json)"},
        "path_roofline": {"achieved": path_achieved, "frac":
                          (path_achieved / HBM_PEAK_GBS) if path_achieved else None,
                          "ms": path_ms,
                          "note": "24 B/record over the whole dpg_bound_aggregate device time"},
        "device_ms_per_step": dev_ms, "bound_aggregate_ms": path_ms, "stage_ms": stage_ms,
        "kept_partitions": kept,
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, P)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if group is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
