"""Benchmark: DPEngine.aggregate COUNT+SUM+PRIVACY_ID_COUNT on MI355X.

Workload = BASELINE.json configs[1] per GPU: 1e9 records, 1e7 privacy ids,
1e6 Zipf(1.1) partitions (fixed permutation seeded 20250202), values
U[0, 10), mpc = 8, mcpp = 2 (bounding triggers), Laplace noise, eps = 1,
delta = 1e-6, truncated-geometric private partition selection.  With N GPUs
every rank holds its own privacy-id shard of the same size (weak scaling,
configs[2]); the partials are merged with one RCCL reduce-scatter.

A step = one full DPEngine.aggregate call on resident inputs: engine +
accountant construction, aggregate(), compute_budgets(), device execution
(bounding, merge, selection, noise, compaction) and the device sync.  Every
step is a fresh release (fresh nonce).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--records R]
       python bench.py --workload config4 [--public]   (BASELINE configs[3]:
       MEAN+VARIANCE, Gaussian, Pareto(1.2) records per privacy id, mpc = 50,
       mcpp = 4, 1e8 partitions; --public: public_partitions = range(1e8))
--gpus N without a torch.distributed launcher re-launches itself as N ranks
(torch.distributed.run, 127.0.0.1) before touching any GPU.  Multi-rank
options: --dist-backend nccl (RCCL, default; one GPU per rank) or gloo (host-
staged collectives; ranks may share a GPU: rank r uses GPU r mod #GPUs, which
is how a one-GPU box rehearses the N-rank path), --exchange auto |
reduce_scatter | all_to_all (distributed.exchange_partials).  After timing,
every multi-rank run checks itself (distributed.check_single; --no-check-single
skips it): each rank keeps the first --check-records of its records (default
min(records, 1e8, 4e8 / N)), the N ranks release them with a fixed nonce, the
prefixes are gathered to rank 0, which releases their union as ONE rank with
the same nonce, and the line reports whether the kept partition sets and the
exact columns agree (the selected set does not depend on N).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "records/sec DPEngine.aggregate COUNT+SUM at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0
ALGO_BYTES_PER_RECORD = 24  # pid int64 + pk int64 + value f64
CPU_SHARE = 16              # host cores of one GPU's share on the GPU box


def reference_local_backend():
    """The reference's own CPU path (LocalBackend, stub PyDP, one Python
    thread), timed in the build container by tools/time_reference_cpu.py on
    this bench's generator at 1e6 and 1e7 records (profiles/cpu_ref_r05.json;
    the reference cannot travel to the GPU box) -- context beside the C-port
    baseline, at the largest size timed."""
    f = os.path.join(ROOT, "profiles", "cpu_ref_r05.json")
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    run = max(d["runs"], key=lambda r: r["records"])
    return {"value": run["records_per_s"], "unit": "records/s", "cores": d["cores"],
            "kind": "reference",
            "sample": f"reference LocalBackend DPEngine.aggregate, {run['records']:.0e} records of "
                      f"this bench's generator ({run['privacy_ids']:.0e} privacy ids, "
                      f"{run['partitions']:.0e} Zipf partitions), mpc 8 / mcpp 2, no-noise PyDP "
                      f"stand-in, build container ({d['host']['nproc']} cores, 1 used), "
                      f"{d['date']}; {os.path.relpath(f, ROOT)}",
            "runs": [{"records": r["records"], "records_per_s": round(r["records_per_s"])}
                     for r in d["runs"]]}


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


def host_tables(P: int):
    """Zipf(1.1) CDF over partition ranks and the fixed rank -> key permutation."""
    w = np.arange(1, P + 1, dtype=np.float64) ** -1.1
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return cdf, np.random.default_rng(20250202).permutation(P)


def host_sample(n: int, n_pid: int, P: int, seed: int, pareto=None, pid_lo: int = 0,
                tables=None):
    """The same generator on the host (numpy): privacy ids in
    [pid_lo, pid_lo + n_pid)."""
    rng = np.random.default_rng(seed)
    cdf, perm = tables if tables is not None else host_tables(P)
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
    return pid + pid_lo, pk, val


# ---------------------------------------------------------------- CPU baseline
_ACC = ("rows", "count", "sum", "nsum", "nsq")


_TABLES = None  # host_tables(P), built once before the workers fork


def _cpu_worker(w, n, n_pid_total, k, P, pareto, fields, seed, start_evt, ready_q, out_q):
    """One host core: generate this worker's privacy-id shard, wait for the
    common start, bound + merge it with the C oracle (timed); returns the
    non-zero partials (sparse, so P = 1e8 does not cross the pipe densely)."""
    from oracle import oracle
    lo = w * n_pid_total // k
    hi = (w + 1) * n_pid_total // k
    pid, pk, val = host_sample(n, hi - lo, P, 99 + w, pareto, pid_lo=lo, tables=_TABLES)
    f = dict(fields, rec_id_offset=w * n)
    oracle.lib()
    ready_q.put(w)
    start_evt.wait()
    t0 = time.perf_counter()
    part = oracle.bound_aggregate(pid, pk, val, f, seed)
    nz = np.nonzero(part["rows"])[0]
    dt = time.perf_counter() - t0
    out_q.put((w, nz, {key: part[key][nz] for key in _ACC}, dt))


def cpu_baseline(args, P):
    """The C oracle's FULL path on the GPU box's host cores: one process per
    core on disjoint privacy-id shards (bounding + merge), then the merge of
    the shards' partials and the oracle's selection + noise -- the same work
    as one GPU step, on a bounded sample of the same generator.  Runs before
    this process touches the GPU (forked workers)."""
    import multiprocessing as mp
    from oracle import oracle
    import pipelinedp_amd as pdp
    from pipelinedp_amd import combiners, partition_selection
    k = max(1, min(CPU_SHARE, os.cpu_count() or 1))
    n_each = args.cpu_records // k
    n_pid = max(k, int(round(args.pids * args.cpu_records / args.records)))
    pareto = (1.2, args.pid_cap) if args.workload == "config4" else None
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    params = make_params(args)
    public = args.workload == "config4" and args.public
    plan = combiners.CompoundPlan(params, acc)
    sel_spec = None if public else acc.request_budget(pdp.MechanismType.GENERIC)
    acc.compute_budgets()
    fields = dict(plan.bound_fields(P), nonce=1)
    global _TABLES
    _TABLES = host_tables(P)
    ctx = mp.get_context("fork")
    start_evt, ready_q, out_q = ctx.Event(), ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(w, n_each, n_pid, k, P, pareto, fields, 5,
                                                   start_evt, ready_q, out_q))
             for w in range(k)]
    for p in procs:
        p.start()
    try:
        for _ in range(k):
            ready_q.get(timeout=600)
        t0 = time.perf_counter()
        start_evt.set()
        tot = {key: np.zeros(P, np.int64 if key in ("rows", "count") else np.float64)
               for key in _ACC}
        slowest = 0.0
        for _ in range(k):
            w, nz, part, dt = out_q.get(timeout=1200)
            slowest = max(slowest, dt)
            for key in _ACC:
                np.add.at(tot[key], nz, part[key])
        if public:
            sel = dict(strategy=0, max_rows_per_privacy_id=1, nonce=1)
            mask = np.full((P + 7) // 8, 0xFF, np.uint8)
            oracle.select_and_noise(tot, sel, plan.noise_fields(True), 5, public_mask=mask)
        else:
            sp = partition_selection.create_partition_selection_strategy(
                params.partition_selection_strategy, sel_spec.eps, sel_spec.delta,
                params.max_partitions_contributed)
            sel = dict(strategy=sp.native_strategy, threshold=sp.threshold,
                       noise_scale=sp.noise_scale, pre_threshold=0,
                       max_rows_per_privacy_id=1, nonce=1)
            oracle.select_and_noise(tot, sel, plan.noise_fields(True), 5,
                                    keep_table=None if sp.table is None else np.asarray(sp.table))
        dt = time.perf_counter() - t0
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    n_done = n_each * k
    return {"value": n_done / dt, "unit": "records/s", "cores": k, "kind": "port",
            "sample": f"{n_done:.1e} records, {n_pid} privacy ids, {P} partitions, same "
                      f"generator (one privacy-id range per core); C oracle full path: "
                      f"bounding+merge in {k} processes (slowest {slowest:.1f} s), merge of "
                      f"the shards' partials, selection + noise; {dt:.1f} s wall",
            "reference_local_backend": reference_local_backend()}


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


# ------------------------------------------------------------ per-stage bytes
def stage_design_bytes(stage: str, n: int, rec: int, item: int, kept_recs: int,
                       kept_pairs: int, P: int, n_accum: int):
    """Design HBM bytes of one stage: what the
    stage must move at minimum for its job, not what it measures."""
    if stage == "pidrange":
        return 8 * n
    if stage == "partition1:hist":
        return 8 * n                      # pid column
    if stage in ("partition1:scatter", "partition1:pieces"):
        return (16 + rec) * n             # pid + pk in, packed record out (pieces: no hist pass)
    if stage in ("partition2:hist", "refine:hist"):
        return rec * n
    if stage in ("partition2:scatter", "refine:scatter", "partition2:team"):
        return 2 * rec * n                # records in and out (team level 2: no hist pass)
    if stage == "bounding":               # all bounding kernels: records in, kept
        return rec * n + 8 * kept_recs + item * kept_pairs  # values gathered, items out
    if stage in ("items:hist", "items2:hist"):
        return item * kept_pairs
    if stage in ("items:scatter", "items2:scatter"):
        return 2 * item * kept_pairs
    if stage == "reduce":
        return item * kept_pairs + 8 * n_accum * P
    return None


def _lib_sha() -> str:
    from pipelinedp_amd import _native
    with open(_native.library_path(), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _default_workload(args, c4: bool) -> bool:
    """The workload configs[1] / configs[3] (private) name, which the PMC
    passes of tools/gpu_r6_final.sh measure (other inputs: no traffic)."""
    return (args.records == 1_000_000_000 and args.pids == 10_000_000 and
            args.partitions == (100_000_000 if c4 else 1_000_000) and
            args.mpc == (50 if c4 else 8) and args.mcpp == (4 if c4 else 2) and
            not (c4 and args.public) and (not c4 or args.pid_cap == 1000.0))


def _traffic(c4: bool, records: int, default: bool = True):
    """PMC HBM bytes per step from profiles/hbm_traffic[_c4].json -- only if
    that file was measured on this exact libdpg.so build, for this workload."""
    if not default:
        return None, "PMC passes measure the default private workload only"
    tfile = os.path.join(ROOT, "profiles", "hbm_traffic_c4.json" if c4 else "hbm_traffic.json")
    if not os.path.exists(tfile):
        return None, "no PMC file"
    try:
        tj = json.load(open(tfile))
    except Exception:
        return None, "unreadable PMC file"
    if tj.get("records") != records:
        return None, "PMC file measured at another record count"
    if tj.get("lib_sha256") != _lib_sha():
        return None, f"PMC file measured on another build ({tj.get('lib_sha256')})"
    return tj, os.path.relpath(tfile, ROOT)


def _launch_ranks(n: int) -> int:
    """Re-executes this script as n ranks under torch.distributed.run, as a
    child process started before this process touches a GPU."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def _ua_options(n_side: int = 8):
    """configs[4]: 64 MultiParameterConfiguration rows, mpc x mcpp in
    {1, 2, 4, ..., 128}^2, COUNT + SUM + PRIVACY_ID_COUNT, private selection."""
    import pipelinedp_amd as pdp
    from pipelinedp_amd import analysis
    vals = [2**i for i in range(n_side)]
    mpc = [a for a in vals for _ in vals]
    mcpp = [b for _ in vals for b in vals]
    multi = analysis.MultiParameterConfiguration(
        max_partitions_contributed=mpc, max_contributions_per_partition=mcpp,
        min_sum_per_partition=[0.0] * len(mpc), max_sum_per_partition=[10.0 * b for b in mcpp])
    params = pdp.AggregateParams(
        metrics=[pdp.Metrics.COUNT, pdp.Metrics.SUM, pdp.Metrics.PRIVACY_ID_COUNT],
        noise_kind=pdp.NoiseKind.LAPLACE, max_partitions_contributed=1,
        max_contributions_per_partition=1, min_sum_per_partition=0.0, max_sum_per_partition=10.0)
    return analysis.UtilityAnalysisOptions(epsilon=1.0, delta=1e-6, aggregate_params=params,
                                           multi_param_configuration=multi), mpc, mcpp


def _ua_cpu_baseline(n_records: int, P: int):
    """The same 64-configuration sweep on the host: the vectorised numpy
    restatement (oracle/utility_sweep_np.py: pre-aggregation + every
    configuration's per-partition keep probability and error terms; the
    configurations split over the host cores) on a sample of the same
    generator (100 records per privacy id, P Zipf partitions)."""
    from oracle import utility_sweep_np as us
    _, mpc, mcpp = _ua_options()
    n_pid = max(1, n_records // 100)
    pid, pk, val = host_sample(n_records, n_pid, P, 7)
    cfgs = [dict(mpc=a, mcpp=b, min_sum=0.0, max_sum=10.0 * b, noise_kind="LAPLACE",
                 strategy="TRUNCATED_GEOMETRIC", pre_threshold=None) for a, b in zip(mpc, mcpp)]
    workers = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    pa, _ = us.sweep(pid, pk, val, cfgs, ["COUNT", "SUM", "PRIVACY_ID_COUNT"], 1.0, 1e-6,
                     workers=workers)
    dt = time.perf_counter() - t0
    return {"value": n_records / dt, "unit": "records/s", "cores": workers, "kind": "port",
            "sample": f"{n_records} records, {n_pid} privacy ids, {P} Zipf partitions "
                      f"({len(pa['pk'])} non-empty), 64 configurations; "
                      f"oracle/utility_sweep_np.py (vectorised numpy, configurations over "
                      f"{workers} processes): pre-aggregation + per-partition keep "
                      f"probabilities and error terms (no cross-partition report), {dt:.1f} s"}


def bench_config5(args):
    """configs[4]: utility-analysis sweep of 64 contribution-bound
    configurations over 1e9 records in one device pass (pre-aggregate +
    per-partition sweep + cross-partition reports), single GPU."""
    import pipelinedp_amd as pdp
    from pipelinedp_amd import analysis
    if args.gpus != 1:
        raise SystemExit("config5 runs on one GPU (the sweep does not shard)")
    P = args.partitions or 1_000_000
    cpu = None if args.no_cpu_baseline else _ua_cpu_baseline(1_000_000, P)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pid, pk, val = generate(args.records, args.pids, P, 0, 1, dev)
    torch.cuda.synchronize()
    backend = pdp.MI355XBackend(device=0, seed=0xD1FF5EED)
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P,
                            privacy_id_range=(0, args.pids))
    opts, _, _ = _ua_options()
    ex = pdp.DataExtractors("pid", "pk", "value")

    def step():
        reports, _ = analysis.perform_utility_analysis(cols, backend, opts, ex)
        return list(reports), reports.analysis

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    stage_tot = {}
    reps = run = None
    for _ in range(args.steps):
        # the previous step's analysis (its ~23 GB of pairs) is released
        # before the next one allocates: a caller keeps one analysis at a time
        reps = run = None
        reps, run = step()
        for k, v in run.stage_ms.items():
            stage_tot[k] = stage_tot.get(k, 0.0) + v
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1) / args.steps
    ms = wall / args.steps * 1e3
    C = len(reps)
    algo = ALGO_BYTES_PER_RECORD * args.records + C * P * 40
    achieved = algo / (dev_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": args.records / (wall / args.steps), "unit": "records/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (device-generated Zipf keys, uniform values)",
        "config": {"workload": f"configs[4]: utility-analysis sweep of {C} configurations "
                               f"(mpc x mcpp in {{1..128}}^2) over {args.records:.0e} records / "
                               f"{args.pids:.0e} privacy ids / {P:.0e} Zipf(1.1) partitions, "
                               "COUNT+SUM+PRIVACY_ID_COUNT, private selection",
                   "records": args.records, "partitions": P, "configurations": C,
                   "pairs": int(run.n_pairs), "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "device_ms": dev_ms,
                     "kernel": "whole sweep (dpg_preaggregate + dpg_utility_analysis + "
                               "cross-partition combine)",
                     "note": "achieved = (24 B x records + configurations x partitions x 40 B) "
                             "/ device time per step (SURVEY.md 8(d))"},
        "stage_ms": {k: v / args.steps for k, v in stage_tot.items()},
        "lib_sha256": _lib_sha(),
    }
    if cpu is not None:
        line["cpu_baseline"] = cpu
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["config2", "config4", "config5"], default="config2")
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
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl")
    ap.add_argument("--exchange", choices=["auto", "reduce_scatter", "all_to_all"],
                    default="auto")
    ap.add_argument("--check-single", action="store_true",
                    help="(default for N > 1; kept for compatibility)")
    ap.add_argument("--no-check-single", action="store_true",
                    help="multi-rank: skip the one-rank equality check after timing")
    ap.add_argument("--check-records", type=int, default=None,
                    help="records per rank in the one-rank check (default min(records, 1e8, "
                         "4e8 / N))")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args.gpus))
    if args.workload == "config5":
        return bench_config5(args)
    c4 = args.workload == "config4"
    if args.partitions is None:
        args.partitions = 100_000_000 if c4 else 1_000_000
    if args.mpc is None:
        args.mpc = 50 if c4 else 8
    if args.mcpp is None:
        args.mcpp = 4 if c4 else 2
    if args.cpu_records is None:
        args.cpu_records = 48_000_000 if c4 else 160_000_000

    import pipelinedp_amd as pdp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # the CPU baseline runs first, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, args.partitions)
    # device_count() does not initialise the GPU; gloo ranks may share one
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev if args.dist_backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    group = None
    if world > 1:
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group("gloo")
        group = torch.distributed.group.WORLD
    P = args.partitions
    pid_cdf = pareto_cdf(args.pids, 1.2, args.pid_cap, 4321, dev) if c4 else None
    pid, pk, val = generate(args.records, args.pids, P, rank, 1, dev, pid_cdf)
    del pid_cdf
    torch.cuda.synchronize()
    backend = pdp.MI355XBackend(device=gpu, seed=0xD1FF5EED, process_group=group,
                                exchange=args.exchange)
    # the generator's privacy-id range and this rank's global record offset
    # are known metadata (like n_partitions): no device min/max pass
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P,
                            privacy_id_range=(rank * args.pids, (rank + 1) * args.pids),
                            record_id_offset=rank * args.records)
    ex = pdp.DataExtractors("pid", "pk", "value")
    params = make_params(args)
    public = range(P) if (c4 and args.public) else None

    def step(resolve=True):
        acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
        eng = pdp.DPEngine(acc, backend)
        res = eng.aggregate(cols, params, ex, public_partitions=public)
        acc.compute_budgets()
        out = res.materialize(gather=False)
        if resolve:
            # every timed release is read back as a caller would: its kept
            # count (one host synchronisation), its compaction tail and the
            # bounding's error check are inside the step
            int(out.partition_ids.numel())
        return res, out

    def timed(resolve):
        torch.cuda.synchronize()
        if group is not None:
            torch.distributed.barrier()
        # device time of the hot path (HIP events on the stream the kernels use)
        stream = torch.cuda.current_stream(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        r = o = None
        for _ in range(args.steps):
            r, o = step(resolve)
        ev1.record(stream)
        torch.cuda.synchronize()
        if group is not None:
            torch.distributed.barrier()
        return time.perf_counter() - t0, ev0.elapsed_time(ev1) / args.steps, r, o

    for _ in range(args.warmup):
        step()
    # headline: releases read one by one; beside it (labelled, not the
    # value), releases enqueued back to back without reading them, where each
    # one's tail overlaps the next one's host work
    wall, dev_ms, res, out = timed(True)
    wall_pl, _, _, _ = timed(False)
    # the per-stage breakdown from one more, untimed step: reading a step's
    # stage events is host work the timed steps do not include
    res, out = step()
    stage_tot = backend.ctx.stage_times()
    # untimed: what a caller that does not declare the privacy-id range pays
    # on top (the device min / max pass over the pid column, stage "pidrange")
    nohint = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P,
                              record_id_offset=rank * args.records)
    acc_nh = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    r_nh = pdp.DPEngine(acc_nh, backend).aggregate(nohint, params, ex, public_partitions=public)
    acc_nh.compute_budgets()
    r_nh.materialize(gather=False)
    pidrange_ms = backend.ctx.stage_times().get("pidrange")
    del r_nh, nohint
    per_rank = [[wall, dev_ms, wall_pl]]
    if group is not None:
        cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        mine = torch.tensor([wall, dev_ms, wall_pl], dtype=torch.float64, device=cdev)
        got = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(got, mine)
        per_rank = [g.cpu().tolist() for g in got]
    wall = max(r[0] for r in per_rank)
    dev_ms_max = max(r[1] for r in per_rank)
    wall_pl = max(r[2] for r in per_rank)
    ms_per_step = wall / args.steps * 1e3
    total_records = args.records * world
    value = total_records / (wall / args.steps)
    kept = int(out.partition_ids.numel())
    lp = res.last_partials
    kept_pairs = int(lp["rows"].sum().item())
    kept_recs = int(lp["count"].sum().item())
    stage_ms = dict(stage_tot)
    path_ms = sum(v for k, v in stage_ms.items() if k != "bounding")
    # 24 B per record; MEAN+VARIANCE (config 4) adds 40 B per
    # partition of partials (rows, count, nsum, nsq + the noised outputs)
    algo_bytes = ALGO_BYTES_PER_RECORD * args.records + (40 * P if c4 else 0)
    # record / item formats of the two workloads: config
    # 4 packs 12-byte R12 records (70 key bits) and 24-byte ItemV items
    # (MEAN + VARIANCE without SUM: rows, count, nsum, nsq partials)
    n_accum = 4 if c4 else 3
    rec_bytes = 12 if c4 else 8
    item_bytes = 24 if c4 else 16
    # the bounding kernels as one stage (the sort kernel's wide pass, the
    # medium and global-memory kernels, the heavy-id filter)
    bparts = [k for k in stage_ms if k in ("heavy", "bound", "bound.wide", "bound.medium", "bound.tail")]
    if bparts:
        stage_ms["bounding"] = sum(stage_ms[k] for k in bparts)
    # headline: the whole path (24 B/record over the device time per step)
    achieved = algo_bytes / (dev_ms_max * 1e-3) / 1e9
    dflt = _default_workload(args, c4)
    tj, tsrc = _traffic(c4, args.records, dflt)
    kernels = {}
    for st, ms in stage_ms.items():
        b = stage_design_bytes(st, args.records, rec_bytes, item_bytes, kept_recs, kept_pairs,
                               P, n_accum)
        kernels[st] = {"ms": round(ms, 4)}
        if b is not None and ms > 0:
            kernels[st].update(design_bytes=b, achieved_gbs=round(b / (ms * 1e-3) / 1e9, 1),
                               frac=round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    if c4:
        workload = (f"configs[3]: {args.records:.0e} records / {args.pids:.0e} privacy ids "
                    f"(Pareto(1.2) records per id, weight cap {args.pid_cap:g}) / {P:.0e} "
                    f"Zipf(1.1) partitions per GPU, MEAN+VARIANCE, Gaussian, "
                    + ("public partitions" if public is not None else "private selection"))
    else:
        workload = (("configs[1]: " if dflt else "envelope input (not configs[1]): ") +
                    f"{args.records:.0e} records / {args.pids:.0e} privacy ids / {P:.0e} "
                    "Zipf(1.1) partitions per GPU, COUNT+SUM+PRIVACY_ID_COUNT, private "
                    "partition selection")
    line = {
        "metric": METRIC, "value": value, "unit": "records/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "ms_per_step_pipelined": wall_pl / args.steps * 1e3,
        "ms_per_step_note": "ms_per_step / value: each release read back (kept count, one host "
                            "sync) inside its step; ms_per_step_pipelined: the same releases "
                            "enqueued back to back without reading them (each tail overlaps "
                            "the next release's host work), not the headline",
        "dtype": "f64", "data": "synthetic (device-generated Zipf keys, uniform values)",
        "config": {"workload": workload,
                   "records_per_gpu": args.records, "privacy_ids_per_gpu": args.pids,
                   "partitions": P, "max_partitions_contributed": args.mpc,
                   "max_contributions_per_partition": args.mcpp,
                   "noise": "gaussian" if c4 else "laplace",
                   "epsilon": 1.0, "delta": 1e-6,
                   "selection": "public" if public is not None else "truncated_geometric",
                   "parallelism": f"pid-sharded x{world}",
                   # caller metadata, like n_partitions: the timed calls skip
                   # the device min / max of the pid column (its cost, from an
                   # untimed call without the hint: kernels["pidrange_untimed"])
                   "privacy_id_range_supplied": True},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (tj["bytes_per_step"] if tj else None),
                     "kernel": "whole path (dpg_bound_aggregate + select/noise + compact)",
                     "device_ms": dev_ms_max,
                     "algorithmic_bytes": algo_bytes,
                     "note": "achieved = 24 B/record x records (+ 40 B/partition for MEAN+VARIANCE, "
                             "SURVEY.md 8(d)) / device time per step (HIP "
                             "events on the kernels' stream, max over ranks); traffic = PMC "
                             "HBM bytes per step (FETCH_SIZE x calibrated factor + WRITE_SIZE) "
                             f"from {tsrc}"},
        "kernels": kernels,
        "kept_partitions": kept, "kept_pairs": kept_pairs, "kept_records": kept_recs,
        "lib_sha256": _lib_sha(),
    }
    if pidrange_ms is not None:
        b = stage_design_bytes("pidrange", args.records, rec_bytes, item_bytes, 0, 0, P, n_accum)
        kernels["pidrange_untimed"] = {
            "ms": round(pidrange_ms, 4), "design_bytes": b,
            "achieved_gbs": round(b / (pidrange_ms * 1e-3) / 1e9, 1),
            "note": "one call WITHOUT privacy_id_range (not in the timed steps): the extra "
                    "device min/max pass a caller that does not declare the range pays"}
    if tj:
        line["roofline"]["traffic_by_kernel"] = tj.get("kernels")
    if cpu is not None:
        line["cpu_baseline"] = cpu
    if group is not None:
        # what the collectives actually saw, and every rank's own timing
        line["distributed"] = {
            "backend": torch.distributed.get_backend(group),
            "world_size": torch.distributed.get_world_size(group),
            "devices": ndev if args.dist_backend == "gloo" else world,
            "exchange": res.last_exchange,
            "rank_ms_per_step": [r[0] / args.steps * 1e3 for r in per_rank],
            "rank_device_ms": [r[1] for r in per_rank]}
        if not args.no_check_single:
            line["distributed"]["check_single"] = check_single(
                args, (pid, pk, val), params, public, world, rank, dev, group)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if group is not None:
        torch.distributed.destroy_process_group()


def check_single(args, data, params, public, world, rank, dev, group):
    """The N-rank path against ONE rank, on a bounded prefix of every rank's
    records (the selected set must not depend on the number of
    GPUs).  Each rank keeps its first m records (global record ids rank * m
    + i, so that the concatenation in rank order carries the same ids); the
    N ranks release them with a fixed nonce; the prefixes are gathered to
    rank 0 (RCCL point-to-point, or through the host for gloo), which
    releases their union as one rank with the same nonce.  Kept partition
    sets and the integer columns (count, privacy id count) must be equal,
    the other columns equal to 1e-9 relative."""
    import pipelinedp_amd as pdp
    nonce = 0x5EED0F2A11
    m = args.check_records or min(args.records, 100_000_000, 400_000_000 // world)
    m = max(1, min(m, args.records))
    pid, pk, val = (t[:m] for t in data)
    ex = pdp.DataExtractors("pid", "pk", "value")
    P = args.partitions
    cols = pdp.ColumnarData(pid=pid, pk=pk, value=val, n_partitions=P,
                            privacy_id_range=(rank * args.pids, (rank + 1) * args.pids),
                            record_id_offset=rank * m)
    backend = pdp.MI355XBackend(device=dev.index, seed=0xD1FF5EED, process_group=group,
                                exchange=args.exchange)
    acc = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res = pdp.DPEngine(acc, backend).aggregate(cols, params, ex, public_partitions=public)
    acc.compute_budgets()
    res.nonce = nonce
    out = res.materialize(gather=True)
    del res, backend
    # the prefixes to rank 0, in rank order
    host = args.dist_backend == "gloo"
    parts = [None] * world
    if rank == 0:
        parts[0] = (pid, pk, val)
        for r in range(1, world):
            got = []
            for t in (pid, pk, val):
                buf = torch.empty(m, dtype=t.dtype, device="cpu" if host else dev)
                torch.distributed.recv(buf, src=r, group=group)
                got.append(buf.to(dev))
            parts[r] = tuple(got)
    else:
        for t in (pid, pk, val):
            torch.distributed.send(t.contiguous().cpu() if host else t.contiguous(), dst=0,
                                   group=group)
    torch.distributed.barrier()
    if rank != 0:
        return None
    ids_n = out.partition_ids.cpu().numpy()
    vals_n = out.values.cpu().numpy()
    one = pdp.ColumnarData(pid=torch.cat([p[0] for p in parts]),
                           pk=torch.cat([p[1] for p in parts]),
                           value=torch.cat([p[2] for p in parts]), n_partitions=P,
                           privacy_id_range=(0, world * args.pids), record_id_offset=0)
    del parts
    acc1 = pdp.NaiveBudgetAccountant(1.0, 1e-6)
    res1 = pdp.DPEngine(acc1, pdp.MI355XBackend(device=dev.index, seed=0xD1FF5EED)).aggregate(
        one, params, ex, public_partitions=public)
    acc1.compute_budgets()
    res1.nonce = nonce
    out1 = res1.materialize()
    ids_1 = out1.partition_ids.cpu().numpy()
    vals_1 = out1.values.cpu().numpy()
    same_set = bool(np.array_equal(np.sort(ids_n), np.sort(ids_1)))
    exact_cols = close_cols = False
    if same_set:
        o, o1 = np.argsort(ids_n), np.argsort(ids_1)
        fields = list(res1.plan.fields)
        ints = [j for j, f in enumerate(fields) if f in ("count", "privacy_id_count")]
        exact_cols = bool(np.array_equal(vals_n[o][:, ints], vals_1[o1][:, ints]))
        close_cols = bool(np.allclose(vals_n[o], vals_1[o1], rtol=1e-9, atol=1e-6))
    return {"records": int(one.pid.numel()), "records_per_rank": int(m),
            "kept_n_rank": int(len(ids_n)), "kept_one_rank": int(len(ids_1)),
            "same_kept_set": same_set, "integer_columns_equal": exact_cols,
            "all_columns_close": close_cols}


if __name__ == "__main__":
    main()
