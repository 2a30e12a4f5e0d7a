#!/bin/bash
# config-4 bench lines (MEAN+VARIANCE, Gaussian, Pareto pids, 1e8 partitions)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --workload config4 --records 200000000 --pids 2000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_small.json 2> gpurun_out/c4_small.err || { echo small failed; tail -20 gpurun_out/c4_small.err; exit 1; }
cat gpurun_out/c4_small.json
timeout -k 10 400 python bench.py --workload config4 --steps 3 --warmup 1 > gpurun_out/c4_private.json 2> gpurun_out/c4_private.err || { echo private failed; tail -20 gpurun_out/c4_private.err; exit 1; }
cat gpurun_out/c4_private.json
timeout -k 10 300 python bench.py --workload config4 --public --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_public.json 2> gpurun_out/c4_public.err || { echo public failed; tail -20 gpurun_out/c4_public.err; exit 1; }
cat gpurun_out/c4_public.json
