#!/bin/bash
# Round-5 experiment 16: config 5 after the positional report construction
# (bench line + host split), and a rocprofv3 kernel trace of the sweep's
# kernels (the two select passes separately).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5r
mkdir -p $O
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5 ms', round(d['ms_per_step'],2))"
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua_timing failed; tail -5 $O/ua_timing.log; exit 1; }
tail -2 $O/ua_timing.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt5 -o run -- python3 $R/bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > $O/kt5_bench.json 2> $O/kt5.err || { echo kt failed; tail -20 $O/kt5.err; exit 1; }
cd $R
python3 tools/kstats.py $O/kt5/run_kernel_stats.csv 2>/dev/null | head -30 || head -30 $O/kt5/run_kernel_stats.csv | cut -c1-160
