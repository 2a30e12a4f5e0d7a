#!/bin/bash
# Grouped-mode partition levels (configs 4 and 5: 12- and 16-byte records):
# the parity suites that cover them, a same-box A/B of configs 4 and 5 against
# libdpg_base.so, and a kernel trace of the (N = 1e9, U = 1e6) input.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${TAG:-grp}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_utility.py \
    tests/test_gpu_histograms.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_u1e6 -o run -- python3 $R/bench.py --records 1000000000 --pids 1000000 --steps 1 --warmup 1 --no-cpu-baseline > $R/$O/kt_u1e6.json 2> $R/$O/kt_u1e6.err || { echo kt failed; tail -5 $R/$O/kt_u1e6.err; exit 1; }
cd $R
python3 tools/kstats.py $(find $O/kt_u1e6 -name "*kernel_stats.csv" | head -1) 12
STEPS=3 TAG=$T/c4 BENCH_ARGS="--workload config4" VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
STEPS=3 TAG=$T/c5 BENCH_ARGS="--workload config5" VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
STEPS=5 TAG=$T/c2 VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
