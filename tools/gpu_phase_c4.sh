#!/bin/bash
# Per-phase shader cycles of config 4's bounding kernels (libdpg_timing.so)
# and a kernel trace of one config-4 step.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-c4phase}
mkdir -p gpurun_out/$T
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --workload config4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/$T/phase.json 2> gpurun_out/$T/phase.err || { tail -5 gpurun_out/$T/phase.err; exit 1; }
grep "dpg phase\|\[dpg\]" gpurun_out/$T/phase.err | tail -12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/$T/kt.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/$T/kt.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kstats.py $(find gpurun_out/$T/kt -name "*kernel_stats.csv" | head -1) 24
