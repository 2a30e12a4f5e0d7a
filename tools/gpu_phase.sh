# Per-phase shader cycles of the bounding kernels (libdpg_timing.so) for the
# config-2 and config-4 workloads.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo phase failed; tail -20 gpurun_out/phase.err; exit 1; }
grep "dpg phase" gpurun_out/phase.err | tail -2
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase_c4.json 2> gpurun_out/phase_c4.err || { echo phase c4 failed; tail -20 gpurun_out/phase_c4.err; exit 1; }
grep "dpg phase" gpurun_out/phase_c4.err | tail -4
