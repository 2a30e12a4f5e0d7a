#!/bin/bash
# Round-5 experiment 1: the 1e9-record GPU test alone (with progress), the
# level-1 scatter's phase clocks (timing build), and a same-box A/B of the
# product library against the round-4 base and the variants in $VARIANTS.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
[ -n "$SKIP_FULLSIZE" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -m gpu --timeout 500 --timeout-method thread > $O/fullsize.log 2>&1 || { echo fullsize failed; tail -30 $O/fullsize.log; exit 1; }
[ -n "$SKIP_FULLSIZE" ] || tail -3 $O/fullsize.log
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/phase.json 2> $O/phase.err || { echo phase failed; tail -20 $O/phase.err; exit 1; }
grep "scatter phases" $O/phase.err | tail -4
VARIANTS=${VARIANTS:-"libdpg_base.so libdpg_philox.so"} TAG=r5c/ab bash tools/gpu_ab.sh
