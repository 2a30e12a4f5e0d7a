#!/bin/bash
# Round-5 experiment 8: the three-pass sort kernel (narrow 128-candidate
# pass at 5 waves per SIMD, mid 256-candidate pass at 4, wide) -- the whole
# GPU suite on it, then same-box A/B against the two-pass build (h) and the
# 128-cap two-pass variant of r5h (v20).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=r5j/ab VARIANTS="new:DPG_X=0 h:DPG_LIB_PATH=$L/libdpg_h.so v20:DPG_LIB_PATH=$L/libdpg_v20.so" bash tools/gpu_env_ab.sh
