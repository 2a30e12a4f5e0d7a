#!/bin/bash
# utility accumulate run length (pairs per wave): variant parity + same-box timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/run
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_run16k.so timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/run/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/run/parity.log | head -30; tail -5 gpurun_out/run/parity.log; exit 1; }
tail -1 gpurun_out/run/parity.log
for v in base run4k run16k; do
  if [ $v = base ]; then L=pipelinedp_amd/lib/libdpg.so; else L=pipelinedp_amd/lib/libdpg_$v.so; fi
  DPG_LIB_PATH=$L timeout -k 10 300 python -u tools/ua_timing.py > gpurun_out/run/$v.log 2>&1 || { echo $v failed; tail -5 gpurun_out/run/$v.log; exit 1; }
  echo $v; tail -n 1 gpurun_out/run/$v.log | cut -c1-80; grep -o "'ua.accumulate': [0-9.]*" gpurun_out/run/$v.log | tail -n 2
done
