#!/bin/bash
# comm pack/unpack test + config-5 host/device split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/comm.log 2>&1 || { echo comm failed; grep -E "^E |FAILED|Error" $O/comm.log | head -30; tail -5 $O/comm.log; exit 1; }
tail -1 $O/comm.log
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua failed; tail -20 $O/ua_timing.log; exit 1; }
cat $O/ua_timing.log
