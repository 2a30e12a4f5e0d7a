#!/bin/bash
# Round-5 experiment 11: host-side cost per config-2 release (cProfile of
# the timed step; tools/host_profile.py) and a bench line with the stage
# reads moved out of the timed loop.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 400 python -u tools/host_profile.py 1000000000 5 > $O/host_profile.log 2>&1 || { echo host_profile failed; tail -20 $O/host_profile.log; exit 1; }
head -8 $O/host_profile.log
grep -A30 "Ordered by" $O/host_profile.log | head -34
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); print('c2 ms', round(d['ms_per_step'],2), 'dev', round(d['roofline']['device_ms'],3))"
