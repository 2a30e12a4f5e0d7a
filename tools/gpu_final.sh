#!/bin/bash
# Round evidence at HEAD, part 1: all GPU tests + smoke, the config-2 bench
# line (with the CPU baseline), configs 4 (private, public) and 5, the
# config-5 host split.  Part 2 (profiles): tools/gpu_final_prof.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'cpu', d.get('cpu_baseline',{}).get('value')); print({k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail -20 $O/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4 ms', round(d['ms_per_step'],2)); print({k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --workload config4 --public --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4p.json 2> $O/bench_c4p.err || { echo c4p failed; tail -20 $O/bench_c4p.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4p.json')); print('c4 public ms', round(d['ms_per_step'],2))"
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5 ms', round(d['ms_per_step'],2), d['stage_ms']); print(d.get('cpu_baseline'))"
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua_timing failed; tail -5 $O/ua_timing.log; exit 1; }
tail -2 $O/ua_timing.log
echo done
