#!/bin/bash
# utility GPU tests, config-5 bench, then level-1 variant A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py tests/test_gpu_histograms.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED|Error" gpurun_out/pytest_ua.log | head -20; tail -3 gpurun_out/pytest_ua.log; exit 1; }
tail -1 gpurun_out/pytest_ua.log
timeout -k 10 400 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo c5 failed; tail -10 gpurun_out/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5.json')); print('c5 ms', round(d['ms_per_step'],1), 'dev', round(d['roofline']['device_ms'],1), {k: round(v,1) for k, v in d['stage_ms'].items() if v > 1})"
VARIANTS="libdpg_a.so libdpg_b.so libdpg_c.so libdpg_d.so" bash tools/gpu_ab.sh > /dev/null
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/ab_*.json')):
    d=json.load(open(f)); k=d['kernels']
    print(f[11:], round(d['ms_per_step'],2), {n: round(k[n]['ms'],2) for n in ('partition1:hist','partition1:scatter','partition2:hist','partition2:scatter','bound')})
PY
