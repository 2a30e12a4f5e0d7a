# round-3 iteration check: GPU parity of the bounding paths, then the config-2
# bench (and config 4 when ITER_C4=1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/iter
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/iter/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/iter/parity.log | head -30; tail -5 gpurun_out/iter/parity.log; exit 1; }
tail -1 gpurun_out/iter/parity.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/iter/c2.json 2> gpurun_out/iter/c2.err || { echo bench failed; tail -20 gpurun_out/iter/c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/iter/c2.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4)); print({k: v['ms'] for k, v in d['kernels'].items()})"
if [ "${ITER_C4:-0}" = 1 ]; then
timeout -k 10 300 python bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/iter/c4.json 2> gpurun_out/iter/c4.err || { echo bench c4 failed; tail -20 gpurun_out/iter/c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/iter/c4.json')); print('c4 ms', round(d['ms_per_step'],2)); print({k: v['ms'] for k, v in d['kernels'].items()})"
fi
