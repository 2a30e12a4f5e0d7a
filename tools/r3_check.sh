# round-3 check: GPU parity tests (sort kernel first), the N-rank bench tests, smoke, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3_parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/r3_parity.log | head -30; tail -5 gpurun_out/r3_parity.log; exit 1; }
tail -1 gpurun_out/r3_parity.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_gpu_parity.py > gpurun_out/r3_gpu.log 2>&1 || { echo gpu tests failed; grep -E "^E |FAILED|Error" gpurun_out/r3_gpu.log | head -30; tail -5 gpurun_out/r3_gpu.log; exit 1; }
tail -1 gpurun_out/r3_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { echo bench failed; tail -20 gpurun_out/r3_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3_bench.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4)); print({k: v['ms'] for k, v in d['kernels'].items()})"
DPG_BOUND_HASH=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3_bench_hash.json 2> gpurun_out/r3_bench_hash.err || { echo bench hash failed; tail -20 gpurun_out/r3_bench_hash.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3_bench_hash.json')); print('c2 hash ms', round(d['ms_per_step'],2)); print({k: v['ms'] for k, v in d['kernels'].items()})"
