# round-3 session checkpoint: the N-rank bench launcher tests, then the default bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_multirank.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3_ranks.log 2>&1 || { echo ranks failed; grep -E "^E |FAILED|Error" gpurun_out/r3_ranks.log | head -30; tail -5 gpurun_out/r3_ranks.log; exit 1; }
tail -2 gpurun_out/r3_ranks.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_base_bench.json 2> gpurun_out/r3_base_bench.err || { echo bench failed; tail -20 gpurun_out/r3_base_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3_base_bench.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4)); print({k: v['ms'] for k, v in d['kernels'].items()})"
