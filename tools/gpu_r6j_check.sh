#!/bin/bash
# After a bounding change: the GPU suites touching medium / oversize buckets,
# then one bench line each of (1e9, 1e6), config 4 and config 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-r6j}
mkdir -p gpurun_out/$T
if [ -z "$SKIP_TESTS" ]; then
TAG=$T TESTS="tests/test_gpu_parity.py tests/test_gpu_envelope.py tests/test_gpu_configs.py" bash tools/gpu_check_ab.sh || exit 1
fi
for w in "u1e6:--records 1000000000 --pids 1000000" "c4:--workload config4" "c2:"; do
  nm=${w%%:*}; args=${w#*:}
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/$T/$nm.json 2> gpurun_out/$T/$nm.err || { echo "$nm failed"; tail -5 gpurun_out/$T/$nm.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/$T/$nm.json')); print('$nm', round(d['ms_per_step'],2), {k: round(v['ms'],2) for k,v in d['kernels'].items() if v['ms']>=0.3})"
done
