#!/bin/bash
# Envelope evidence: the envelope tests and the parity
# suites that cover the partition paths, then builder-run bench lines at
# (N = 2e9, U = 2e7) and (N = 1e9, U = 1e6) beside the default config-2 line.
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-env}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_envelope.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline"
$B > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
$B --records 1000000000 --pids 1000000 > $O/bench_u1e6.json 2> $O/bench_u1e6.err || { tail -5 $O/bench_u1e6.err; exit 1; }
$B --records 2000000000 --pids 20000000 > $O/bench_n2e9.json 2> $O/bench_n2e9.err || { tail -5 $O/bench_n2e9.err; exit 1; }
python3 - <<PY
import json
for n in ("bench_c2", "bench_u1e6", "bench_n2e9"):
    d = json.load(open("$O/%s.json" % n))
    k = {a: round(b["ms"], 2) for a, b in d["kernels"].items() if b["ms"] >= 0.1}
    print(n, d["config"]["records_per_gpu"], d["config"]["privacy_ids_per_gpu"], round(d["ms_per_step"], 2),
          "ns/record %.3f" % (d["ms_per_step"] * 1e6 / d["config"]["records_per_gpu"]), k)
PY
# same-box A/B: the 2048-digit piece level as two 512-thread workgroups per CU
if [ -n "$AB_HALF" ]; then
  STEPS=5 TAG=$T/ab VARIANTS="one:DPG_PC_HALF=0 half:DPG_PC_HALF=1" bash tools/gpu_env_ab.sh || exit 1
fi
