#!/bin/bash
# key-only multi-wave sort: parity, config-4 and config-2 lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lex
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python -u bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo c4 failed; tail -5 $O/c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo c2 failed; tail -5 $O/c2.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c4", "c2"):
    d = json.load(open(f"gpurun_out/lex/{f}.json"))
    print(f, round(d["ms_per_step"], 2), {k: round(v["ms"], 2) for k, v in d["kernels"].items() if v["ms"] > 0.3})
PY
