#!/bin/bash
# parity tests with variant $V, then same-box A/B of $V against the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DPG_LIB_PATH=pipelinedp_amd/lib/$V timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_v.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" gpurun_out/pytest_v.log | head; tail -2 gpurun_out/pytest_v.log; exit 1; }
tail -1 gpurun_out/pytest_v.log
VARIANTS="$V" bash tools/gpu_ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_*.json")):
    d = json.load(open(f)); k = d["kernels"]
    print(f[11:], round(d["ms_per_step"], 2), {n: round(k[n]["ms"], 2) for n in k if k[n]["ms"] > 0.3})
PY
