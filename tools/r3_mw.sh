#!/bin/bash
# multi-wave sort kernels: parity tests, then same-box config-4 A/B
# (default vs DPG_MW_OFF=1) and a config-2 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mw
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -rA --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() {  # name, env..., args
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
}
run c4_mw_1 DPG_X=0
run c4_off_1 DPG_MW_OFF=1
run c4_mw_2 DPG_X=0
run c4_off_2 DPG_MW_OFF=1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo c2 failed; tail -5 $O/c2.err; exit 1; }
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/mw/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={v:.2f}" for k, v in st.items() if k.startswith("bound") or k in ("reduce",)))
PY
