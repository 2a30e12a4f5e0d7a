#!/bin/bash
# level-2 digits beside the level-1 records (DPG_L2_AUX): parity of the
# partition tests, same-box config-2 A/B; phase cycles at config 4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/aux
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" $O/parity.log | head -30; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
}
run aux_1 DPG_L2_AUX=1
run noaux_1 DPG_L2_AUX=0
run aux_2 DPG_L2_AUX=1
run noaux_2 DPG_L2_AUX=0
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/aux/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("partition1:hist", "partition1:scatter", "partition2:hist", "partition2:scatter", "bound")))
PY
bash tools/r3_phase.sh
timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py tests/test_gpu_histograms.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ua.log 2>&1 || { echo ua tests failed; grep -E "^E |FAILED|Error" $O/ua.log | head -30; tail -5 $O/ua.log; exit 1; }
tail -1 $O/ua.log
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua timing failed; tail -20 $O/ua_timing.log; exit 1; }
tail -2 $O/ua_timing.log
