#!/bin/bash
# 2-wave medium kernel (variant lib, DPG_MW_M2=1): parity, then same-box config-4 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m2
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_m2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "medium or wide or config4 or exactly" > gpurun_out/m2/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/m2/parity.log | head -30; tail -5 gpurun_out/m2/parity.log; exit 1; }
tail -1 gpurun_out/m2/parity.log
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_m2.so DPG_MW_M2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread -k config4 > gpurun_out/m2/parity_c4.log 2>&1 || { echo parity c4 failed; grep -E "^E |FAILED|Error" gpurun_out/m2/parity_c4.log | head -30; tail -5 gpurun_out/m2/parity_c4.log; exit 1; }
tail -1 gpurun_out/m2/parity_c4.log
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/m2/$nm.json 2> gpurun_out/m2/$nm.err || { echo "$nm failed"; tail -5 gpurun_out/m2/$nm.err; exit 1; }
}
for i in 1 2; do
run base_$i DPG_X=0
run m2_$i DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_m2.so DPG_MW_M2=1
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/m2/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("bound", "bound.wide", "bound.medium", "bound.tail")))
PY
