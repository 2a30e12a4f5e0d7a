#!/bin/bash
# Level-split / chunk-capacity experiment on the config-2 bench: each line is
# "name env lib", run twice alternately on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env assignments, lib
  env $2 DPG_LIB_PATH=pipelinedp_amd/lib/$3 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/exp_$1_$i.json 2> gpurun_out/exp_$1_$i.err || { echo "$1 failed"; tail -5 gpurun_out/exp_$1_$i.err; exit 1; }
}
for i in 1 2; do
  run base "X=1" libdpg.so
  run b1_10 "DPG_DEBUG_B1=10" libdpg.so
  run t128 "DPG_DEBUG_TARGET=128" libdpg.so
  run w256_t128 "DPG_DEBUG_TARGET=128" libdpg_w256.so
  run w256 "X=1" libdpg_w256.so
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/exp_*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[4:-5], round(d["ms_per_step"], 2),
          {k: round(v, 2) for k, v in st.items() if v >= 0.3})
PY
