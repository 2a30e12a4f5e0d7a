#!/bin/bash
# wave-aggregated ranking threshold (DPG_AGG_BITS): same-box config-2 / 4 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/agg
mkdir -p $O
run() {  # name, args, env...
  local nm=$1; local a=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $a > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
}
for i in 1 2; do
run c2_base_$i "" DPG_X=0
run c2_agg8_$i "" DPG_AGG_BITS=8
run c2_agg11_$i "" DPG_AGG_BITS=11
done
run c4_base_1 "--workload config4" DPG_X=0
run c4_agg8_1 "--workload config4" DPG_AGG_BITS=8
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/agg/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={v:.2f}" for k, v in st.items() if ("hist" in k or "scatter" in k or k == "reduce")))
PY
