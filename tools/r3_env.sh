#!/bin/bash
# env-only same-box config-2 A/B: sort candidate multiplier, bucket target
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/env
mkdir -p $O
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
}
for i in 1 2; do
run base_$i DPG_X=0
run cand125_$i DPG_SORT_CAND_C=1.25
run cand175_$i DPG_SORT_CAND_C=1.75
run tgt192_$i DPG_DEBUG_TARGET=192
run tgt384_$i DPG_DEBUG_TARGET=384
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/env/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st.get(k, 0):.2f}" for k in ("partition1:scatter", "partition2:hist", "partition2:scatter", "chunks", "bound", "bound.wide", "bound.medium")))
PY
