#!/bin/bash
# level-2 groups per level-1 bucket (DPG_SEG_GROUP records per group): same-box config-2 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/grp2
mkdir -p $O
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/$nm.json 2> $O/$nm.err || { echo "$nm failed"; tail -5 $O/$nm.err; exit 1; }
}
for i in 1 2; do
run base_$i DPG_X=0
run g256k_$i DPG_SEG_GROUP=262144
run g128k_$i DPG_SEG_GROUP=131072
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/grp2/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("partition1:hist", "partition1:scatter", "partition2:hist", "partition2:scatter", "chunks", "bound")))
PY
