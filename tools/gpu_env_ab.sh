#!/bin/bash
# Same-box A/B over environment knobs (DPG_DEBUG_*, DPG_SORT_*, DPG_LIB_PATH):
# every variant runs the bench twice, alternating, so box-to-box variance
# cancels.  Variants are "name:VAR=val[,VAR=val...]" words in $VARIANTS;
# $BENCH_ARGS selects the workload, $TAG names the result directory.
#   VARIANTS="base:DPG_X=0 cand125:DPG_SORT_CAND_C=1.25" bash tools/gpu_env_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}
mkdir -p $O
VARIANTS=${VARIANTS:-base:DPG_X=0}
for i in 1 2; do
  for v in $VARIANTS; do
    nm=${v%%:*}; kv=${v#*:}
    env ${kv//,/ } timeout -k 10 300 python -u bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/${nm}_$i.json 2> $O/${nm}_$i.err || { echo "$nm failed"; tail -5 $O/${nm}_$i.err; exit 1; }
  done
done
O=$O python3 - <<'PY'
import glob, json, os
o = os.environ["O"]
for f in sorted(glob.glob(f"{o}/*.json")):
    d = json.load(open(f))
    st = d.get("stage_ms") or {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2),
          {k: round(v, 2) for k, v in st.items() if v >= 0.3})
PY
