#!/bin/bash
# Same-box A/B: the bench with pipelinedp_amd/lib/libdpg.so (a) and each
# variant library in $VARIANTS (files under pipelinedp_amd/lib/), alternating
# twice, so that box-to-box variance cancels.  $BENCH_ARGS selects the
# workload, $TAG prefixes the result files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-libdpg_b.so}
BA=${BENCH_ARGS:-}
T=${TAG:-ab}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $BA > gpurun_out/${T}_a$i.json 2> gpurun_out/${T}_a$i.err || { echo "a failed"; tail -5 gpurun_out/${T}_a$i.err; exit 1; }
  for v in $VARIANTS; do
    DPG_LIB_PATH=pipelinedp_amd/lib/$v timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $BA > gpurun_out/${T}_${v%.so}_$i.json 2> gpurun_out/${T}_${v%.so}_$i.err || { echo "$v failed"; tail -5 gpurun_out/${T}_${v%.so}_$i.err; exit 1; }
  done
done
T=$T python3 - <<'PY'
import glob, json, os
t = os.environ["T"]
for f in sorted(glob.glob(f"gpurun_out/{t}_*.json")):
    d = json.load(open(f))
    st = d.get("stage_ms") or {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[len(t) + 1:-5], round(d["ms_per_step"], 2),
          {k: round(v, 2) for k, v in st.items() if v >= 0.3})
PY
