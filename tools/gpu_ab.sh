#!/bin/bash
# Same-box A/B: the 1e9 bench with pipelinedp_amd/lib/libdpg.so (a) and each
# variant library in $VARIANTS (files under pipelinedp_amd/lib/), alternating
# twice, so that box-to-box variance cancels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-libdpg_b.so}
BA=${BENCH_ARGS:-}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $BA > gpurun_out/ab_a$i.json 2> gpurun_out/ab_a$i.err || { echo "a failed"; tail -5 gpurun_out/ab_a$i.err; exit 1; }
  for v in $VARIANTS; do
    DPG_LIB_PATH=pipelinedp_amd/lib/$v timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline $BA > gpurun_out/ab_${v%.so}_$i.json 2> gpurun_out/ab_${v%.so}_$i.err || { echo "$v failed"; tail -5 gpurun_out/ab_${v%.so}_$i.err; exit 1; }
  done
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/ab_*.json")):
    d = json.load(open(f))
    st = d.get("stage_ms") or {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[3:-5], round(d["ms_per_step"], 2),
          {k: round(st.get(k, 0), 2) for k in ("partition1:scatter", "partition2:scatter", "bound", "bound.medium", "bound.tail", "heavy")})
PY
