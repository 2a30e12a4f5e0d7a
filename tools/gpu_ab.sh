#!/bin/bash
# Same-box A/B: the 1e9 bench with pipelinedp_amd/lib/libdpg.so (A) and
# $LIB_B (B), alternating, so that box-to-box variance cancels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${LIB_B:-pipelinedp_amd/lib/libdpg_b.so}
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_a$i.json 2> gpurun_out/ab_a$i.err || { echo "A failed"; tail -5 gpurun_out/ab_a$i.err; exit 1; }
  DPG_LIB_PATH=$B timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_b$i.json 2> gpurun_out/ab_b$i.err || { echo "B failed"; tail -5 gpurun_out/ab_b$i.err; exit 1; }
done
python3 - <<'PY'
import json
for v in ("a1","b1","a2","b2"):
    d=json.load(open(f"gpurun_out/ab_{v}.json"))
    st=d["stage_ms"]
    print(v, round(d["ms_per_step"],2), {k: round(st[k],2) for k in ("partition1:hist","partition1:scatter","partition2:hist","partition2:scatter","bound")})
PY
