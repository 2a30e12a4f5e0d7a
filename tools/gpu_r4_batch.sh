#!/bin/bash
# Round-4 checkpoint: config-2 level-path parity tests, same-box A/B of the
# histogram-free level 1 (pieces vs DPG_L1_PIECES=0, alternating twice), then
# the k_bound_sorted fetch split (tools/gpu_fetch_split.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k config2 > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/c2_pc_$i.json 2> $O/c2_pc_$i.err || { echo c2 failed; tail -5 $O/c2_pc_$i.err; exit 1; }
  DPG_L1_PIECES=0 timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/c2_nopc_$i.json 2> $O/c2_nopc_$i.err || { echo c2 nopc failed; tail -5 $O/c2_nopc_$i.err; exit 1; }
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/r4h/*.json")):
    d = json.load(open(f))
    st = d.get("stage_ms") or {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2),
          {k: round(v, 2) for k, v in st.items() if v >= 0.3})
PY
bash tools/gpu_fetch_split.sh > $O/split.log 2>&1 || { echo split failed; tail -20 $O/split.log; exit 1; }
tail -30 $O/split.log
