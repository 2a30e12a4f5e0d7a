# round-3: candidate multiplier A/B of the sort kernel (config 2, same box)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cand
run() {  # name, env assignments
  env $2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/cand/$1.json 2> gpurun_out/cand/$1.err || { echo "$1 failed"; tail -5 gpurun_out/cand/$1.err; exit 1; }
}
for i in 1 2; do
run c20_$i "DPG_SORT_CAND_C=2.0"
run c15_$i "DPG_SORT_CAND_C=1.5"
run c125_$i "DPG_SORT_CAND_C=1.25"
run c10_$i "DPG_SORT_CAND_C=1.0"
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/cand/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), "bound", round(st["bound"], 3), "wide", round(st.get("bound.wide", 0), 3))
PY
