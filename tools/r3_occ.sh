# round-3: occupancy sensitivity of the small-chunk bounding kernels (waves
# per CU 4 vs 8), config 2, same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
run() {  # name, env assignments
  env $2 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/occ/$1.json 2> gpurun_out/occ/$1.err || { echo "$1 failed"; tail -5 gpurun_out/occ/$1.err; exit 1; }
}
run sort8 "X=1"
run sort4 "DPG_DEBUG_WPC=4"
run hash8 "DPG_BOUND_HASH=1"
run hash4 "DPG_BOUND_HASH=1 DPG_DEBUG_WPC=4"
run sort8b "X=1"
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/occ/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2),
          {k: round(v, 2) for k, v in st.items() if v >= 0.3})
PY
