# round-3: partition tile-size A/B (config 2, same box): sub-tiles per
# XCD-local tile at level 2, XCD-local level 1 with k sub-tiles per tile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/part
run() {  # name, env assignments
  env $2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/part/$1.json 2> gpurun_out/part/$1.err || { echo "$1 failed"; tail -5 gpurun_out/part/$1.err; exit 1; }
}
for i in 1 2; do
run base_$i "X=1"
run l2s2_$i "DPG_L2_SUBS=2"
run l2s4_$i "DPG_L2_SUBS=4"
run l1x1_$i "DPG_L1_XCD=1 DPG_L1_SUBS=1 DPG_L2_SUBS=2"
run l1x2_$i "DPG_L1_XCD=1 DPG_L1_SUBS=2 DPG_L2_SUBS=2"
run l1x4_$i "DPG_L1_XCD=1 DPG_L1_SUBS=4 DPG_L2_SUBS=2"
run l1x8_$i "DPG_L1_XCD=1 DPG_L1_SUBS=8 DPG_L2_SUBS=2"
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/part/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("partition1:hist", "partition1:scatter", "partition2:hist", "partition2:scatter", "bound")))
PY
