# round-3: grouped XCD-local partition levels A/B (config 2, same box) + parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/grp
DPG_L1_GRP=1 DPG_L2_GRP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/grp/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/grp/parity.log | head -30; tail -5 gpurun_out/grp/parity.log; exit 1; }
tail -1 gpurun_out/grp/parity.log
run() {  # name, env assignments
  env $2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/grp/$1.json 2> gpurun_out/grp/$1.err || { echo "$1 failed"; tail -5 gpurun_out/grp/$1.err; exit 1; }
}
for i in 1 2; do
run base_$i "X=1"
run l1x_$i "DPG_L1_XCD=1"
run g1_$i "DPG_L1_GRP=1"
run g2_$i "DPG_L2_GRP=1"
run g12_$i "DPG_L1_GRP=1 DPG_L2_GRP=1"
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/grp/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("partition1:hist", "partition1:scatter", "partition2:hist", "partition2:scatter", "bound")))
PY
