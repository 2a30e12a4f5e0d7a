# round-3: scatter cross-tile prefetch and level-2 records-per-thread A/B
# (config 2, same box) + parity of the default library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu -rA --timeout 300 --timeout-method thread > gpurun_out/pf/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/pf/parity.log | head -30; tail -5 gpurun_out/pf/parity.log; exit 1; }
tail -1 gpurun_out/pf/parity.log
run() {  # name, lib
  DPG_LIB_PATH=pipelinedp_amd/lib/$2 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/pf/$1.json 2> gpurun_out/pf/$1.err || { echo "$1 failed"; tail -5 gpurun_out/pf/$1.err; exit 1; }
}
for i in 1 2; do
run base_$i libdpg.so
run nopf_$i libdpg_nopf.so
run ln12_$i libdpg_ln12.so
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/pf/*.json")):
    d = json.load(open(f))
    st = {k: v["ms"] for k, v in d["kernels"].items()}
    print(os.path.basename(f)[:-5], round(d["ms_per_step"], 2), " ".join(f"{k}={st[k]:.2f}" for k in ("partition1:hist", "partition1:scatter", "partition2:hist", "partition2:scatter", "bound")))
PY
