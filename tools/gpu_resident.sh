#!/bin/bash
# Fusion bound (tools/gpu_resident.sh): the bounding kernel's time per record
# when its input -- the team level 2's output, written just before -- still
# sits in the 256 MB Infinity Cache (N = 3e7 records of 8 bytes: 240 MB)
# against inputs that cannot (1e8: 800 MB; 1e9: 8 GB), at config 2's 100
# records per privacy id.  Same box, two runs each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-r6q}
mkdir -p gpurun_out/$T
for i in 1 2; do
for w in "n3e7:30000000:300000" "n1e8:100000000:1000000" "n1e9:1000000000:10000000"; do
  nm=${w%%:*}; r=${w#*:}; n=${r%%:*}; u=${r#*:}
  timeout -k 10 300 python -u bench.py --records $n --pids $u --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$T/${nm}_$i.json 2> gpurun_out/$T/${nm}_$i.err || { echo "$nm failed"; tail -5 gpurun_out/$T/${nm}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/$T/${nm}_$i.json')); k={a:b['ms'] for a,b in d['kernels'].items()}; s=1e9/$n
print('${nm}_$i', 'step', round(d['ms_per_step']*s,2), 'per-1e9 ms: pieces', round(k.get('partition1:pieces',0)*s,2), 'team', round(k.get('partition2:team',0)*s,2), 'bound', round(k.get('bound',0)*s,2), 'items', round((k.get('items:hist',0)+k.get('items:scatter',0))*s,2))"
done
done
