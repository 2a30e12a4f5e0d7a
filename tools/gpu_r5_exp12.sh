#!/bin/bash
# Round-5 experiment 12: the asynchronous compaction (the kept count read
# when the result is first used, so the host enqueues the next release
# before the previous one finishes) -- GPU tests that read results, then a
# same-box A/B against the synchronising compaction (DPG_SYNC_COMPACT=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_release.py tests/test_gpu_configs.py tests/test_gpu_bench_ranks.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=r5n/ab STEPS=10 VARIANTS="async:DPG_X=0 sync:DPG_SYNC_COMPACT=1" bash tools/gpu_env_ab.sh
