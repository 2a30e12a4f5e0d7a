#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 5 90 python tools/diag_levels.py "$@" || { echo "FAILED rc=$? on $*"; exit 1; }; }
run 200000 20000 5000 1024 2048 check
run 200000 20000 5000 64 2048 check
run 200000 20000 5000 8 2048 check
run 2000000 20000 50000 1024 2048 check
run 4000000 40000 100000 1024 2048 check
run 20000000 200000 1000000 1024 2048
