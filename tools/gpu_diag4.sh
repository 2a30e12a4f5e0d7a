#!/bin/bash
export TMPDIR=/tmp
export DPG_WATCHDOG_S=20
run() { echo "== $*"; timeout -k 5 120 python tools/diag_levels.py "$@" || { echo "FAILED rc=$? on $*"; exit 1; }; }
run 20000 2000 500 1024 64 check
run 200000 2000 5000 1024 64 check
run 2000000 20000 50000 1024 2048 check
run 4000000 40000 100000 64 2048 check
run 20000000 200000 1000000 1024 2048
run 100000000 1000000 1000000 1024 2048
