#!/bin/bash
export TMPDIR=/tmp
export DPG_WATCHDOG_S=10
run() { echo "== $*"; timeout -k 5 60 python tools/diag_levels.py "$@"; echo "rc=$?"; }
run 20000 2000 500 1024 64 check
