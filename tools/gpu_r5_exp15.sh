#!/bin/bash
# Round-5 experiment 15: what a context pays after losing the team level 2
# (a barrier timeout is sticky: later releases take the histogram paths of
# both levels, as DPG_TEAM_L2=0), and the team level 2 over a histogram
# level 1 (DPG_L1_PIECES=0), against the default, config 2.
set -o pipefail
export TMPDIR=/tmp
TAG=r5q/ab STEPS=10 VARIANTS="default:DPG_X=0 hist_l1:DPG_L1_PIECES=0 no_team:DPG_TEAM_L2=0" bash tools/gpu_env_ab.sh
