#!/bin/bash
# One GPU call: the GPU tests in $TESTS (if set; "-m gpu" selection), then a
# same-box A/B over $VARIANTS (tools/gpu_env_ab.sh: "name:VAR=val[,...]"
# words, each run twice alternating).  $TAG names the outputs under
# gpurun_out/.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
T=${TAG:-chk}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
  tail -3 gpurun_out/${T}_pytest.log
fi
if [ -n "$VARIANTS" ]; then
  TAG=$T bash tools/gpu_env_ab.sh || exit 1
fi
