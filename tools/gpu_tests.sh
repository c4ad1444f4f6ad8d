#!/bin/bash
# Run a subset of the GPU test suite: tools/gpu_tests.sh <pytest args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
rc=$?
tail -30 gpurun_out/tests.log
exit $rc
