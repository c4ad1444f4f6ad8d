#!/bin/bash
# Last check of the committed tree: GPU test suite, smoke, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/last; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 200 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
