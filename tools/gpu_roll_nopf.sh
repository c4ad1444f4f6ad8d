#!/bin/bash
# Check of the 4-wave EW window default: full GPU test suite, rolling A/B, end-to-end job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/roll_nopf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1 && cat $O/rolling_ab.jsonl \
 && timeout -k 10 300 python tools/pipeline_e2e.py > $O/pipeline_e2e.log 2>&1 && tail -2 $O/pipeline_e2e.log
