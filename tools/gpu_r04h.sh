#!/bin/bash
# round 4: rolling kernels -- GPU tests + interleaved A/B (no PMC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_factor_engine.py tests/test_perf_regression.py -m gpu -s -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1; rc=$?; exit $rc
