#!/bin/bash
# round 4: two-rows-per-lane RSTR scan pass -- tests, guards, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_factor_engine.py tests/test_perf_regression.py tests/test_e2e.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|ms \(ceiling|Mismatch|Greatest" $O/pytest.log | cut -c1-160 | tail -40
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1; rc=$?
grep '"kernel"' $O/rolling_ab.jsonl | cut -c1-600; exit $rc
