#!/bin/bash
# round 4: native wide eigh (EIG mode of the two-lanes-per-row solver) -- tests and timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wide_k.py tests/test_eigen.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|Mismatch|Greatest|assert" $O/pytest.log | cut -c1-200 | tail -40
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python tools/wide_bias_ab.py > $O/wide_bias_ab.jsonl 2>&1; rc=$?; tail -3 $O/wide_bias_ab.jsonl; exit $rc
