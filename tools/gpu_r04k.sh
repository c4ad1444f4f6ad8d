#!/bin/bash
# round 4: two-lanes-per-row wide bias solver -- GPU tests and A/B with phase ablations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wide_k.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|Mismatch|Greatest" $O/pytest.log | cut -c1-200 | tail -30
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python tools/wide_bias_ab.py > $O/wide_bias_ab.jsonl 2>&1; rc=$?; cat $O/wide_bias_ab.jsonl | tail -6; exit $rc
