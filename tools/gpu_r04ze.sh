#!/bin/bash
# round 4 closing numbers after the bias-solver changes (padded eigenvector phase + skipped
# no-op steps as the default): every BASELINE.json configuration and the perf guards
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04ze; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python tools/baseline_configs.py > $O/baseline_configs.log 2>&1; rc=$?
tail -1 $O/baseline_configs.log | cut -c1-1200
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python -u -m pytest tests/test_perf_regression.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/perf_guards.log 2>&1; rc2=$?
grep -E "ceiling" $O/perf_guards.log | cut -c1-160; exit $(( rc | rc2 ))
