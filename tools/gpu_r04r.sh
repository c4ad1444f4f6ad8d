#!/bin/bash
# round 4: resident fused CS-WLS kernel (mode 30) -- numerics vs the oracle / DMA kernel, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_xs_resident.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|Mismatch|Greatest" $O/pytest.log | cut -c1-200 | tail -30
case $rc in 124|137|134|139) exit $rc;; esac
MODES=31,30 DATES=315,2520 DTYPES=fp64 timeout -k 10 300 python tools/xs_mode_time.py > $O/mode_ab.jsonl 2>&1; rc2=$?
cat $O/mode_ab.jsonl | tail -5; exit $(( rc | rc2 ))
