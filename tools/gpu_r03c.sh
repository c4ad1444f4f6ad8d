#!/bin/bash
# Attribution sub-step timings + perf-regression guards (printing their measured numbers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/attr_prof.py > gpurun_out/c/attr_prof.json 2>gpurun_out/c/attr_prof.err; rc=$?
cat gpurun_out/c/attr_prof.json; [ $rc -ne 0 ] && { tail gpurun_out/c/attr_prof.err; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_perf_regression.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/c/perf.log 2>&1; rc=$?
grep -E "ms|reg/s|passed|failed" gpurun_out/c/perf.log | tail -12
timeout -k 10 300 python -u tools/rolling_ab.py > gpurun_out/c/rolling_ab.jsonl 2>&1; rc2=$?
cat gpurun_out/c/rolling_ab.jsonl | grep kernel; exit $((rc | rc2))
