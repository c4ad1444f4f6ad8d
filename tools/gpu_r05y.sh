#!/bin/bash
# round 5: wide solvers without the end-of-step barrier -- wide-K GPU tests, K = 80 / 140 risk
# model traces, K = 140 phase ablations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05y; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_wide_k.py tests/test_eigen.py > $O/pytest.log 2>&1 \
 && for K in 80 140; do
      P=$(( K - 17 )); $T 120 python tools/risk_run_only.py --make /tmp/panel$K.pt --dates 252 --P $P --Q 16 > $O/make_k$K.log 2>&1 \
      && $T 240 python tools/risk_run_only.py --load /tmp/panel$K.pt --P $P --Q 16 --reps 3 > $O/risk_k$K.log 2>&1 || exit 1
    done \
 && $T 400 python tools/wide_bias_phases.py > $O/wide_bias_phases.jsonl 2>&1
rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; grep -h total_ms $O/risk_k*.log; tail -1 $O/wide_bias_phases.jsonl; exit $rc
