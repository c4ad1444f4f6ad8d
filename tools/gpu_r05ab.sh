#!/bin/bash
# round 5: warm-started Jacobi re-solve of flagged F0 matrices -- eigen GPU tests, risk_stages
# kernel trace (eigh_pairs_kernel was 0.54 ms there), e2e kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05ab; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_eigen.py tests/test_wide_k.py tests/test_mfm_compat.py > $O/pytest.log 2>&1 \
 && $T 300 rocprofv3 --kernel-trace --stats -d $O/rs -o run -- python3 tools/risk_stages.py --reps 1 > $O/risk_stages.log 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/rs -name '*.db' | head -1) --top 14 > $O/risk_stages_kernel_stats.txt 2>&1 && rm -rf $O/rs \
 && $T 400 rocprofv3 --kernel-trace --stats -d $O/e2e -o run -- python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/e2e -name '*.db' | head -1) --runs 7 --top 14 > $O/e2e_kernel_stats.txt 2>&1 && rm -rf $O/e2e
rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -5; grep -h "eigh_pairs\|total" $O/*_kernel_stats.txt | cut -c1-150; tail -2 $O/pipeline_e2e.jsonl | cut -c1-250; exit $rc
