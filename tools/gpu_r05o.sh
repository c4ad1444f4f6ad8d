#!/bin/bash
# round 5: eps ||T|| eigenvalue accuracy in every tridiagonal solver (bias + F0 eigh)
# GPU tests, RiskModel.run kernel traces at K = 42 (2520 dates) and K = 80 / 140 (252 dates)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05o; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_eigen.py \
   tests/test_wide_k.py tests/test_pipeline.py tests/test_determinism.py tests/test_mfm_compat.py tests/test_perf_regression.py > $O/pytest.log 2>&1 \
 && tail -1 $O/pytest.log \
 && $T 120 python tools/risk_run_only.py --make /tmp/panel42.pt > $O/make_k42.log 2>&1 \
 && $T 240 rocprofv3 --kernel-trace --stats -d $O/k42 -o run -- python tools/risk_run_only.py --load /tmp/panel42.pt > $O/risk_k42.log 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/k42 -name '*.db' | head -1) --runs 3 --top 30 > $O/risk_k42_kernel_stats.txt 2>&1 \
 && rm -rf $O/k42 \
 && for K in 80 140; do
      P=$(( K - 17 )); $T 120 python tools/risk_run_only.py --make /tmp/panel$K.pt --dates 252 --P $P --Q 16 > $O/make_k$K.log 2>&1 \
      && $T 240 rocprofv3 --kernel-trace --stats -d $O/k$K -o run -- python tools/risk_run_only.py --load /tmp/panel$K.pt --P $P --Q 16 > $O/risk_k$K.log 2>&1 \
      && python3 tools/rocpd_stats.py $(find $O/k$K -name '*.db' | head -1) --runs 3 --top 30 > $O/risk_k${K}_kernel_stats.txt 2>&1 \
      && rm -rf $O/k$K || exit 1
    done
rc=$?; [ $rc -eq 0 ] && MODES=5,21 ROUNDS=3 timeout -k 10 400 python tools/bias_chain_ab.py > $O/bias_chain_ab.jsonl 2>&1; rc=$?; tail -1 $O/bias_chain_ab.jsonl; tail -1 $O/pytest.log; grep -h "total_ms" $O/risk_k*.log 2>/dev/null; head -4 $O/risk_k*_kernel_stats.txt | cut -c1-150; exit $rc
