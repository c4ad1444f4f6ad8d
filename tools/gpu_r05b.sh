#!/bin/bash
# round 5: production library (A/B variants pruned) -- GPU tests of the changed suites, the
# warm-chain bias A/B, the wide-K RiskModel kernel traces (K = 80 / 140: no rocSOLVER / rocBLAS)
# and the 1-GPU bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05b; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_eigen.py \
   tests/test_wide_k.py tests/test_xs_wls.py tests/test_xs_resident.py tests/test_factor_shard.py \
   tests/test_factor_engine.py tests/test_mfm_compat.py > $O/pytest.log 2>&1 \
 && tail -3 $O/pytest.log \
 && $T 300 python tools/bias_chain_ab.py > $O/bias_chain_ab.jsonl 2>&1 && tail -1 $O/bias_chain_ab.jsonl \
 && for K in 80 140; do
      P=$(( K - 17 )); $T 120 python tools/risk_run_only.py --make /tmp/panel$K.pt --dates 252 --P $P --Q 16 > $O/make_k$K.log 2>&1 \
      && $T 240 rocprofv3 --kernel-trace --stats -d $O/k$K -o run -- python tools/risk_run_only.py --load /tmp/panel$K.pt --P $P --Q 16 > $O/risk_k$K.log 2>&1 \
      && python3 tools/rocpd_stats.py $(find $O/k$K -name '*.db' | head -1) --runs 3 --top 40 > $O/risk_k${K}_kernel_stats.txt 2>&1 \
      && rm -rf $O/k$K || exit 1
    done \
 && $T 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
rc=$?; grep -h "total_ms" $O/risk_k*.log 2>/dev/null; exit $rc
