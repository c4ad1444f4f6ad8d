#!/bin/bash
# production bias solver with 2-step Householder groups: tests, risk stages, bench
set -o pipefail
O=gpurun_out/r05ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_eigen.py tests/test_mfm_compat.py tests/test_wide_k.py tests/test_determinism.py tests/test_perf_regression.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/risk_stages.py > $O/risk_stages.log 2>&1 || { tail -20 $O/risk_stages.log; exit 1; }
tail -1 $O/risk_stages.log | cut -c1-400
timeout -k 10 300 python -u tools/baseline_configs.py > $O/baseline_configs.log 2>&1 || { tail -20 $O/baseline_configs.log; exit 1; }
tail -1 $O/baseline_configs.log | cut -c1-900
bash tools/gpu_r05an.sh > /dev/null 2>&1 && cp gpurun_out/r05an/risk_run_only_kernel_stats.txt $O/ && head -8 $O/risk_run_only_kernel_stats.txt
