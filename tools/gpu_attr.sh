#!/bin/bash
# Attribution kernels (incl. the trailing specific-vol kernel) + risk-model stage timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/attr; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attribution.py tests/test_eigen.py tests/test_serving.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/attr/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/attr/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/risk_stages.py --attribution > gpurun_out/attr/risk_ref.json 2>gpurun_out/attr/risk_ref.err && cat gpurun_out/attr/risk_ref.json
