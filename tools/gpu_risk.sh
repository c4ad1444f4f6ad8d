#!/bin/bash
# GPU session: eigen/attribution kernel tests + risk-model stage timings (reference, bootstrap10k).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py tests/test_attribution.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_risk.log 2>&1 \
 && tail -2 gpurun_out/pytest_risk.log \
 && timeout -k 10 300 python -u tools/risk_stages.py --attribution > gpurun_out/risk_ref.json 2>gpurun_out/risk_ref.err && cat gpurun_out/risk_ref.json \
 && timeout -k 10 300 python -u tools/risk_stages.py --preset bootstrap10k --attribution --reps 1 > gpurun_out/risk_10k.json 2>gpurun_out/risk_10k.err && cat gpurun_out/risk_10k.json
