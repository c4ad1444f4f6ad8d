#!/bin/bash
# Eigen stage: GPU tests, bias-solver phase ablations (mode 5 and 61..67), risk-model stages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/eig; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/eig/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/eig/pytest.log; [ $rc -ne 0 ] && exit $rc
SETTINGS=1e-15:30 MODES=${MODES:-5,61,62,64,63,67} timeout -k 10 300 python -u tools/eigen_tol.py > gpurun_out/eig/phases.jsonl 2>&1 || { tail gpurun_out/eig/phases.jsonl; exit 1; }
grep '"mode"' gpurun_out/eig/phases.jsonl
timeout -k 10 300 python -u tools/risk_stages.py --attribution > gpurun_out/eig/risk_ref.json 2>gpurun_out/eig/risk_ref.err && cat gpurun_out/eig/risk_ref.json
