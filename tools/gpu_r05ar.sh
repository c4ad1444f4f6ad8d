#!/bin/bash
# full GPU suite on the A/B library after the bias-solver layout changes (A/B variants vs mode 5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05ar; mkdir -p $O; export TMPDIR=/tmp
MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_ab_lib.log 2>&1
rc=$?; tail -1 $O/pytest_ab_lib.log; grep -hE "^FAILED" $O/*.log | head; exit $rc
