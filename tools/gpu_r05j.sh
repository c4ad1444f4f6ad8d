#!/bin/bash
# round 5: the GPU suite on the A/B library (every variant that left the production build, and
# the tests that skip on the production library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05j; mkdir -p $O; export TMPDIR=/tmp
export MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_ab_lib.log 2>&1
rc=$?; tail -2 $O/pytest_ab_lib.log; grep -E "^FAILED|^ERROR" $O/pytest_ab_lib.log | head -8; exit $rc
