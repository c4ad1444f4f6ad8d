#!/bin/bash
# round 5: CS-WLS suite on both libraries after the mode-7 dispatch fix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_xs_wls.py tests/test_xs_resident.py > $O/pytest_prod.log 2>&1 \
 && MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_xs_wls.py tests/test_xs_resident.py > $O/pytest_ab_lib.log 2>&1
rc=$?; tail -1 $O/pytest_prod.log; tail -1 $O/pytest_ab_lib.log; grep -hE "^FAILED" $O/*.log | head; exit $rc
