#!/bin/bash
# round 5: bias solver with eps ||T|| eigenvalue accuracy (A/B mode 24) vs mode 5, on the
# pipeline's own inputs (A/B library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05n; mkdir -p $O; export TMPDIR=/tmp
export MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so
MODES=5,24 ROUNDS=3 timeout -k 10 400 python tools/bias_chain_ab.py > $O/bias_abstol_ab.jsonl 2>&1
rc=$?; tail -4 $O/bias_abstol_ab.jsonl; exit $rc
