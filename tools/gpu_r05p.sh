#!/bin/bash
# round 5: phase ablations of the production bias kernel (eps ||T|| tolerance): 61 = no Laguerre,
# 62 = no eigenvectors / back-transform, 64 = no tridiagonalisation (A/B library, timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05p; mkdir -p $O; export TMPDIR=/tmp
export MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so
MODES=5,61,62,64 ROUNDS=3 timeout -k 10 400 python tools/bias_chain_ab.py > $O/bias_phase_ablation.jsonl 2>&1
rc=$?; tail -4 $O/bias_phase_ablation.jsonl | cut -c1-300; exit $rc
