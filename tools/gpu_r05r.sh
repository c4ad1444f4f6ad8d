#!/bin/bash
# round 5: Sturm-evaluation counts per eigenvalue rank of the bias solver (A/B mode 68)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05r; mkdir -p $O; export TMPDIR=/tmp
export MFA_HIP_LIB=$PWD/llm_driven_multi_factor_model_amd/_lib/ab/libmfa_hip.so
timeout -k 10 300 python tools/bias_sturm_counts.py > $O/bias_sturm_counts.json 2>&1
rc=$?; tail -2 $O/bias_sturm_counts.json | cut -c1-1500; exit $rc
