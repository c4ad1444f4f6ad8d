#!/bin/bash
# round 5: F0 eigh at K = 140 on the risk model's Newey-West covariances -- LAPACK-style absolute
# eigenvalue tolerance vs the 1e-22 ||T|| default (time, errors vs LAPACK)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05l; mkdir -p $O; export TMPDIR=/tmp
ABSTOL=1 K=140 D=252 timeout -k 10 300 python tools/wide_eigh_rounds_ab.py > $O/wide_eigh_abstol_k140.jsonl 2>&1 \
 && ABSTOL=1 K=80 D=252 timeout -k 10 300 python tools/wide_eigh_rounds_ab.py > $O/wide_eigh_abstol_k80.jsonl 2>&1
rc=$?; tail -1 $O/wide_eigh_abstol_k140.jsonl; tail -1 $O/wide_eigh_abstol_k80.jsonl; exit $rc
