#!/bin/bash
# round 4: bias solver with four accumulators per matvec / dot product (mode 13) vs mode 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04x; mkdir -p $O; export TMPDIR=/tmp
MODES=5,13,5,13 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_acc4_ab.jsonl 2>&1; rc=$?
grep '"mode"' $O/bias_acc4_ab.jsonl | cut -c1-300; exit $rc
