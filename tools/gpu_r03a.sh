#!/bin/bash
# Round-3 check: team CS-WLS kernel tests + timing, then bias-solver modes 3/4/5 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_team.sh || exit $?
MODES=3,4,5 bash tools/gpu_eigen_ab.sh > gpurun_out/eigen_ab.log 2>&1 || { tail -20 gpurun_out/eigen_ab.log; exit 1; }
grep '"mode"' gpurun_out/eigen_ab.jsonl
