#!/bin/bash
# round 5: flagged F0 matrices of the K = 42 tridiagonal eigh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05ad; mkdir -p $O; export TMPDIR=/tmp
for sd in 3 0 1234; do SEED=$sd timeout -k 10 200 python tools/eigh_flag_stats.py >> $O/eigh_flag_stats.jsonl 2>&1 || exit 1; done
tail -3 $O/eigh_flag_stats.jsonl
