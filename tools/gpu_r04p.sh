#!/bin/bash
# round 4 evidence: kernel trace of the K = 140 risk model (wide HIP solvers), PMC of the
# round-4 rolling kernels (one A/B round under the counters)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04p; mkdir -p $O; export TMPDIR=/tmp
bash tools/prof_kernels.sh r04p/k140 python3 tools/risk_stages.py --P 123 --Q 16 --stocks 5000 --dates 252 --reps 1 > /dev/null 2>&1; rc=$?
head -12 gpurun_out/r04p/k140_stats.txt; case $rc in 124|137|134|139) exit $rc;; esac
ROUNDS=1 O=$O/pmc bash tools/pmc_roll2.sh > $O/pmc_rolling.txt 2>&1; rc=$?; grep -v "^$" $O/pmc_rolling.txt | cut -c1-240 | tail -16; exit $rc
