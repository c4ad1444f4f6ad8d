#!/bin/bash
# round 5: kernel trace of the in-HBM e2e job (6 runs of tools/pipeline_e2e.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05aa; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/e2e -o run -- python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/e2e -name '*.db' | head -1) --runs 7 --top 40 > $O/e2e_kernel_stats.txt 2>&1 \
 && rm -rf $O/e2e
rc=$?; head -25 $O/e2e_kernel_stats.txt | cut -c1-160; exit $rc
