#!/bin/bash
# round 5: every BASELINE config and the in-HBM e2e job with the eps-tolerance solvers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05q; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python tools/baseline_configs.py > $O/baseline_configs.json 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1
rc=$?; tail -1 $O/baseline_configs.json | cut -c1-1200; tail -2 $O/pipeline_e2e.jsonl | cut -c1-250; exit $rc
