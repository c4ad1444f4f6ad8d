#!/bin/bash
# round 5: sub-steps of the e2e job's exposures -> RiskPanel phase
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python tools/post_prof.py > $O/post_prof.jsonl 2>&1
rc=$?; tail -3 $O/post_prof.jsonl | cut -c1-600; exit $rc
