#!/bin/bash
# round 5: phase ablations of the K = 140 bias solver on the risk model's inputs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05w; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python tools/wide_bias_phases.py > $O/wide_bias_phases.jsonl 2>&1
rc=$?; tail -2 $O/wide_bias_phases.jsonl; exit $rc
