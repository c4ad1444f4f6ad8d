#!/bin/bash
# round 4: resident CS-WLS kernel -- moments-phase ablations (atomics / Gram FMAs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04t; mkdir -p $O; export TMPDIR=/tmp
MODES=30,36,37,38 timeout -k 10 200 python tools/xs_resident_phases.py > $O/phases_ablation.jsonl 2>&1; rc=$?
cat $O/phases_ablation.jsonl; exit $rc
