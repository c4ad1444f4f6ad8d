#!/bin/bash
# Pipelined team CS-WLS kernel: GPU tests, then timing against the fused kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/team
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xs_wls.py -m gpu -x -q --timeout 120 --timeout-method thread -k "team" > gpurun_out/team/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/team/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/xs_team_time.py > gpurun_out/team/time.jsonl 2>&1; rc=$?
cat gpurun_out/team/time.jsonl; exit $rc
