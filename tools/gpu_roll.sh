#!/bin/bash
# Rolling kernels: GPU tests + A/B timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/roll; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_factor_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/roll/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/roll/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/rolling_ab.py > gpurun_out/roll/ab.jsonl 2>&1; rc=$?
grep kernel gpurun_out/roll/ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/baseline_configs.py > gpurun_out/roll/baseline_configs.json 2>gpurun_out/roll/baseline_configs.err; rc=$?
tail -3 gpurun_out/roll/baseline_configs.json; exit $rc
