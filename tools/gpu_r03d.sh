#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attribution.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c/pytest_attr.log 2>&1; rc=$?
tail -2 gpurun_out/c/pytest_attr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attr_prof.py > gpurun_out/c/attr_prof.json 2>gpurun_out/c/attr_prof.err; rc=$?
cat gpurun_out/c/attr_prof.json; exit $rc
