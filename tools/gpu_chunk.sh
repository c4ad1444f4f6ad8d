#!/bin/bash
# Chunked (strong-scaling) CS-WLS path: GPU tests, then per-path timings (tools/xs_time.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/chunk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_xs_wls.py tests/test_xs_sharded.py tests/test_determinism.py tests/test_perf_regression.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
OLD_LIB=$PWD/ab_libs/r01_xs.so timeout -k 10 400 python -u tools/xs_time.py > $O/xs_time.jsonl 2> $O/xs_time.err; rc=$?
cat $O/xs_time.jsonl
exit $rc
