#!/bin/bash
# Check of the fp64 residual prefetch default: CS-WLS / determinism GPU tests, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/pre64b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xs_wls.py tests/test_determinism.py tests/test_perf_regression.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --check > $O/bench_fp64.log 2>&1 && tail -1 $O/bench_fp64.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --storage fp32 > $O/bench_fp32.log 2>&1 && tail -1 $O/bench_fp32.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --dates 1260 > $O/bench_fp64_d1260.log 2>&1 && tail -1 $O/bench_fp64_d1260.log
