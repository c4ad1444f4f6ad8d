#!/bin/bash
# fp64-storage CS-WLS: kernel tests, 1-GPU bench at both storages, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/xs64
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_xs_wls.py tests/test_mfm_compat.py tests/test_xs_sharded.py tests/test_attribution.py tests/test_pipeline.py tests/test_determinism.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --check > $O/bench_fp64.log 2>&1 && tail -1 $O/bench_fp64.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --storage fp32 > $O/bench_fp32.log 2>&1 && tail -1 $O/bench_fp32.log \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --prewarm 20 > $O/prof.log 2>&1 \
 && find $O/prof -name '*kernel_stats.csv' | head -1 | xargs head -6 | cut -c1-200
