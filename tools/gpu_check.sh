#!/bin/bash
# One GPU-box session: kernel tests, smoke, 1-GPU bench and a rocprofv3 kernel-stats profile.
# Every GPU step has its own time limit and the steps are chained with && (stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-30}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 \
 && tail -3 $OUT/pytest_gpu.log \
 && timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log \
 && timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --check > $OUT/bench.log 2>&1 && cat $OUT/bench.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $OUT/prof.log 2>&1 \
 && find $OUT/prof -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-220
