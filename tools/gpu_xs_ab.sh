#!/bin/bash
# GPU session: CS-WLS kernel tests + fused-kernel ablation + phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_xs_wls.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_xs.log 2>&1 \
 && tail -2 $OUT/pytest_xs.log \
 && VARIANTS=${VARIANTS:-0,4,8,12} timeout -k 10 200 python -u tools/xs_ablate.py > $OUT/abl.log 2>&1 && cat $OUT/abl.log \
 && timeout -k 10 200 python -u tools/xs_fused_stamps.py > $OUT/fst.log 2>&1 && cat $OUT/fst.log \
 && SORT=${SORT:-0} timeout -k 10 200 python -u tools/xs_modes.py > $OUT/xs_modes.log 2>&1 && cat $OUT/xs_modes.log
