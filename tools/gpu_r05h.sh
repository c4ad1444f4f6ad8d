#!/bin/bash
# round 5: direct rolling kernels with 8-tap batched LDS loads
# BETA / DASTD kernels -- their GPU tests, the sharded-pipeline GPU tests, the slowest-rank
# stand-in (rank 7 of 8 at 5000 x 2520), the in-HBM e2e job with / without rank_invariant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05h; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_factor_engine.py \
   tests/test_factor_shard.py tests/test_e2e_dist.py tests/test_row_index.py > $O/pytest.log 2>&1
prc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -8
[ $prc -le 1 ] && $T 300 python tools/shard_prof.py 5000 2520 8 7 > $O/shard_prof_rank7of8.jsonl 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1
rc=$?; [ $prc -le 1 ] || rc=$prc; grep -h non_io $O/shard_prof_rank7of8.jsonl | tail -2 | cut -c1-500
tail -4 $O/pipeline_e2e.jsonl | cut -c1-420; exit $rc
