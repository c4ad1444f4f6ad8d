#!/bin/bash
# round 5: full GPU suite after the row-index / direct-kernel / aligned-layout changes, the
# slowest-rank stand-in, the in-HBM e2e job with / without rank_invariant, and the 1-GPU bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05i; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
prc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -8
[ $prc -le 1 ] && $T 300 python tools/shard_prof.py 5000 2520 8 7 > $O/shard_prof_rank7of8.jsonl 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1 \
 && $T 300 python bench.py > $O/bench.log 2>&1
rc=$?; [ $prc -le 1 ] || rc=$prc; grep -h non_io $O/shard_prof_rank7of8.jsonl | tail -2 | cut -c1-400
tail -2 $O/pipeline_e2e.jsonl | cut -c1-300; tail -1 $O/bench.log; exit $rc
