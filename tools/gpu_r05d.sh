#!/bin/bash
# round 5: cold bias default + rank-invariant sharded descriptors -- the affected GPU suites, perf
# guards (-s, for perf_guards.log), the slowest-rank stand-in, the wide F0-eigh multisection A/B,
# and the 4-rank one-GPU gloo rehearsal of the date-sharded e2e job at 5000 x 2520 (bitwise?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05d; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_eigen.py \
   tests/test_e2e_dist.py tests/test_factor_shard.py tests/test_wide_k.py > $O/pytest.log 2>&1
prc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -8
[ $prc -le 1 ] \
 && $T 300 python -u -m pytest -s -v --timeout 280 --timeout-method thread -m gpu tests/test_perf_regression.py > $O/perf_guards.log 2>&1 \
 ; grc=$?; [ $prc -le 1 ] && [ $grc -le 1 ] \
 && $T 300 python tools/shard_prof.py 5000 2520 8 7 > $O/shard_prof_rank7of8.jsonl 2>&1 \
 && K=140 D=504 $T 300 python tools/wide_eigh_rounds_ab.py > $O/wide_eigh_rounds_ab.jsonl 2>&1 \
 && MFA_DIST_BACKEND=gloo $T 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
      --master-addr 127.0.0.1 --master-port 29517 tools/pipeline_dist.py 5000 2520 > $O/pipeline_dist4_gloo.log 2>&1
rc=$?; [ $prc -le 1 ] || rc=$prc; tail -2 $O/perf_guards.log; tail -1 $O/wide_eigh_rounds_ab.jsonl
grep -h non_io $O/shard_prof_rank7of8.jsonl | tail -2 | cut -c1-400; grep -h "vs_one_process\|rep" $O/pipeline_dist4_gloo.log | tail -3 | cut -c1-600; exit $rc
