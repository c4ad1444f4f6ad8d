#!/bin/bash
# round 5: column-batched scatter / winsorize / gather in the e2e post-processing and RiskPanel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05t; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_e2e.py \
   tests/test_e2e_dist.py tests/test_pipeline.py tests/test_xs_reduce.py tests/test_factor_shard.py > $O/pytest.log 2>&1 \
 && $T 400 python tools/post_prof.py > $O/post_prof.jsonl 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1
rc=$?; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -5; tail -1 $O/post_prof.jsonl | cut -c1-400; tail -2 $O/pipeline_e2e.jsonl | cut -c1-260; exit $rc
