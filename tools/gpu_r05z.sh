#!/bin/bash
# round 5: loader-column uploads on a copy stream overlapped with the build / descriptors
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05z; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_e2e.py \
   tests/test_e2e_dist.py tests/test_pipeline.py tests/test_row_index.py tests/test_cli_io.py > $O/pytest.log 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1
timeout -k 10 300 python tools/post_prof.py > $O/post_prof.jsonl 2>&1; rc=$?; tail -1 $O/post_prof.jsonl | cut -c1-400; tail -1 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head -5; tail -4 $O/pipeline_e2e.jsonl | cut -c1-300; exit $rc
