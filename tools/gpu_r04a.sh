#!/bin/bash
# Round-4 check: GPU suite, smoke, bench, 1-GPU in-HBM pipeline, 4-rank gloo rehearsal of the
# date-sharded pipeline on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 200 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log \
 && timeout -k 10 300 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1 && tail -2 $O/pipeline_e2e.jsonl \
 && MFA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py > $O/pipeline_dist4_gloo.log 2>&1 \
 && tail -3 $O/pipeline_dist4_gloo.log
