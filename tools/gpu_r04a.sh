#!/bin/bash
# Round-4 check: GPU suite, smoke, bench, 1-GPU in-HBM pipeline, 4-rank gloo rehearsal of the
# date-sharded pipeline on one GPU.  Timeouts / crashes end the script; test failures do not.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
step() {
  local log=$1; shift
  "$@" > "$log" 2>&1; local rc=$?
  tail -3 "$log"
  case $rc in 124|137|134|139) echo "stopping: rc=$rc in $log"; exit $rc;; esac
  return 0
}
step $O/pytest.log timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step $O/smoke.log timeout -k 10 200 python __graft_entry__.py smoke
step $O/bench.log timeout -k 10 200 python bench.py
step $O/pipeline_e2e.jsonl timeout -k 10 240 python tools/pipeline_e2e.py
MFA_DIST_BACKEND=gloo step $O/pipeline_dist4_gloo.log timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py
