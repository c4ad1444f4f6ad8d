#!/bin/bash
# Is the 4-rank gloo rehearsal slow because 4 processes share one GPU?  4 concurrent copies of
# the single-process sharded-exposures profile (no collectives), then a 2-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04d; mkdir -p $O; export TMPDIR=/tmp
pids=""
for r in 0 1 2 3; do
  timeout -k 10 300 python -u tools/shard_prof.py 5000 2520 4 $r > $O/shard_prof_4proc_r$r.jsonl 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
tail -2 $O/shard_prof_4proc_r*.jsonl
case $rc in 124|137|134|139) echo "stopping rc=$rc"; exit $rc;; esac
MFA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py > $O/pipeline_dist2_gloo.log 2>&1
tail -5 $O/pipeline_dist2_gloo.log
