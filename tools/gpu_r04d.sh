#!/bin/bash
# Is the 4-rank gloo rehearsal slow because 4 processes share one GPU?  4 concurrent copies of
# the single-process sharded-exposures profile (no collectives), then a 2-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04d; mkdir -p $O; export TMPDIR=/tmp
PIN=${PIN:-0}
pids=""
for r in 0 1 2 3; do
  MFA_PINNED=$PIN timeout -k 10 300 python -u tools/shard_prof.py 5000 2520 4 $r > $O/shard_prof_4proc_pin${PIN}_r$r.jsonl 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for f in $O/shard_prof_4proc_pin${PIN}_r*.jsonl; do tail -n 1 $f | cut -c1-200; done
case $rc in 124|137|134|139) echo "stopping rc=$rc"; exit $rc;; esac
