#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04c; mkdir -p $O; export TMPDIR=/tmp
step() {
  local log=$1; shift
  "$@" > "$log" 2>&1; local rc=$?
  tail -4 "$log"
  case $rc in 124|137|134|139) echo "stopping: rc=$rc in $log"; exit $rc;; esac
  return 0
}
step $O/xs_split_ab.jsonl timeout -k 10 200 python tools/xs_split_ab.py
step $O/shard_prof.jsonl timeout -k 10 200 python -u tools/shard_prof.py 5000 2520 4 1
