#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/shard_prof.py 5000 2520 4 1 2>&1 | tee $O/shard_prof.jsonl
