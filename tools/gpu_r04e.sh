#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04e; mkdir -p $O; export TMPDIR=/tmp
MFA_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py > $O/pipeline_dist4_gloo.log 2>&1
rc=$?; grep -v "socket.cpp\|amdgpu.ids" $O/pipeline_dist4_gloo.log | tail -4; exit $rc
