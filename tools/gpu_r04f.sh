#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_newey_west.py tests/test_time_scan.py tests/test_e2e.py tests/test_wide_k.py tests/test_eigen.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
MFA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py > $O/pipeline_dist2_gloo.log 2>&1
rc=$?; grep -v "socket.cpp\|amdgpu.ids" $O/pipeline_dist2_gloo.log | tail -2 | cut -c1-700; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python tools/wide_eigh_probe.py > $O/wide_eigh_probe.jsonl 2>&1; rc=$?; tail -3 $O/wide_eigh_probe.jsonl; exit $rc
