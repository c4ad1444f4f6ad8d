#!/bin/bash
# round 4: rolling kernels (tests, guards, A/B) + one-rank RCCL runs of bench.py / the pipeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04i; mkdir -p $O; export TMPDIR=/tmp
step() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_factor_engine.py tests/test_perf_regression.py tests/test_force_pg.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|ms \(ceiling" $O/pytest.log | tail -30; step $rc
timeout -k 10 400 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1; rc=$?; step $rc
MFA_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --steps 30 > $O/bench_rccl_world1.log 2>&1; rc=$?
grep '^{' $O/bench_rccl_world1.log | cut -c1-300; exit $rc
