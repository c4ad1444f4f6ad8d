#!/bin/bash
# round 5: the production library with the date-chained bias default -- the whole GPU suite,
# the slowest-rank stand-in of the host-sharded e2e job, RiskModel.run-only trace, bias A/B,
# in-HBM e2e (rank-invariant vs tile descriptors), every BASELINE config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05c; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
prc=$?; tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -8
# test failures (1) do not stop the measurements; a timeout / crash / fault does
[ $prc -le 1 ] \
 && $T 300 python tools/shard_prof.py 5000 2520 8 7 > $O/shard_prof_rank7of8.jsonl 2>&1 \
 && $T 120 python tools/risk_run_only.py --make /tmp/panel.pt > $O/make_panel.log 2>&1 \
 && $T 240 rocprofv3 --kernel-trace --stats -d $O/riskrun -o run -- python tools/risk_run_only.py --load /tmp/panel.pt > $O/risk_run_only.log 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/riskrun -name '*.db' | head -1) --runs 3 --top 12 > $O/risk_run_only_kernel_stats.txt 2>&1 \
 && rm -rf $O/riskrun \
 && MODES=5,21 ROUNDS=4 $T 300 python tools/bias_chain_ab.py > $O/bias_chain_ab.jsonl 2>&1 \
 && $T 400 python tools/pipeline_e2e.py > $O/pipeline_e2e.jsonl 2>&1 \
 && $T 600 python tools/baseline_configs.py > $O/baseline_configs.json 2>&1
rc=$?; [ $prc -le 1 ] || rc=$prc; tail -1 $O/bias_chain_ab.jsonl; grep non_io $O/shard_prof_rank7of8.jsonl | tail -2; tail -4 $O/pipeline_e2e.jsonl | cut -c1-300; exit $rc
