#!/bin/bash
# Round-4 evidence: perf guards from the committed guards, a RiskModel.run-only kernel trace,
# K = 140 risk-model stage times, strong-scaling chunk A/B.  A step that times out, aborts or
# faults ends the script (no further GPU step); test failures do not.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04b; mkdir -p $O; export TMPDIR=/tmp
step() {  # step LOG CMD...: run, keep going on ordinary failures, stop on timeout / crash
  local log=$1; shift
  "$@" > "$log" 2>&1; local rc=$?
  tail -2 "$log"
  case $rc in 124|137|134|139) echo "stopping: rc=$rc in $log"; exit $rc;; esac
  return 0
}
step $O/perf_guards.log timeout -k 10 300 python -u -m pytest tests/test_perf_regression.py -m gpu -q -s --timeout 200 --timeout-method thread
step $O/make_panel.log timeout -k 10 120 python tools/risk_run_only.py --make /tmp/panel.pt
step $O/risk_run_only.log timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/riskrun -o run -- python tools/risk_run_only.py --load /tmp/panel.pt
step $O/xs_chunk_ab.jsonl timeout -k 10 300 python tools/xs_chunk_ab.py
step $O/risk_stages_k140.log timeout -k 10 300 python tools/risk_stages.py --P 123 --Q 16 --stocks 5000 --dates 252 --reps 2
step $O/bias_dense_ab.jsonl timeout -k 10 300 env MODES=5,11,61,62,111,112,5,11 SETTINGS=1e-15:30 python tools/eigen_tol.py
MFA_DIST_BACKEND=gloo step $O/pipeline_dist4_gloo.log timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/pipeline_dist.py
