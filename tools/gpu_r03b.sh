#!/bin/bash
# Attribution tests + risk stages + bias-solver occupancy A/B (modes 5/6/7) + kernel trace of RiskModel.run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_attr.sh || exit $?
SETTINGS=1e-15:30 MODES=5,6,7 timeout -k 10 300 python -u tools/eigen_tol.py > gpurun_out/attr/wpe.jsonl 2>&1 || { tail gpurun_out/attr/wpe.jsonl; exit 1; }
grep '"mode"' gpurun_out/attr/wpe.jsonl
bash tools/prof_kernels.sh risk_run python3 tools/risk_stages.py --reps 1 && cat gpurun_out/risk_run_stats.txt
timeout -k 10 400 python -u tools/pipeline_e2e.py 5000 2520 > gpurun_out/pipeline_e2e.jsonl 2>gpurun_out/pipeline_e2e.err; rc=$?
cat gpurun_out/pipeline_e2e.jsonl; exit $rc
