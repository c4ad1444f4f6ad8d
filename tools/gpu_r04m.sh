#!/bin/bash
# round 4: wide-K multisection A/B, K = 140 stages, BASELINE configurations, in-HBM job
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04m; mkdir -p $O; export TMPDIR=/tmp
step() { local rc=$1; case $rc in 124|137|134|139) echo "fatal rc $rc"; exit $rc;; esac; }
timeout -k 10 300 python tools/wide_bias_ab.py > $O/wide_bias_ab.jsonl 2>&1; rc=$?; tail -4 $O/wide_bias_ab.jsonl | cut -c1-700; step $rc
timeout -k 10 300 python tools/risk_stages.py --P 123 --Q 16 --stocks 5000 --dates 252 --reps 2 > $O/risk_stages_k140.log 2>&1; rc=$?; tail -2 $O/risk_stages_k140.log | cut -c1-500; step $rc
timeout -k 10 400 python tools/baseline_configs.py > $O/baseline_configs.log 2>&1; rc=$?; tail -8 $O/baseline_configs.log | cut -c1-300; step $rc
timeout -k 10 300 python tools/pipeline_e2e.py > $O/pipeline_e2e.log 2>&1; rc=$?; tail -2 $O/pipeline_e2e.log | cut -c1-400; exit $rc
