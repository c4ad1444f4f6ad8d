#!/bin/bash
# RiskModel.run-only kernel trace with the current bias default (K = 42, 2520 dates)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r05an; mkdir -p $O
timeout -k 10 120 python tools/risk_run_only.py --make /tmp/panel.pt > $O/make_panel.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/riskrun -o run -- python tools/risk_run_only.py --load /tmp/panel.pt > $O/risk_run_only.log 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/riskrun -name '*.db' | head -1) --runs 3 --top 14 > $O/risk_run_only_kernel_stats.txt 2>&1 \
 && cat $O/risk_run_only_kernel_stats.txt && tail -3 $O/risk_run_only.log && rm -rf $O/riskrun
