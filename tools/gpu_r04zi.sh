#!/bin/bash
# round 4: RiskModel.run-only kernel trace with the new bias-solver default (the committed trace
# predates the padded eigenvector phase): saved fp64 panel, no generator kernels in the trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zi; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python tools/risk_run_only.py --make /tmp/panel.pt > $O/make_panel.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/riskrun -o run -- python tools/risk_run_only.py --load /tmp/panel.pt > $O/risk_run_only.log 2>&1 \
 && tail -3 $O/risk_run_only.log \
 && python3 tools/rocpd_stats.py $(find $O/riskrun -name '*.db' | head -1) --runs 3 --top 12 > $O/risk_run_only_kernel_stats.txt 2>&1 \
 ; rc=$?; head -16 $O/risk_run_only_kernel_stats.txt 2>/dev/null | cut -c1-150; exit $rc
