#!/bin/bash
# round 5 opening run: 1-GPU bench, RiskModel.run-only kernel trace with the current bias default,
# the resident CS-WLS stream ablations (modes 36/37/38 vs 30) and rolling variant 12's A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r05a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log \
 && timeout -k 10 120 python tools/risk_run_only.py --make /tmp/panel.pt > $O/make_panel.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/riskrun -o run -- python tools/risk_run_only.py --load /tmp/panel.pt > $O/risk_run_only.log 2>&1 \
 && python3 tools/rocpd_stats.py $(find $O/riskrun -name '*.db' | head -1) --runs 3 --top 12 > $O/risk_run_only_kernel_stats.txt 2>&1 \
 && rm -rf $O/riskrun \
 && MODES=30,36,37,38,34 timeout -k 10 240 python tools/xs_resident_phases.py > $O/resident_phases.jsonl 2>&1 \
 && timeout -k 10 300 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1 \
 && timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_wide_k.py tests/test_xs_wls.py > $O/pytest_wide_xs.log 2>&1
rc=$?; head -16 $O/risk_run_only_kernel_stats.txt 2>/dev/null | cut -c1-150; cat $O/resident_phases.jsonl; tail -5 $O/pytest_wide_xs.log; exit $rc
