#!/bin/bash
# round 4: sanitised-row BETA/DASTD kernels -- correctness, A/B timing, PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_factor_engine.py tests/test_perf_regression.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1; rc=$?; cut -c1-400 $O/rolling_ab.jsonl; [ $rc = 0 ] || exit $rc
O=$O/pmc bash tools/pmc_roll2.sh > $O/pmc.txt 2>&1; rc=$?; cat $O/pmc.txt; exit $rc
