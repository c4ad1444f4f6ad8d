#!/bin/bash
# round 4: resident CS-WLS kernel -- phase stamps and geometry A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_xs_resident.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
MODES=30,32,33,34,35 timeout -k 10 200 python tools/xs_resident_phases.py > $O/phases.jsonl 2>&1; rc=$?
cat $O/phases.jsonl
case $rc in 124|137|134|139) exit $rc;; esac
MODES=31,30,32,33,34,35 DATES=2520 DTYPES=fp64 timeout -k 10 300 python tools/xs_mode_time.py > $O/mode_ab.jsonl 2>&1; rc2=$?
cat $O/mode_ab.jsonl | tail -3; exit $(( rc | rc2 ))
