#!/bin/bash
# round 4 final tree (bias-solver default changed since r04v, tridiag.h templated): the whole
# GPU suite, smoke and the headline bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zg; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --check > $O/bench_fp64.log 2>&1 && tail -1 $O/bench_fp64.log | cut -c1-300
rc2=$?; exit $(( rc | rc2 ))
