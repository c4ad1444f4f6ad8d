#!/bin/bash
# round 4: bias solver mode 18 (the no-op steps s >= K-2 skip the Householder update with a
# uniform branch: no per-read fallback-row select) -- bitwise checks, then the timed A/B vs mode 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zc; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "padded or agree" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
MODES=5,18,5,18,5,18 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_sk_ab.jsonl 2>&1; rc2=$?
grep '"mode"' $O/bias_sk_ab.jsonl | cut -c1-200; exit $(( rc | rc2 ))
