#!/bin/bash
# round 4: bias solver mode 20 (back-transform steps skipped on tau = 0 alone, padded tau past K:
# no spilled scalar mask per step) -- bitwise checks, then the timed A/B against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "padded or agree" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
MODES=5,20,5,20,5,20 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_bt_ab.jsonl 2>&1; rc2=$?
grep '"mode"' $O/bias_bt_ab.jsonl | cut -c1-200; exit $(( rc | rc2 ))
