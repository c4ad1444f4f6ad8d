#!/bin/bash
# round 4: bias solver mode 19 (Newton-refined square root / reciprocals in the Laguerre loop)
# -- agreement tests, then the timed A/B against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zd; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "mode19 or padded or agree" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
MODES=5,19,5,19,5,19 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_fl_ab.jsonl 2>&1; rc2=$?
grep '"mode"' $O/bias_fl_ab.jsonl | cut -c1-200; exit $(( rc | rc2 ))
