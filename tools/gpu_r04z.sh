#!/bin/bash
# round 4: bias solver with the padded, mask-free eigenvector phase (mode 14): eigen GPU tests
# (mode 14 bitwise mode 5), then the timed A/B against mode 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04z; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eigen.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
MODES=5,14,5,14 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_pad_ab.jsonl 2>&1; rc2=$?
grep '"mode"' $O/bias_pad_ab.jsonl | cut -c1-300; exit $(( rc | rc2 ))
