#!/bin/bash
# round 4: padded eigenvector phase as the mode-5 default -- eigen / risk-model GPU tests, perf
# guards, risk stages, BASELINE configurations 2 / 3 / 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04za; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_eigen.py tests/test_distributed.py tests/test_presets.py tests/test_determinism.py tests/test_perf_regression.py tests/test_e2e_dist.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ceiling" $O/pytest.log | cut -c1-200 | tail -14; case $rc in 124|137|134|139) exit $rc;; esac
MODES=14,5,14,5 SETTINGS=1e-15:30 timeout -k 10 400 python tools/eigen_tol.py > $O/bias_pad_default_ab.jsonl 2>&1 && grep '"mode"' $O/bias_pad_default_ab.jsonl | cut -c1-200 \
 && timeout -k 10 400 python tools/baseline_configs.py > $O/baseline_configs.log 2>&1 && tail -1 $O/baseline_configs.log | cut -c1-900
rc2=$?; exit $(( rc | rc2 ))
