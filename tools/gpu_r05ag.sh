#!/bin/bash
# register-resident warm re-solve setup: eigen tests, split, flag stats
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_eigen.py tests/test_mfm_compat.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for s in 3 0 1234; do
  SEED=$s timeout -k 10 240 python -u tools/eigh_resolve_split.py >> $O/eigh_resolve_split.jsonl 2>>$O/err.log || exit $?
done
