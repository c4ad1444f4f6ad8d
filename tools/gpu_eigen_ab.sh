#!/bin/bash
# Bias-solver A/B on the pipeline's own inputs (tools/eigen_tol.py): bias modes MODES of the
# in-tree library and of every abl/*.so alternative build, plus the eigen GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/eigen_ab.jsonl; : > $O
for L in default abl/*.so; do
  [ -e "$L" ] || [ "$L" = default ] || continue
  if [ "$L" = default ]; then unset MFA_HIP_LIB; else export MFA_HIP_LIB=$PWD/$L; fi
  echo "== $L" | tee -a $O
  SETTINGS=1e-15:30 MODES=${MODES:-3,4,5} timeout -k 10 300 python -u tools/eigen_tol.py 2>&1 | tee -a $O | grep '"mode"' || exit 1
done
unset MFA_HIP_LIB
