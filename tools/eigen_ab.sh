#!/bin/bash
# Time the Monte-Carlo eigen adjustment under alternative compile-time configs (ab_libs/*.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for L in default ab_libs/*.so; do
  if [ "$L" = default ]; then unset MFA_HIP_LIB; else export MFA_HIP_LIB=$PWD/$L; fi
  echo "== $L"; timeout -k 10 120 python -u tools/eigen_bench.py 2520 || exit 1
done
done
