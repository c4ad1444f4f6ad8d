#!/bin/bash
# Time the fused CS-WLS kernel under alternative compile-time configs (ab_libs/*.so) vs default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in default ab_libs/*.so; do
  if [ "$L" = default ]; then unset MFA_HIP_LIB; else export MFA_HIP_LIB=$PWD/$L; fi
  echo "== $L"; VARIANTS=${VARIANTS:-0,12} timeout -k 10 120 python -u tools/xs_ablate.py 2>&1 | grep variant || exit 1
done
