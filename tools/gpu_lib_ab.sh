#!/bin/bash
# Production-path CS-WLS timing (tools/xs_lat_ab.py, mode 0) of the in-tree library vs the
# alternative builds abl/*.so (copied from tools/build_ab_lib.sh output; ab_libs/ is gpurun-ignored), alternated twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for L in default abl/*.so; do
    if [ "$L" = default ]; then unset MFA_HIP_LIB; else export MFA_HIP_LIB=$PWD/$L; fi
    echo "== $L"
    MODES=0 DS=${DS:-315,2520} timeout -k 10 200 python -u tools/xs_lat_ab.py 2>&1 | grep '"us"' || exit 1
  done
done
