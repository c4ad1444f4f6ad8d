#!/bin/bash
# A/B: residual prefetch during the solve on fp64 panels (CS-WLS modes 23 / 24) vs the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pre64; export TMPDIR=/tmp
MODES=0,23,24,20 DATES=64,315,630,1260,2520 DTYPES=fp64,fp32 timeout -k 10 400 python -u tools/xs_mode_time.py > gpurun_out/pre64/ab.jsonl 2> gpurun_out/pre64/ab.err; rc=$?
cat gpurun_out/pre64/ab.jsonl; exit $rc
