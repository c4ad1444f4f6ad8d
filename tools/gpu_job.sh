#!/bin/bash
# One parametrised GPU job for `gpurun` (replaces the per-round tools/gpu_r0*.sh one-offs):
#   tools/gpu_job.sh TAG SECONDS 'command' [SECONDS 'command' ...]
# Every step runs under its own `timeout -k 10 SECONDS`, writes gpurun_out/TAG/NN.log, and the
# job stops at the first failing step (a fault, abort or time limit ends the GPU work of the
# call).  A progress line per step keeps the box's silence watchdog fed.
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
i=0
while [ $# -ge 2 ]; do
  t=$1; cmd=$2; shift 2
  i=$((i + 1))
  log=$(printf '%s/%02d.log' "$out" "$i")
  echo "[$tag] step $i (<= ${t}s): $cmd" | tee -a "$out/steps.txt"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "[$tag] step $i rc=$rc $(( $(date +%s) - start ))s" | tee -a "$out/steps.txt"
  tail -5 "$log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
