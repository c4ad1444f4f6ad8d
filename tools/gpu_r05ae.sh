#!/bin/bash
# flagged-matrix re-solve split: warm / cold setup vs sweeps
set -o pipefail
O=gpurun_out/r05ae; mkdir -p $O
for s in 3 0 1234; do
  SEED=$s timeout -k 10 240 python -u tools/eigh_resolve_split.py >> $O/eigh_resolve_split.jsonl 2>>$O/err.log || exit $?
done
