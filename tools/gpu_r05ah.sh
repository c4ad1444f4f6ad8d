#!/bin/bash
# A/B: bias mode 5 (8-step Householder groups) vs mode 25 (4-step groups)
set -o pipefail
O=gpurun_out/r05ah; mkdir -p $O
MODES=5,25 ROUNDS=4 timeout -k 10 400 python -u tools/bias_chain_ab.py > $O/bias_gs_ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
tail -2 $O/bias_gs_ab.jsonl
