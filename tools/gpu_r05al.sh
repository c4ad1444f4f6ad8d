#!/bin/bash
# A/B: bias mode 5 (64-entry LDS tables) vs mode 28 (KP-entry tables: 15 instead of 13 workgroups per CU)
set -o pipefail
O=gpurun_out/r05al; mkdir -p $O
MODES=5,28,29 ROUNDS=4 timeout -k 10 400 python -u tools/bias_chain_ab.py > $O/bias_lt_ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
tail -2 $O/bias_lt_ab.jsonl
