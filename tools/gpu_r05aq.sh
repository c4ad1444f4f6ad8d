#!/bin/bash
# after the final build(): smoke + 1-GPU bench
set -o pipefail
O=gpurun_out/r05aq; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-300
