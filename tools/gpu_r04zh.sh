#!/bin/bash
# round 4: rolling EW kernels with the chunk-map scan on DPP moves (variant 12) -- A/B incl.
# numerics against the round-1 direct kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04zh; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1; rc=$?
grep '"kernel": "beta\|"kernel": "dastd' $O/rolling_ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['kernel'], {k: (v['ms'], '%.1e' % v['max_rel_vs_r01']) for k, v in r.items() if isinstance(v, dict) and k in ('san_8x256_prefetch','san_dpp_scan','default','r03_default')})"
exit $rc
