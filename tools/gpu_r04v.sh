#!/bin/bash
# round 4 tree with the resident CS-WLS kernel and the 16-row-chunk rolling variants: whole GPU
# suite, smoke, bench lines, bench kernel stats, rolling A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r04v; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python tools/rolling_ab.py > $O/rolling_ab.jsonl 2>&1 \
 && grep '"kernel": "beta\|"kernel": "dastd' $O/rolling_ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['kernel'], {k: v['ms'] for k, v in r.items() if isinstance(v, dict)})" \
 && timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --check > $O/bench_fp64.log 2>&1 && tail -1 $O/bench_fp64.log | cut -c1-300 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --prewarm 20 > $O/prof.log 2>&1 \
 && find $O/prof -name '*kernel_stats.csv' | head -1 | xargs head -4 | cut -c1-160
rc2=$?; exit $(( rc | rc2 ))
