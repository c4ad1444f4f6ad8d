#!/bin/bash
# rocprofv3 kernel stats for the full risk pipeline (+ attribution) and the rolling descriptors.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof_pipe; export TMPDIR=/tmp
O=gpurun_out/prof_pipe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/risk -o run --output-format csv -- python3 tools/risk_stages.py --attribution --reps 2 > $O/risk.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fac -o run --output-format csv -- python3 tools/factor_bench.py > $O/fac.log 2>&1 \
 && python3 - <<'PY'
import csv, glob
for tag in ("risk", "fac"):
    f = glob.glob(f"gpurun_out/prof_pipe/{tag}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    print(f"== {tag}")
    for r in rows[:14]:
        print(f"{float(r['TotalDurationNs'])/1e3:11.1f} us total  {r['Calls']:>5} calls  {float(r['AverageNs'])/1e3:9.1f} us avg  {r['Name'][:110]}")
PY
