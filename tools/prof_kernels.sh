#!/bin/bash
# per-kernel trace stats for a command (args), summary to gpurun_out/<name>_stats.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
NAME=$1; shift
O=gpurun_out/$NAME
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- "$@" > $O/log.txt 2>&1
rc=$?
python3 - "$O" <<'PY'
import csv, re, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True) or glob.glob(sys.argv[1] + "/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
with open(sys.argv[1] + "_stats.txt", "w") as out:
    for r in rows[:25]:
        m = re.search(r"(\w+_kernel\w*|\w+)\s*[<(]", r["Name"])
        nm = r["Name"][:90]
        line = f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {float(r["Percentage"]):5.1f}%  {nm}'
        out.write(line + "\n")
        print(line)
PY
exit $rc
