#!/bin/bash
# L2 <-> fabric traffic per CS-WLS call (FETCH_SIZE / WRITE_SIZE in KB), fused vs team kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_traffic; rm -rf $O; mkdir -p $O
for w in ${WHICH:-fused team4}; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f_$w -o run --output-format csv -- python3 tools/xs_traffic.py $w > $O/f_$w.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w_$w -o run --output-format csv -- python3 tools/xs_traffic.py $w > $O/w_$w.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections, json
res = {}
for d in sorted(glob.glob("gpurun_out/pmc_traffic/[fw]_*")):
    if d.endswith(".log"):
        continue
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            if "xs_fused_kernel" in kn or "xs_pipe_kernel" in kn or "reduce_kernel" in kn:
                agg[kn.split("(")[0][-60:] + " " + r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        res[d.split("/")[-1] + " " + k] = {"calls": len(v), "median_GB": round(sorted(v)[len(v) // 2] / 1e6, 3)}
print(json.dumps(res, indent=1))
PY
