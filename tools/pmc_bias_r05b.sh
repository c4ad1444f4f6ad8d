#!/bin/bash
# round 5: instructions per problem of the production bias solver (mode 5) inside RiskModel.run
# (252 dates x 5000 stocks, K = 42, M = 100): one PMC pass of 8 SQ counters, then per-wave
# (= per-problem: one 64-lane workgroup per (date, sim)) averages of mc_bias_tri2_kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_bias_r05b; rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 tools/risk_run_only.py --make /tmp/panel252.pt --dates 252 > $O/make.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o run --output-format csv -- python3 tools/risk_run_only.py --load /tmp/panel252.pt --reps 1 > $O/a.log 2>&1 || exit 1
python3 - <<'PY' | tee gpurun_out/pmc_bias_r05b/summary.txt
import csv, glob, collections
agg = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_bias_r05b/a/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mc_bias_tri2_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
w = agg.get("SQ_WAVES", 0.0)
print("dispatch records per counter:", dict(n))
print("totals:", {k: f"{v:.4g}" for k, v in sorted(agg.items())})
if w:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64"):
        print(f"{k} per wave (problem): {agg.get(k, 0.0) / w:.0f}")
PY
