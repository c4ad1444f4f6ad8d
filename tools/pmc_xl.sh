#!/bin/bash
# round 6: where the XL solver's time goes (RiskModel.run at K = 200: P = 183, Q = 16, 452 dates,
# M = 100).  One PMC pass of 8 SQ counters over the run, then per-problem totals of the bias
# kernel (eig_xl_kernel<false, 4>: 452 x 100 problems on persistent workgroups) and the share
# of wave cycles spent waiting on an instruction's operands (memory / LDS / dependencies).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_xl; rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 tools/risk_run_only.py --make /tmp/panel200.pt --dates 452 --P 183 --Q 16 > $O/make.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o run --output-format csv -- python3 tools/risk_run_only.py --load /tmp/panel200.pt --P 183 --Q 16 --nw-half-life 1000 --reps 1 > $O/a.log 2>&1 || exit 1
rm -f /tmp/panel200.pt
python3 - <<'PY' | tee gpurun_out/pmc_xl/summary.txt
import csv, glob, collections
agg = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_xl/a/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "eig_xl_kernel<false" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
print("dispatch records per counter:", dict(n))
print("totals:", {k: f"{v:.4g}" for k, v in sorted(agg.items())})
runs = max(n.values()) if n else 1          # warm-up + timed runs
B = 452 * 100                                # problems per run (invalid dates exit early)
for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
    print(f"{k} per problem (wave instructions): {agg.get(k, 0.0) / runs / B:.0f}")
if agg.get("SQ_WAVE_CYCLES"):
    print(f"SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: {agg.get('SQ_WAIT_INST_ANY', 0.0) / agg['SQ_WAVE_CYCLES']:.3f}")
PY
