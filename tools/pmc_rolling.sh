#!/bin/bash
# Kernel stats + PMC counters of the rolling-descriptor scan kernels (tools/factor_bench.py,
# 5000 x 3780 flat panel).  Two runs: kernel trace/stats, then one PMC pass of <= 8 SQ counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_roll; rm -rf $O; mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/k -o run --output-format csv -- python3 tools/factor_bench.py > $O/k.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/a -o run --output-format csv -- python3 tools/factor_bench.py > $O/a.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/pmc_roll/k/**/run_kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  x{r["Calls"]:>4}  {r["Name"][:90]}')
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_roll/a/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if any(t in kn for t in ("scan_kernel", "ew_window", "vhgw", "rstr_ew")):
            key = kn.split("(")[0][-70:]
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    v = {c: sum(x) / len(x) for c, x in d.items()}
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(k, f"busy {v.get('SQ_BUSY_CYCLES',0):.3g} wave-cyc {wc:.3g} VALU-active {v.get('SQ_ACTIVE_INST_VALU', 0) / wc:.1%} "
          f"LDS-active {v.get('SQ_ACTIVE_INST_LDS', 0) / wc:.1%} wait-LDS {v.get('SQ_WAIT_INST_LDS', 0) / wc:.1%} "
          f"insts VALU {v.get('SQ_INSTS_VALU',0):.3g} LDS {v.get('SQ_INSTS_LDS',0):.3g} bank-conf {v.get('SQ_LDS_BANK_CONFLICT',0):.3g}")
PY
