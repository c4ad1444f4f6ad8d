#!/bin/bash
# PMC of the default rolling kernels (tools/rolling_ab.py, 5000 x 3780): VALU / LDS activity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=${O:-gpurun_out/pmc_roll2}; rm -rf $O; mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVES -d $O/a -o run --output-format csv -- python3 tools/rolling_ab.py > $O/a.log 2>&1 || exit 1
O=$O python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(__import__("os").environ.get("O", "gpurun_out/pmc_roll2") + "/a/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if any(t in kn for t in ("ew_window", "vhgw", "vh2", "rstr_ew")):
            agg[kn[:kn.rfind("(")].replace("(anonymous namespace)::", "")[-70:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    v = {c: sum(x) / len(x) for c, x in d.items()}
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(k, f"waves {v.get('SQ_WAVES',0):.3g} VALU-active {v.get('SQ_ACTIVE_INST_VALU',0)/wc:.1%} LDS-active {v.get('SQ_ACTIVE_INST_LDS',0)/wc:.1%} "
          f"wait-LDS {v.get('SQ_WAIT_INST_LDS',0)/wc:.1%} wait-any {v.get('SQ_WAIT_INST_ANY',0)/wc:.1%} VALU-insts {v.get('SQ_INSTS_VALU',0):.3g} busy {v.get('SQ_BUSY_CYCLES',0):.3g}")
PY
