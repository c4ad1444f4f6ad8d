#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmc_eig
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/a -o run --output-format csv -- python3 tools/eigen_bench.py 630 > $O/a.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES -d $O/b -o run --output-format csv -- python3 tools/eigen_bench.py 630 > $O/b.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ["a", "b"]:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_eig/{d}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"gpurun_out/pmc_eig/{d}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "mc_bias" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {c: f"{sum(v)/len(v):.3g}" for c, v in agg.items()})
PY
