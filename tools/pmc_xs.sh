#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmc_xs
mkdir -p $O
for v in ${VARS:-0 1}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/a$v -o run --output-format csv -- python3 tools/xs_one.py $v > $O/a$v.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d $O/b$v -o run --output-format csv -- python3 tools/xs_one.py $v > $O/b$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, re, collections
for d in sorted(glob.glob("gpurun_out/pmc_xs/[ab]*[0-9]")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True) + glob.glob(d + "/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(xs_\w+)", r["Kernel_Name"])
            if m:
                agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        print(d.split("/")[-1], k, {c: f"{sum(v)/len(v):.3g}" for c, v in dd.items()})
PY
