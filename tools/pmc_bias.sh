#!/bin/bash
# PMC counters of mc_bias_kernel on the pipeline's own inputs (tools/eigen_tol.py, one setting).
# Two passes of <= 8 SQ counters each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_bias; rm -rf $O; mkdir -p $O
export SETTINGS="${SETTINGS:-1e-15:30}" SUB=2
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/a -o run --output-format csv -- python3 tools/eigen_tol.py > $O/a.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 -d $O/b -o run --output-format csv -- python3 tools/eigen_tol.py > $O/b.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
import os
agg = collections.defaultdict(list)
# the tool runs the Jacobi (mode 0) once as its baseline: count only the selected solver
want = "mc_bias_tri" if os.environ.get("MODES", "0") != "0" else "mc_bias_kernel"
for f in glob.glob("gpurun_out/pmc_bias/*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if want in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
v = {c: sum(x) / len(x) for c, x in agg.items()}
print({c: f"{x:.4g}" for c, x in sorted(v.items())})
wc = v.get("SQ_WAVE_CYCLES", 1)
print(f"LDS active {v.get('SQ_ACTIVE_INST_LDS', 0) / wc:.1%} of wave-cycles, VALU active {v.get('SQ_ACTIVE_INST_VALU', 0) / wc:.1%}, "
      f"bank-conflict / LDS-idx-active {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(v.get('SQ_LDS_IDX_ACTIVE', 1), 1):.1%}, "
      f"wait-LDS {v.get('SQ_WAIT_INST_LDS', 0) / wc:.1%}, LDS-idx-active / busy {v.get('SQ_LDS_IDX_ACTIVE', 0) / max(v.get('SQ_BUSY_CYCLES', 1), 1):.3g}")
PY
