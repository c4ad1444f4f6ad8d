#!/bin/bash
# PMC counters of the Monte-Carlo bias kernel (eigen_bench: 2520 dates x 100 sims, K = 42).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_eig; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/a -o run --output-format csv -- python3 tools/eigen_bench.py 2520 > $O/a.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_eig/a/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mc_bias" in r["Kernel_Name"]:
            agg["mc_bias"][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    v = {c: sum(x) / len(x) for c, x in d.items()}
    print(k, {c: f"{x:.3g}" for c, x in v.items()})
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(f"  LDS active {v.get('SQ_ACTIVE_INST_LDS', 0) / wc:.1%} of wave-cycles, VALU active {v.get('SQ_ACTIVE_INST_VALU', 0) / wc:.1%}, "
          f"bank-conflict / LDS-active {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(v.get('SQ_ACTIVE_INST_LDS', 1), 1):.1%}, "
          f"wait-LDS {v.get('SQ_WAIT_INST_LDS', 0) / wc:.1%}")
PY
