#!/bin/bash
# Instruction-cache behaviour of the mode-5 bias kernel (~14k instructions, larger than the
# 64 KB instruction cache two CUs share?): one PMC pass of four SQ-block counters on the
# pipeline's inputs (tools/eigen_tol.py, mode 5 only), then the per-kernel sums.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/pmc_icache; rm -rf $O; mkdir -p $O
export SETTINGS=1e-15:30 SUB=2 MODES=5
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_VALU -d $O/a -o run --output-format csv -- python3 tools/eigen_tol.py > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmc_icache/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "bias_tri2(mode5)" if "mc_bias_tri2" in r["Kernel_Name"] else ("jacobi" if "mc_bias_kernel" in r["Kernel_Name"] else None)
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    h, m = v.get("SQC_ICACHE_HITS", 0), v.get("SQC_ICACHE_MISSES", 0)
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())},
          f"icache miss rate {m / max(h + m, 1):.3%}, misses per wave {m / max(v.get('SQ_WAVES', 1), 1):.1f}")
PY
