#!/bin/bash
# per-kernel stats + PMC counters of the CS-WLS kernels (bench config), results under gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prof_xs
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $O/trace.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d $O/pmc1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $O/pmc1.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $O/pmc2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $O/pmc2.log 2>&1 \
 && timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > $O/pmc3.log 2>&1
echo "rc=$?"
