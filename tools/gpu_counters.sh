#!/bin/bash
# List the PMC counters rocprofv3 offers on this box (TCC / MALL related) into gpurun_out/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/counters_avail.txt 2>&1
grep -i -E "^\s*(TCC_EA|TCC_BUBBLE|MALL|TCC_READ|TCC_HIT|TCC_MISS)|DRAM|mall" gpurun_out/counters_avail.txt | head -60
