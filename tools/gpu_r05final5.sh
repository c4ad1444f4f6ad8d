#!/bin/bash
# Round-5 closing check on one GPU: full GPU test suite, smoke, headline bench (fp64 + fp32 storage),
# per-shard-size bench (strong-scaling shard sizes), rocprofv3 kernel stats of the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05final5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --check > $O/bench_fp64.log 2>&1 && tail -1 $O/bench_fp64.log \
 && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --storage fp32 > $O/bench_fp32.log 2>&1 && tail -1 $O/bench_fp32.log \
 && for d in 315 630 1260; do timeout -k 10 120 python bench.py --steps 30 --warmup 5 --dates $d > $O/bench_fp64_d$d.log 2>&1 && tail -1 $O/bench_fp64_d$d.log || exit 1; done \
 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --prewarm 20 > $O/prof.log 2>&1 \
 && find $O/prof -name '*kernel_stats.csv' | head -1 | xargs head -6 | cut -c1-160
echo "== 2-rank gloo rehearsal (two ranks share the GPU)" \
 && MFA_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --prewarm 5 > $O/bench_gloo2.log 2>&1 && tail -1 $O/bench_gloo2.log
bash tools/prof_kernels.sh risk_run python3 tools/risk_stages.py --reps 1 > /dev/null 2>&1 && cp gpurun_out/risk_run_stats.txt $O/risk_run_kernel_stats.txt && head -8 $O/risk_run_kernel_stats.txt
echo "== stage timings / BASELINE configs / end-to-end job" \
 && timeout -k 10 300 python tools/risk_stages.py > $O/risk_stages.log 2>&1 && tail -2 $O/risk_stages.log \
 && timeout -k 10 400 python tools/baseline_configs.py > $O/baseline_configs.log 2>&1 && tail -6 $O/baseline_configs.log \
 && timeout -k 10 300 python tools/pipeline_e2e.py > $O/pipeline_e2e.log 2>&1 && tail -2 $O/pipeline_e2e.log
