set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
DATES=64,315,2520 CHUNKS=8 DTYPES=fp64 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt/p -o run --output-format csv -- python3 tools/xs_time.py > gpurun_out/kt/xs_time.txt 2>&1
rc=$?
f=$(find gpurun_out/kt/p -name '*kernel_trace.csv' | head -1)
python3 tools/ktrace_summary.py "$f" xs_ > gpurun_out/kt/summary.txt
rm -rf gpurun_out/kt/p
cat gpurun_out/kt/summary.txt
exit $rc
