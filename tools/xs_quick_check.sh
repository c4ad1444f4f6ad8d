set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_xs_wls.py tests/test_determinism.py tests/test_mfm_compat.py tests/test_xs_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/xs_phase_latency.sh > gpurun_out/q/phase.txt 2>&1 && cat gpurun_out/q/phase.txt
