set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for rep in 1 2; do
for L in default abl/wpe3.so abl/wpe4.so; do
  if [ "$L" = default ]; then unset MFA_HIP_LIB; else export MFA_HIP_LIB=$PWD/$L; fi
  echo "== $L"
  if [ $rep = 1 ]; then timeout -k 10 200 python -u -m pytest tests/test_eigen.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -n1 || exit 1; fi
  timeout -k 10 200 python -u tools/risk_stages.py --reps 3 2>&1 | grep shape | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['stage_ms']['eigen_adjust'], d['total_ms'])" || exit 1
done
done
