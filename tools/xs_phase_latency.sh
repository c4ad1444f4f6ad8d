# Phase latency of the fused CS-WLS kernel vs dates per launch (timing-only ablation variants:
# 0 full, 4 no residual pass, 8 no solve, 12 moments only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/phase
for dt in fp64 fp32; do
  for D in 64 315 2520; do
    echo "== $dt D=$D"
    DTYPE=$dt D=$D VARIANTS=0,4,8,12 timeout -k 10 120 python3 tools/xs_ab_variants.py 2>/dev/null || exit 1
  done
done
