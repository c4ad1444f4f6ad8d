# Moments-phase ablation of the fused CS-WLS kernel: 12 = moments only, 13 = without the segment
# atomics, 14 = without the style-Gram FMAs, 15 = without both (DMA + reads + reduction only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for dt in fp64 fp32; do
  for D in 64 2520; do
    echo "== $dt D=$D"
    DTYPE=$dt D=$D VARIANTS=12,13,14,15 timeout -k 10 120 python3 tools/xs_ab_variants.py 2>/dev/null || exit 1
  done
done
