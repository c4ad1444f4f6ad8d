#!/bin/bash
# Build an alternative kernel library with extra -D flags for A/B timing (tools/gpu_ab_libs.sh):
#   tools/build_ab_lib.sh NAME -DMFA_XS_PREU=3 ...   -> ab_libs/NAME.so (git-ignored)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ab_libs/obj_$NAME
OBJS=()
for s in llm_driven_multi_factor_model_amd/csrc/*.hip; do
  o=ab_libs/obj_$NAME/$(basename ${s%.hip}).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=fast -munsafe-fp-atomics \
    -Illm_driven_multi_factor_model_amd/csrc "$@" -c $s -o $o &
  OBJS+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${OBJS[@]}" -o ab_libs/$NAME.so
rm -rf ab_libs/obj_$NAME
echo ab_libs/$NAME.so
