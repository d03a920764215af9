#!/bin/bash
# Build timing-only ablation variants of the critic kernel as standalone .so files
# (build/variants/critic_ablate/libcritic_<mask>.so; ABL_DIR overrides); time them with tools/critic_ablate.py on the GPU.
set -e
cd "$(dirname "$0")/../swarmacb-isaaclab_amd/csrc"
OUT=../../${ABL_DIR:-build/variants/critic_ablate}
mkdir -p $OUT
cat > $OUT/stub.cpp <<'EOS'
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace swarm { int32_t record_hip_status() { return hipGetLastError() == hipSuccess ? 0 : -3; } }
EOS
rm -f $OUT/libcritic_*.so
if [ -n "$VARIANTS" ]; then
  # named flag sets: VARIANTS="name:flags;name2:flags2" (timing + output comparison, no ablation)
  IFS=';' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    name=${v%%:*}; flags=${v#*:}
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -shared $flags \
      -o $OUT/libcritic_$name.so swarm_critic.hip $OUT/stub.cpp &
  done
else
  for m in ${MASKS:-0 1 2 4 8 16 6}; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -shared -DRSA_ABLATE=$m \
      -o $OUT/libcritic_$m.so swarm_critic.hip $OUT/stub.cpp &
  done
fi
wait
ls $OUT
