#!/bin/bash
# Timing-only ablation study of the step kernel (results of the variants are
# wrong by design). `tools/ablate.sh build` cross-compiles the variants here;
# `tools/ablate.sh run` times each with bench.py on the GPU box.
set -o pipefail
cd "$(dirname "$0")/.."
MASKS=${MASKS:-"0 1 2 3 4 8 16 31"}
OUT=build/ablate
if [ "$1" = build ]; then
  # variants differ only in the Homing translation unit: reuse the other objects
  make -s -j8 -C swarmacb-isaaclab_amd/csrc || exit 1
  mkdir -p $OUT
  for m in $MASKS; do
    rm -rf $OUT/obj_$m && cp -rp build/obj $OUT/obj_$m && rm -f $OUT/obj_$m/swarm_mission_2.o
    make -s -C swarmacb-isaaclab_amd/csrc OBJDIR=$PWD/$OUT/obj_$m OUT=$PWD/$OUT/lib_$m.so EXTRA=-DSWARM_ABLATE=$m &
  done
  wait
  rm -rf $OUT/obj_*
  ls -la $OUT
  exit 0
fi
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in $MASKS; do
  SWARMSTEP_LIB=$PWD/$OUT/lib_$m.so timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 ${BENCH_ARGS:-} > gpurun_out/ablate_$m.log 2>&1 || { echo "mask $m failed"; tail -5 gpurun_out/ablate_$m.log; exit 3; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ablate_$m.log').read().strip().splitlines()[-1]); print('mask $m', 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % d['roofline']['kernel_avg_us'])"
done
