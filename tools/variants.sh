#!/bin/bash
# Build-time variant study of the Homing step kernel.
#   VARIANTS="name:flags;name2:flags2" tools/variants.sh build   (here, cross-compiles)
#   tools/variants.sh run                                         (GPU box: bench each lib x WAVES)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${VOUT:-build/variants}
if [ "$1" = build ]; then
  make -s -j8 -C swarmacb-isaaclab_amd/csrc || exit 1
  rm -rf $OUT && mkdir -p $OUT
  IFS=';' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    name=${v%%:*}; flags=${v#*:}
    cp -rp build/obj $OUT/obj_$name && rm -f $OUT/obj_$name/swarm_mission_2.o
    make -s -C swarmacb-isaaclab_amd/csrc OBJDIR=$PWD/$OUT/obj_$name OUT=$PWD/$OUT/lib_$name.so EXTRA="$flags" &
  done
  wait
  rm -rf $OUT/obj_*
  ls $OUT
  exit 0
fi
mkdir -p gpurun_out
if [ "$1" = pmc ]; then
  export TMPDIR=/tmp
  for lib in $OUT/lib_*.so; do
    name=$(basename $lib .so); name=${name#lib_}
    for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
                "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
                "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
      tag=$(echo $pass | cut -c1-12 | tr ' ' _)
      SWARMSTEP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-include-regex step_kernel --pmc $pass \
        -d gpurun_out/vpmc/$name/$tag -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --steps 100 --warmup 10 \
        --layout ${WAVES:-0} > gpurun_out/vpmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/vpmc_$name.log; exit 3; }
    done
  done
  python3 tools/pmc_table.py gpurun_out/vpmc
  exit 0
fi
# REPS alternating repetitions over the libraries (A B C A B C ...): box drift hits all alike
for rep in $(seq ${REPS:-1}); do
  for lib in $OUT/lib_*.so; do
    name=$(basename $lib .so); name=${name#lib_}
    for w in ${WAVES:-0}; do
      SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps ${VSTEPS:-600} --layout $w ${BENCH_ARGS:-} \
        > gpurun_out/var_${name}_${w}_$rep.log 2>&1 || { echo "$name W=$w failed"; tail -5 gpurun_out/var_${name}_${w}_$rep.log; exit 3; }
      python3 -c "import json; d=json.loads(open('gpurun_out/var_${name}_${w}_$rep.log').read().strip().splitlines()[-1]); print('rep $rep $name W=$w', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
    done
  done
done
