#!/bin/bash
# bench.py's --groups (swarm_step_streams: each decision as K env-range launches on K streams with
# no per-decision join) at the C2 workload, alternating K, layouts and (optionally) variant
# libraries over REPS passes on one box, default and driver (--steps 20 --warmup 5) arguments.
#   OUT=gpurun_out/x REPS=2 KS="1 2 3" LAYOUTS="0 203" VLIBS="build/variants/lib_a.so ..." tools/groups_sweep.sh
# ORDERS="0 6 10" also alternates the layout-203 dispatch order (SWARM_ARENA_ORDER: heavy threshold, 0 = identity).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/groups}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for ord in ${ORDERS:-lib}; do
  for lib in ${VLIBS:-product}; do
    lname=$(basename $lib .so); lname=${lname#lib_}
    if [ "$ord" = lib ]; then unset SWARM_ARENA_ORDER; else export SWARM_ARENA_ORDER=$ord; lname=${lname}_o$ord; fi
    for ly in ${LAYOUTS:-0}; do
      for k in ${KS:-1 2 3}; do
        for args in "" "--steps 20 --warmup 5"; do
          tag="${lname}_k${k}_ly${ly}_$( [ -z "$args" ] && echo default || echo driver )"
          if [ "$lib" = product ]; then
            timeout -k 10 120 python3 bench.py --cpu-seconds 0 --groups $k --layout $ly $args > $OUT/$tag.log 2>&1
          else
            SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --groups $k --layout $ly $args \
              > $OUT/$tag.log 2>&1
          fi
          [ $? -ne 0 ] && { echo "bench $tag failed"; tail -5 $OUT/$tag.log; exit 5; }
          grep '^{' $OUT/$tag.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']
print(json.dumps({'rep': $rep, 'tag': '$tag', 'value': d['value'], 'decision_us': r['kernel_avg_us'],
                  'layout': r['layout'], 'groups': r['groups'], 'ms_per_step': d['ms_per_step'],
                  'stream_launch_us': r.get('launch_avg_us_per_stream'),
                  'order': '$ord'}))" | tee -a $OUT/sweep.jsonl
        done
      done
    done
  done
  done
done
