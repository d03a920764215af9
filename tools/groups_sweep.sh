#!/bin/bash
# bench.py's --groups (swarm_step_streams: each decision as K env-range launches on K streams with
# no per-decision join) at the C2 workload, alternating K and layouts over REPS passes on one box.
#   OUT=gpurun_out/x REPS=2 KS="1 2 3 4" LAYOUTS="0 203" tools/groups_sweep.sh
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/groups}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for ly in ${LAYOUTS:-0}; do
    for k in ${KS:-1 2 3 4}; do
      for args in "" "--steps 20 --warmup 5"; do
        tag="k${k}_ly${ly}_$( [ -z "$args" ] && echo default || echo driver )"
        timeout -k 10 120 python3 bench.py --cpu-seconds 0 --groups $k --layout $ly $args > $OUT/$tag.log 2>&1 \
          || { echo "bench $tag failed"; tail -5 $OUT/$tag.log; exit 5; }
        grep '^{' $OUT/$tag.log | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']
print(json.dumps({'rep': $rep, 'tag': '$tag', 'value': d['value'], 'decision_us': r['kernel_avg_us'],
                  'layout': r['layout'], 'groups': r['groups']}))" | tee -a $OUT/sweep.jsonl
      done
    done
  done
done
