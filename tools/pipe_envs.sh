#!/bin/bash
# Layouts (LAYOUTS, default: 0 = the library's choice, 103) at env counts ENVS, REPS alternating
# repetitions; the library in SWARMSTEP_LIB (default: the in-tree one). Prints kernel us per launch.
mkdir -p gpurun_out/pe
for rep in $(seq ${REPS:-1}); do
  for E in ${ENVS:-1024 2048 4096}; do for w in ${LAYOUTS:-0 103}; do
    timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps ${PE_STEPS:-600} --envs $E --layout $w \
      > gpurun_out/pe/pe_${E}_${w}_$rep.log 2>&1 || { tail -5 gpurun_out/pe/pe_${E}_${w}_$rep.log; exit 3; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pe/pe_${E}_${w}_$rep.log').read().strip().splitlines()[-1]); print('rep $rep E=$E layout=$w', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
  done; done
done
