#!/bin/bash
# Times the step kernel at 1, 2 and 4 cooperating waves per workgroup.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in ${WAVES:-1 2 4}; do
  timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 --layout $w ${BENCH_ARGS:-} > gpurun_out/waves_$w.log 2>&1 || { echo "W=$w failed"; tail -5 gpurun_out/waves_$w.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/waves_$w.log').read().strip().splitlines()[-1]); print('W=$w', 'value %.4g' % d['value'], 'kernel_us %.1f' % d['roofline']['kernel_avg_us'])"
done
