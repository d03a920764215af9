#!/bin/bash
# Round-4 step-kernel study 6 on one MI355X: wall-split variants against base / zlfr
# (build/variants6, 600-step bench, alternating REPS times), then parity on the wall-split ones.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-3}); do
  for lib in build/variants6/lib_*.so; do
    name=$(basename $lib .so); name=${name#lib_}
    SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 > $OUT/var_${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -5 $OUT/var_${name}_$rep.log; exit 3; }
    python3 -c "import json; d=json.loads(open('$OUT/var_${name}_$rep.log').read().strip().splitlines()[-1]); print('$name rep $rep', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
  done
done
for name in ${PARITY:-exactmd}; do
  SWARMSTEP_LIB=$PWD/build/variants6/lib_$name.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_philox.py \
    -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$name.log 2>&1
  echo "$name parity rc=$?"; tail -1 $OUT/pytest_$name.log; grep '^FAILED' $OUT/pytest_$name.log | head -5
done
echo R4O_DONE
