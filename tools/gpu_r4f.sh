#!/bin/bash
# Round-4 step-kernel study 2 on one MI355X: wave timing (identity vs arena order), the variant
# libraries of build/variants2 (600-step bench, alternating twice), then the parity tests on the
# non-bitwise pair-term variant and on the combined bitwise variants.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
for lib in build/wt/lib_*.so; do
  [ -e "$lib" ] || continue
  name=$(basename $lib .so); name=${name#lib_}
  SWARMSTEP_LIB=$PWD/$lib timeout -k 10 240 python3 -u tools/wave_timing.py > $OUT/wave_timing_$name.jsonl 2> $OUT/wave_timing_$name.err \
    || { echo "wave timing $name failed"; tail -5 $OUT/wave_timing_$name.err; exit 2; }
  python3 -c "
import json
for l in open('$OUT/wave_timing_$name.jsonl'):
    d = json.loads(l); s = d['sched']
    print('$name', d['launch'], 'span %.1f' % d['span_us'], 'simd_end', d['simd_end_us'], 'life p50 %.1f max %.1f' % (d['life_us']['p50'], d['life_us']['p100']), 'prev corr', s.get('corr_life_prev_launch'))
"
done
for rep in 1 2; do
  for lib in build/variants2/lib_*.so; do
    name=$(basename $lib .so); name=${name#lib_}
    SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 > $OUT/var_${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -5 $OUT/var_${name}_$rep.log; exit 3; }
    python3 -c "import json; d=json.loads(open('$OUT/var_${name}_$rep.log').read().strip().splitlines()[-1]); print('$name rep $rep', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
  done
done
for name in rsq bw4 bw4order; do
  SWARMSTEP_LIB=$PWD/build/variants2/lib_$name.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_philox.py \
    -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_$name.log 2>&1
  echo "$name parity rc=$?"; tail -1 $OUT/pytest_$name.log; grep '^FAILED' $OUT/pytest_$name.log | head -5
done
echo R4F_DONE
