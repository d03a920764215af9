#!/bin/bash
# Round-4 step-kernel study on one MI355X: the variant libraries of build/variants (600-step bench,
# alternating twice) and the wave-timing build's schedule view (tools/wave_timing.py with
# build/wt/lib_wt.so). Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4c
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
    print('$name', d['launch'], 'span %.1f' % d['span_us'], 'simd_end', d['simd_end_us'], 'life p50 %.1f max %.1f' % (d['life_us']['p50'], d['life_us']['p100']),
          {k: s[k] for k in s if k not in ('rank_of_block_quarters', 'simd_end_by_xcc_us')})
"
done
for rep in 1 2; do
  for lib in build/variants/lib_*.so; do
    [ -e "$lib" ] || continue
    name=$(basename $lib .so); name=${name#lib_}
    SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 --graph 0 > $OUT/var_${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -5 $OUT/var_${name}_$rep.log; exit 3; }
    python3 -c "import json; d=json.loads(open('$OUT/var_${name}_$rep.log').read().strip().splitlines()[-1]); print('$name rep $rep', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
  done
done
if [ -f build/variants/lib_all6.so ]; then
  SWARMSTEP_LIB=$PWD/build/variants/lib_all6.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_philox.py \
    -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_all6.log 2>&1
  echo "all6 parity rc=$?"; tail -3 $OUT/pytest_all6.log
fi
echo R4C_DONE
