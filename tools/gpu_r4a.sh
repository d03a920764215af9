#!/bin/bash
# Round-4 session A on one MI355X: step-kernel variant timings (build/variants/lib_*.so,
# alternating twice), the step parity tests on the all-variants library (its pair term is not
# bitwise), the full GPU suite + smoke on the in-tree library, and the bench of record with the
# driver's arguments under rocprofv3. Each GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
OUT=gpurun_out/r4a
for rep in ${VARIANT_REPS-1 2}; do
  for lib in build/variants/lib_*.so; do
    [ -e "$lib" ] || continue
    name=$(basename $lib .so); name=${name#lib_}
    SWARMSTEP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 --graph 0 > $OUT/var_${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -5 $OUT/var_${name}_$rep.log; exit 2; }
    python3 -c "import json; d=json.loads(open('$OUT/var_${name}_$rep.log').read().strip().splitlines()[-1]); print('$name rep $rep', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'])"
  done
done
if [ -n "${VARIANT_REPS-1 2}" ] && [ -f build/variants/lib_all6.so ]; then
  SWARMSTEP_LIB=$PWD/build/variants/lib_all6.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_philox.py \
    -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_all6.log 2>&1
  echo "all6 parity rc=$?"; tail -3 $OUT/pytest_all6.log
fi
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
RC=$?; tail -3 $OUT/pytest_gpu.log; grep '^FAILED' $OUT/pytest_gpu.log | head -20
# 1 = tests failed (numerics): the bench still runs; anything else (timeout, crash) ends the script
[ $RC -gt 1 ] && { echo "pytest rc=$RC"; exit 3; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 4; }
echo "smoke ok"
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 5; }
tail -1 $OUT/bench.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 6; }
tail -1 $OUT/bench_driver.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1 || { tail -20 $OUT/prof_driver.log; exit 7; }
tail -1 $OUT/prof_driver.log
find $OUT/prof_driver -name "*kernel_trace*" -delete
echo "R4A_DONE pytest rc=$RC"
