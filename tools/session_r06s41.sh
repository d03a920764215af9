#!/bin/bash
# Packed-fp32 disc rays (SWARM_PK_DISC=1): the pipe / Philox parity suites on the variant library,
# then the default bench alternating the product library / the variant (3 reps).
set -u
OUT=gpurun_out/r06s41
mkdir -p $OUT
SWARMSTEP_LIB=$PWD/build/variants/lib_pkdisc.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_pkdisc.log 2>&1
RC=$?; tail -n 2 $OUT/pytest_pkdisc.log; grep -E "^FAILED" $OUT/pytest_pkdisc.log | head -3
if [ $RC -ne 0 ]; then exit 3; fi
for rep in 1 2 3; do
  for v in base pkdisc; do
    if [ $v = base ]; then unset SWARMSTEP_LIB; else export SWARMSTEP_LIB=$PWD/build/variants/lib_pkdisc.so; fi
    timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 1200 > $OUT/bench_${v}_$rep.log 2>&1 \
      || { echo "$v rep $rep failed"; tail -n 5 $OUT/bench_${v}_$rep.log; exit 4; }
    grep '^{' $OUT/bench_${v}_$rep.log | tail -n 1 > $OUT/bench_${v}_$rep.json
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$rep.json')); print('rep $rep $v value %.4g' % d['value'], 'launch_us', d['roofline'].get('launch_avg_us_per_stream'), 'sha', d['roofline']['lib_sha256'][:8])"
  done
done
