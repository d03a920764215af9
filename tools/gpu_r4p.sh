#!/bin/bash
# Round-4: the OC2 termination advantage reads Q(s', omega) from the focal counterfactual row
# (one critic pass fewer): the OC2 trainer GPU tests, then the C5 optimizer step and its kernels.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_oc2_trainer.py > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -gt 1 ] && exit 3
timeout -k 10 300 python3 bench.py --train --config C5 > $OUT/c5.log 2>&1 || { echo "C5 failed"; tail -5 $OUT/c5.log; exit 4; }
grep '^{' $OUT/c5.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C5 -o run --output-format csv \
  -- python3 bench.py --train --config C5 > $OUT/prof_C5.log 2>&1 || { tail -5 $OUT/prof_C5.log; exit 5; }
find $OUT/prof_C5 -name "*kernel_trace*" -delete
echo "R4P_DONE pytest rc=$RC"
