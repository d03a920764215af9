#!/bin/bash
# One GPU session: build, GPU parity tests, smoke, bench, rocprof kernel-trace stats.
# Every GPU step has its own time limit. A crash / abort / time-out of any GPU
# step ends the script; plain parity-test failures (pytest rc 1) are reported
# and the bench still runs (it is a separate measurement).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
python3 -c "import torch; print('torch', torch.__version__, 'gpu', torch.cuda.get_device_name(0))" > gpurun_out/env.log 2>&1 || exit 1
test -f swarmacb-isaaclab_amd/SwarmACB_isaac/libswarmstep.so && test -f oracle/liboracle.so || { echo "prebuilt libraries missing: run __graft_entry__.build() before gpurun"; exit 2; }
TEST_RC=0
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  timeout -k 10 900 python3 -m pytest tests ${PYTEST_ARGS:--x} -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
  TEST_RC=$?
  tail -30 gpurun_out/pytest_gpu.log
  if [ $TEST_RC -ne 0 ] && [ $TEST_RC -ne 1 ]; then echo "pytest rc=$TEST_RC: stopping"; exit 3; fi
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  RC=$?
  tail -5 gpurun_out/smoke.log
  if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then echo "smoke rc=$RC: stopping"; exit 4; fi
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 5; }
  tail -1 gpurun_out/bench.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 6; }
  find gpurun_out/prof -name "*stats*"
fi
echo "GPU_ROUND_DONE test_rc=$TEST_RC"
