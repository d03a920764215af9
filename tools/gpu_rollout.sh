#!/bin/bash
# GPU session for the rollout-buffer kernels: parity tests, bench, rocprof stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_glue.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_rollout.log 2>&1
RC=$?
tail -30 gpurun_out/pytest_rollout.log
if [ $RC -ne 0 ]; then echo "pytest rc=$RC"; exit 3; fi
timeout -k 10 300 python3 bench.py --rollout > gpurun_out/bench_rollout.log 2>&1 || { tail -20 gpurun_out/bench_rollout.log; exit 5; }
cat gpurun_out/bench_rollout.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rollout -o run --output-format csv -- \
  python3 bench.py --rollout --cpu-envs 1 > gpurun_out/prof_rollout.log 2>&1 || { tail -20 gpurun_out/prof_rollout.log; exit 6; }
echo ROLLOUT_DONE
