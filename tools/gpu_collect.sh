#!/bin/bash
# GPU session for the C3 rollout decision loop: critic + glue parity tests, the
# end-to-end bench (this build vs the reference loop on the same GPU), rocprof stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_critic.py tests/test_gpu_glue.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_collect.log 2>&1
RC=$?
tail -5 gpurun_out/pytest_collect.log
if [ $RC -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/pytest_collect.log | head -20; echo "pytest rc=$RC"; exit 3; fi
timeout -k 10 300 python3 -u bench.py --collect > gpurun_out/bench_collect.log 2>&1 || { tail -20 gpurun_out/bench_collect.log; exit 5; }
grep rollout_decision gpurun_out/bench_collect.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_collect -o run --output-format csv -- \
  python3 -u bench.py --collect --ref-decisions 0 > gpurun_out/prof_collect.log 2>&1 || { tail -20 gpurun_out/prof_collect.log; exit 6; }
find gpurun_out/prof_collect -name "*kernel_trace.csv" -delete
echo COLLECT_DONE
