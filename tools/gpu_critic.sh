#!/bin/bash
# GPU session for the fused critic attention: parity tests, bench, rocprof stats, MFMA PMC pass.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_critic.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_critic.log 2>&1
RC=$?
tail -20 gpurun_out/pytest_critic.log
if [ $RC -ne 0 ]; then echo "pytest rc=$RC"; exit 3; fi
timeout -k 10 300 python3 bench.py --critic > gpurun_out/bench_critic.log 2>&1 || { tail -20 gpurun_out/bench_critic.log; exit 5; }
cat gpurun_out/bench_critic.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_critic -o run --output-format csv -- \
  python3 bench.py --critic --cpu-envs 1 > gpurun_out/prof_critic.log 2>&1 || { tail -20 gpurun_out/prof_critic.log; exit 6; }
timeout -s KILL 120 rocprofv3 --kernel-include-regex "rsa_(pool|baselines)" --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_critic -o run --output-format csv -- python3 bench.py --critic --cpu-envs 1 --reps 3 \
  > gpurun_out/pmc_critic.log 2>&1 || { tail -20 gpurun_out/pmc_critic.log; exit 7; }
echo CRITIC_DONE
