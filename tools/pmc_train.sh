#!/bin/bash
# PMC passes over C3 PPO optimizer steps (tools/prof_train.py's workload without the
# torch profiler: PROF_TRAIN_NOPROF=1), one counter group per pass, kernel-trace only.
# Summarised per kernel by tools/pmc_table.py into gpurun_out/pmc_train/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_train
export TMPDIR=/tmp PROF_TRAIN_NOPROF=1
CFG=${CFG:-C3}
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/pmc_train/$name -o run --output-format csv \
    -- python3 tools/prof_train.py --config $CFG --steps 4 > gpurun_out/pmc_train/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name rc=$rc"; tail -5 gpurun_out/pmc_train/$name.log; exit 3; fi
  echo "pass $name ok"
}
run_pass mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_train/trace -o run --output-format csv \
  -- python3 tools/prof_train.py --config $CFG --steps 4 > gpurun_out/pmc_train/trace.log 2>&1 || { echo "trace failed"; exit 4; }
# summarise on the box, then drop the raw per-dispatch files (the merge-back is capped at 64 MiB)
python3 tools/pmc_train_table.py gpurun_out/pmc_train gpurun_out/pmc_train/mfma_table.csv > gpurun_out/pmc_train/mfma_table.txt || exit 5
rm -f gpurun_out/pmc_train/mfma/run_counter_collection.csv gpurun_out/pmc_train/trace/run_kernel_trace.csv
echo PMC_TRAIN_DONE
