#!/bin/bash
# PMC counter passes (rocprofv3 --pmc, one counter group per pass, kernel-trace
# only, no sys/runtime tracing) over a short bench run, restricted to the step
# kernel. Summarised by tools/pmc_summary.py into gpurun_out/pmc/summary.json.
# Every pass has its own time limit; the first failing pass ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
test -f swarmacb-isaaclab_amd/SwarmACB_isaac/libswarmstep.so || exit 2
ARGS="--cpu-seconds 0 --steps ${PMC_STEPS:-100} --warmup 10 --groups ${PMC_GROUPS:-2} ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || echo "rocprofv3 -L rc=$?"
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-include-regex step_kernel --pmc "$@" -d gpurun_out/pmc/$name -o run \
    --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name rc=$rc"; tail -5 gpurun_out/pmc/$name.log; exit 3; fi
  echo "pass $name ok"
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
run_pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run_pass sq3 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py gpurun_out/pmc --groups ${PMC_GROUPS:-2} --traffic-json gpurun_out/pmc/pmc_traffic.json > gpurun_out/pmc/summary.txt 2>&1 || { cat gpurun_out/pmc/summary.txt; exit 4; }
cat gpurun_out/pmc/summary.txt
echo PMC_DONE
