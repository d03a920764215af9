#!/bin/bash
# End-of-round measurements on one MI355X: the bench line (default and the driver's short
# arguments), the rocprofv3 kernel-trace summary of each of the same commands, and the PMC
# passes of the step kernel (tools/pmc.sh -> pmc_traffic.json). Every GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log > $OUT/bench_line.json
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 4; }
tail -1 $OUT/bench_driver.log > $OUT/bench_driver_line.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1 || { tail -20 $OUT/prof_driver.log; exit 6; }
# keep the summaries, drop the per-dispatch traces (merge-back size)
find $OUT/prof $OUT/prof_driver -name "*kernel_trace*" -delete
bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 7; }
find gpurun_out/pmc -name "*counter_collection*" -size +20M -delete
echo GPU_FINAL_DONE
