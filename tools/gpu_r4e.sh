#!/bin/bash
# Round-4 check on one MI355X after the LSTM activation / parity-envelope / bench-gate changes:
# the affected GPU tests, smoke, the bench (default and the driver's arguments) and the rocprofv3
# kernel stats of the driver's command. Each GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_lstm_seq.py tests/test_gpu_philox.py "tests/test_gpu_trainer.py" "tests/test_gpu_oc2_trainer.py" \
  -k "lstm or L128 or philox or order or production or groups or partial" > $OUT/pytest.log 2>&1
RC=$?; tail -3 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -gt 1 ] && { echo "pytest rc=$RC"; exit 3; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 4; }
echo "smoke ok"
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 5; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 6; }
python3 -c "import json; d=json.loads(open('$OUT/bench_driver.log').read().strip().splitlines()[-1]); print('driver args value %.4g kernel_us %.2f' % (d['value'], d['roofline']['kernel_avg_us']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1 || { tail -20 $OUT/prof_driver.log; exit 7; }
find $OUT/prof_driver -name "*kernel_trace*" -delete
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4e/prof_driver/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "step_kernel" in r["Name"]:
        print("rocprof step_kernel calls", r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
echo "R4E_DONE pytest rc=$RC"
