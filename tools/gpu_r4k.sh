#!/bin/bash
# Round-4 HEAD on one MI355X: the full GPU suite (parity stats for the envelope record), smoke,
# the bench (default, and the driver's arguments with its rocprofv3 kernel stats), then the PMC
# passes of the step kernel (tools/pmc.sh). Each GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
rm -f gpurun_out/parity_stats.jsonl
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
RC=$?; tail -3 $OUT/pytest_gpu.log; grep '^FAILED' $OUT/pytest_gpu.log | head -20
[ $RC -gt 1 ] && { echo "pytest rc=$RC"; exit 3; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 4; }
echo "smoke ok"
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 5; }
python3 -c "import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print('default value %.4g kernel_us %.2f' % (d['value'], d['roofline']['kernel_avg_us']))"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 6; }
python3 -c "import json; d=json.loads(open('$OUT/bench_driver.log').read().strip().splitlines()[-1]); print('driver args value %.4g kernel_us %.2f' % (d['value'], d['roofline']['kernel_avg_us']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1 || { tail -20 $OUT/prof_driver.log; exit 7; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv \
  -- python3 bench.py --cpu-seconds 0 > $OUT/prof_default.log 2>&1 || { tail -20 $OUT/prof_default.log; exit 8; }
find $OUT/prof_driver $OUT/prof_default -name "*kernel_trace*" -delete
python3 - <<'PY'
import csv, glob
for tag in ("driver", "default"):
    f = glob.glob(f"gpurun_out/r4k/prof_{tag}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Name"]:
            print(f"rocprof {tag} step_kernel calls", r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { tail -10 $OUT/pmc.log; exit 9; }
grep -E 'valu_insts_per_launch|hbm_bytes_per_launch|sq_wait_any_frac|sq_active_inst_valu_frac' $OUT/pmc.log | head
echo "R4K_DONE pytest rc=$RC"
