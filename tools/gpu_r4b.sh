#!/bin/bash
# Round-4 session B on one MI355X: the optimizer-step bench per config (CONFIGS), the kernel
# count of an OC2 optimizer step and the GEMM shapes of the C3 decision loop (unless SKIP_PROF),
# then ONE measured training iteration (train(), rollout to
# the trigger + the whole update) of each ITER_CONFIGS config at its per-GPU env count (tools/train_iteration.py).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${CONFIGS-C3 C4 C5}; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/bench_train_$cfg.log 2>&1 \
    || { echo "bench train $cfg failed"; tail -5 $OUT/bench_train_$cfg.log; exit 4; }
  grep '^{' $OUT/bench_train_$cfg.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'ms/opt-step %.3f' % d['ms_per_optimizer_step'], 'ms/decision %.3f' % d['ms_per_decision'], 'graphed', d['graphed_steps'], 'peak GB %.1f' % d['peak_mem_gb'])"
done
# kernels per OC2 optimizer step (C5): two profiled runs of 4 and 12 steps, the difference / 8
if [ -z "${SKIP_PROF:-}" ]; then
for n in 4 12; do
  PROF_TRAIN_NOPROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_C5_$n -o run --output-format csv \
    -- python3 tools/prof_train.py --config C5 --steps $n > $OUT/prof_C5_$n.log 2>&1 || { echo "prof C5 $n failed"; tail -5 $OUT/prof_C5_$n.log; exit 6; }
  find $OUT/prof_C5_$n -name "*kernel_trace*" -delete
done
python3 - <<'PY'
import csv, glob
def total(n):
    f = glob.glob(f"gpurun_out/r4b/prof_C5_{n}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    return sum(int(r["Calls"]) for r in rows), sum(float(r["TotalDurationNs"]) for r in rows)
(c4, t4), (c12, t12) = total(4), total(12)
print(f"C5 kernels per optimizer step {(c12 - c4) / 8:.1f}, device time per step {(t12 - t4) / 8 / 1e6:.3f} ms")
PY
# the library GEMM shapes of the C3 decision loop (hipBLASLt's own log)
HIPBLASLT_LOG_MASK=32 HIPBLASLT_LOG_FILE=$OUT/hipblaslt_collect_%i.log ROCBLAS_LAYER=2 ROCBLAS_LOG_BENCH_PATH=$OUT/rocblas_collect_%i.log timeout -k 10 300 python3 bench.py --collect \
  --decisions 4 --ref-decisions 0 > $OUT/collect_log.log 2>&1 || { echo "collect log failed"; tail -5 $OUT/collect_log.log; exit 7; }
fi
for cfg in ${ITER_CONFIGS-C4 C3}; do
  timeout -k 10 600 python3 -u tools/train_iteration.py --config $cfg --out $OUT/train_iteration.jsonl \
    > $OUT/train_iteration_$cfg.log 2>&1 || { echo "train iteration $cfg failed"; tail -8 $OUT/train_iteration_$cfg.log; exit 5; }
  tail -1 $OUT/train_iteration_$cfg.log | cut -c1-600
done
echo R4B_DONE
