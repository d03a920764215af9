#!/bin/bash
# Trainer-kernel GPU session: the trainer / attention / norm GPU tests, the optimizer-step bench
# (bench.py --train) per config with the fused norms on and off, and torch-profiler tables of the
# eager optimizer steps (tools/prof_train.py). Each GPU step has its own time limit; a crash, abort
# or time-out ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/train
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_setnorm.py tests/test_gpu_attn.py tests/test_gpu_trainer.py tests/test_gpu_oc_trainer.py \
    tests/test_gpu_oc2_trainer.py tests/test_gpu_graph_step.py tests/test_gpu_lstm_seq.py ${PYTEST_EXTRA:-} \
    > $OUT/pytest.log 2>&1
  RC=$?
  tail -4 $OUT/pytest.log
  if [ $RC -ne 0 ]; then echo "pytest rc=$RC"; exit 3; fi
fi
for cfg in ${CONFIGS:-C3 C5}; do
  for fused in ${NORMS:-1 0}; do
    SWARM_FUSED_NORMS=$fused timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/bench_${cfg}_norms$fused.log 2>&1 \
      || { echo "bench $cfg norms=$fused failed"; tail -5 $OUT/bench_${cfg}_norms$fused.log; exit 4; }
    python3 - "$OUT/bench_${cfg}_norms$fused.log" "$cfg" "$fused" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[2], "norms", sys.argv[3], "ms/opt-step", d.get("ms_per_optimizer_step", d.get("value")))
PY
  done
done
if [ "${PROF:-1}" = 1 ]; then
  for cfg in ${PROF_CONFIGS:-C3 C5}; do
    timeout -k 10 300 python3 tools/prof_train.py --config $cfg --steps 3 > $OUT/prof_$cfg.txt 2>&1 \
      || { echo "prof $cfg failed"; tail -5 $OUT/prof_$cfg.txt; exit 5; }
  done
fi
echo GPU_TRAIN_DONE
