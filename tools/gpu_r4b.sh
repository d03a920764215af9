#!/bin/bash
# Round-4 session B on one MI355X: the OC2 fused-term tests and the trainers' GPU parity tests,
# the optimizer-step bench per config, then ONE measured training iteration (train(), rollout to
# the trigger + the whole update) of C4 and C3 at their per-GPU env counts (tools/train_iteration.py).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_oc2terms.py tests/test_gpu_oc2_trainer.py tests/test_gpu_trainer.py tests/test_gpu_oc_trainer.py \
  tests/test_gpu_graph_step.py tests/test_gpu_rccl_graph.py tests/test_gpu_rollout.py > $OUT/pytest.log 2>&1
RC=$?; tail -4 $OUT/pytest.log
[ $RC -ne 0 ] && { echo "pytest rc=$RC"; exit 3; }
for cfg in ${CONFIGS:-C3 C4 C5}; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/bench_train_$cfg.log 2>&1 \
    || { echo "bench train $cfg failed"; tail -5 $OUT/bench_train_$cfg.log; exit 4; }
  grep '^{' $OUT/bench_train_$cfg.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'ms/opt-step %.3f' % d['ms_per_optimizer_step'], 'ms/decision %.3f' % d['ms_per_decision'], 'graphed', d['graphed_steps'], 'peak GB %.1f' % d['peak_mem_gb'])"
done
for cfg in ${ITER_CONFIGS:-C4 C3}; do
  timeout -k 10 600 python3 -u tools/train_iteration.py --config $cfg --out $OUT/train_iteration.jsonl \
    > $OUT/train_iteration_$cfg.log 2>&1 || { echo "train iteration $cfg failed"; tail -8 $OUT/train_iteration_$cfg.log; exit 5; }
  tail -1 $OUT/train_iteration_$cfg.log | cut -c1-600
done
echo R4B_DONE
