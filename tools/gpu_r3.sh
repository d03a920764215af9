#!/bin/bash
# Round-3 GPU session: the new kernels' tests first (short limit), then the whole GPU
# suite + smoke, the step-kernel variants (product layout 103) and the trainer bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES=${STAGES:-"new suite variants train"}
for st in $STAGES; do
  case $st in
    new)
      timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_attn.py \
        tests/test_gpu_lstm_seq.py -s > gpurun_out/pytest_new.log 2>&1
      RC=$?; tail -15 gpurun_out/pytest_new.log
      [ $RC -eq 0 ] || { echo "new-kernel tests rc=$RC: stopping"; exit 3; } ;;
    suite)
      PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_round.sh test || exit 4 ;;
    variants)
      WAVES=103 bash tools/variants.sh run || exit 5 ;;
    train)
      timeout -k 10 900 python3 bench.py --train --config all > gpurun_out/train_bench.jsonl 2> gpurun_out/train_bench.err
      RC=$?; cat gpurun_out/train_bench.jsonl | cut -c1-200; [ $RC -eq 0 ] || { echo "train bench rc=$RC"; exit 6; } ;;
  esac
done
echo GPU_R3_DONE
