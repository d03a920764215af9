#!/bin/bash
# Round-4: one measured training iteration each of C3 and C5 at their per-GPU env counts
# (tools/train_iteration.py through the trainers' own train()), peak HBM recorded.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${ITER:-C5 C3}; do
  timeout -k 10 560 python3 -u tools/train_iteration.py --config $cfg --out $OUT/train_iteration.jsonl \
    > $OUT/train_iteration_$cfg.log 2>&1 || { echo "train iteration $cfg failed"; tail -8 $OUT/train_iteration_$cfg.log; exit 5; }
  tail -1 $OUT/train_iteration_$cfg.log | cut -c1-700
done
echo R4N_DONE
