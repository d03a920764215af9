#!/bin/bash
# HEAD: one measured training iteration per config (C5, C4, C3) through the trainer's own train().
set -u
OUT=gpurun_out/r06s37
mkdir -p $OUT
for c in C5 C4 C3; do
  timeout -k 10 600 python3 -u tools/train_iteration.py --config $c > $OUT/train_iteration_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"; tail -n 1 $OUT/train_iteration_$c.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
