#!/bin/bash
# A/B: shorter split-row chunks for narrow layers (SWARM_SPLITK_NARROW_ROWS) in the optimizer steps.
# The trainer GPU tests with the variant on, then bench.py --train alternating off / on per config.
set -u
OUT=gpurun_out/r06s40
mkdir -p $OUT
SWARM_SPLITK_NARROW_ROWS=256 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_trainer.py tests/test_gpu_oc_trainer.py tests/test_gpu_oc2_trainer.py tests/test_gpu_graph_step.py \
  > $OUT/pytest_narrow256.txt 2>&1
rc=$?; tail -n 3 $OUT/pytest_narrow256.txt
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # cfg rows rep
  SWARM_SPLITK_NARROW_ROWS=$2 timeout -k 10 300 python3 bench.py --train --config $1 > $OUT/train_$1_n$2_$3.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "train $1 n$2 rc=$rc"; tail -n 5 $OUT/train_$1_n$2_$3.log; exit $rc; fi
  grep '^{' $OUT/train_$1_n$2_$3.log | tail -n 1 > $OUT/bench_train_$1_n$2_$3.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$1_n$2_$3.jsonl').read()); print('$1 narrow=$2 rep $3 ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
}
for rep in 1 2; do
  for n in 0 256 128; do run C3 $n $rep; done
done
for rep in 1 2; do
  for n in 0 256; do run C5 $n $rep; run C4 $n $rep; done
done
