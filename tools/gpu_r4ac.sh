#!/bin/bash
# Round-4: split-row weight gradients from 4,096 rows: the trainer / critic / LSTM GPU tests and
# the C3 / C4 / C5 optimizer steps.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_lstm_seq.py tests/test_gpu_oc2_trainer.py tests/test_gpu_oc_trainer.py tests/test_gpu_trainer.py \
  tests/test_gpu_critic.py tests/test_gpu_setnorm.py tests/test_gpu_graph_step.py tests/test_gpu_train_main.py > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED\|^ERROR' $OUT/pytest.log | head
[ $RC -ne 0 ] && exit 3
for cfg in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/$cfg.log; exit 4; }
  grep '^{' $OUT/$cfg.log | tail -1 > $OUT/bench_train_$cfg.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
done
echo R4AC_DONE
