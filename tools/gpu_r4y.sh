#!/bin/bash
# Round-4: split-row weight gradients for the one-step LSTM ([x | h0] [W_ih | W_hh]^T as one product)
# and the OC2 option heads over >= 8,192 rows: LSTM / OC2 GPU tests, C5 / C4 / C3 optimizer steps.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r4y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_lstm_seq.py tests/test_gpu_oc2_trainer.py tests/test_gpu_oc2terms.py tests/test_gpu_oc_trainer.py \
  > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -ne 0 ] && exit 3
for cfg in ${CFGS:-C5 C4 C3}; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/$cfg.log; exit 4; }
  grep '^{' $OUT/$cfg.log | tail -1 > $OUT/bench_train_$cfg.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
done
SWARM_GRAPHS=0 timeout -k 10 300 python3 -u tools/prof_train.py --config C5 --steps 3 > $OUT/prof_C5.txt 2>&1 || { tail -5 $OUT/prof_C5.txt; exit 5; }
tail -1 $OUT/prof_C5.txt
echo "R4Y_DONE"
