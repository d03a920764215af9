#!/bin/bash
# Round-4: forward LSTM on LDS-broadcast packed FMAs (backward unchanged) and one-step recurrences
# over >= 512 rows on library GEMMs + elementwise cell terms: the LSTM / trainer GPU tests, the
# C3 / C4 / C5 optimizer steps, and the C5 LSTM launch trace.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_lstm_seq.py tests/test_gpu_oc2_trainer.py tests/test_gpu_oc_trainer.py tests/test_gpu_trainer.py \
  > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -gt 1 ] && exit 3
for cfg in C5 C3 C4; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/$cfg.log; exit 4; }
  grep '^{' $OUT/$cfg.log | tail -1 > $OUT/bench_train_$cfg.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
done
bash tools/gpu_r4q.sh
echo "R4S_DONE pytest rc=$RC"
