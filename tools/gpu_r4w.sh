#!/bin/bash
# Round-4: the OC2 attention-term forward one row per wave: its GPU tests and the OC2 trainer's,
# the C5 optimizer step, then the HEAD validation (gpu_r4k.sh).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_oc2terms.py tests/test_gpu_oc2_trainer.py > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -ne 0 ] && exit 3
timeout -k 10 300 python3 bench.py --train --config C5 > $OUT/C5.log 2>&1 || { echo "C5 failed"; tail -5 $OUT/C5.log; exit 4; }
grep '^{' $OUT/C5.log | tail -1 > $OUT/bench_train_C5.jsonl
python3 -c "import json; d=json.loads(open('$OUT/bench_train_C5.jsonl').read()); print('C5 ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
bash tools/gpu_r4k.sh
