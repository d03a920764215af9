#!/bin/bash
# Round-4 check of the multi-block OC2 term forwards on one MI355X: their GPU tests and the OC2
# trainer parity tests, then the C5 optimizer step (fused terms on / off) and the per-kernel time
# of an OC2 step; then one measured training iteration of C4 (tools/train_iteration.py).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_oc2terms.py tests/test_gpu_oc2_trainer.py > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -gt 1 ] && exit 3
for terms in 1 0; do
  SWARM_FUSED_OC2_TERMS=$terms timeout -k 10 300 python3 bench.py --train --config C5 > $OUT/c5_terms$terms.log 2>&1 \
    || { echo "C5 terms=$terms failed"; tail -5 $OUT/c5_terms$terms.log; exit 4; }
  grep '^{' $OUT/c5_terms$terms.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 fused_terms=$terms ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
done
CONFIGS= ITER_CONFIGS=C4 bash tools/gpu_r4b.sh > $OUT/r4b.log 2>&1 || { tail -5 $OUT/r4b.log; exit 5; }
tail -4 $OUT/r4b.log
echo "R4M_DONE pytest rc=$RC"
