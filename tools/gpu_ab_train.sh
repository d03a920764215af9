#!/bin/bash
# A/B of one trainer switch on the same box: the trainer / loss / entity GPU tests, then
# bench.py --train per config with $AB_VAR=1 and =0. Each GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
VAR=${AB_VAR:-SWARM_FUSED_ENTITIES}
timeout -k 10 600 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_entity.py tests/test_gpu_ppoloss.py tests/test_gpu_setnorm.py tests/test_gpu_trainer.py \
  tests/test_gpu_oc_trainer.py tests/test_gpu_oc2_trainer.py tests/test_gpu_graph_step.py > $OUT/pytest.log 2>&1
RC=$?; tail -3 $OUT/pytest.log; [ $RC -eq 0 ] || { echo "pytest rc=$RC"; exit 3; }
for cfg in ${CONFIGS:-C3 C4 C5}; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/bench_${cfg}_$v.log 2>&1 \
      || { echo "bench $cfg $VAR=$v failed"; tail -5 $OUT/bench_${cfg}_$v.log; exit 4; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_${cfg}_$v.log') if l.startswith('{')][-1]); print('$cfg $VAR=$v ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
  done
done
echo AB_DONE
