#!/bin/bash
# Round-4: the focal counterfactual sets on shared rows (swarm_rsa_pool_focal): the critic and
# option-critic trainer GPU tests, the C5 / C4 optimizer steps, and the C5 trace rows.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_critic.py tests/test_gpu_oc2_trainer.py tests/test_gpu_oc_trainer.py tests/test_gpu_rollout.py \
  > $OUT/pytest.log 2>&1
RC=$?; tail -2 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
[ $RC -gt 1 ] && exit 3
for cfg in C5 C4; do
  timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 $OUT/$cfg.log; exit 4; }
  grep '^{' $OUT/$cfg.log | tail -1 > $OUT/bench_train_$cfg.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'], 'ms/decision %.3f' % d['ms_per_decision'])"
done
bash tools/gpu_r4q.sh
echo "R4T_DONE pytest rc=$RC"
