set -o pipefail
OUT=gpurun_out/r06s35; mkdir -p $OUT
# POCA / OC steps with the critic branch on a side stream: trainer fixtures + graphed==eager (3x), then C3 / C4 A/B
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_oc_trainer.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_trainers.log 2>&1
RC=$?; echo "trainer fixtures rc=$RC $(tail -n 1 $OUT/pytest_trainers.log)"; grep -E "^FAILED" $OUT/pytest_trainers.log | head -n 3
[ $RC -ne 0 ] && exit 3
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_step.py -q -s -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/graph_rep${rep}.log 2>&1
  RC=$?
  echo "graph rep $rep rc=$RC $(tail -n 1 $OUT/graph_rep${rep}.log)"; grep -E "\[graph\]|^E .*Assertion|^FAILED" $OUT/graph_rep${rep}.log | head -n 8
  if [ $RC -ne 0 ]; then exit 4; fi
done
for cfg in C3 C4; do
  for cs in 0 1; do
    SWARM_CRITIC_STREAM=$cs timeout -k 10 400 python3 bench.py --train --config $cfg > $OUT/train_${cfg}_cs$cs.log 2>&1 || { tail -n 5 $OUT/train_${cfg}_cs$cs.log; exit 5; }
    grep '^{' $OUT/train_${cfg}_cs$cs.log | tail -n 1 > $OUT/bench_train_${cfg}_cs$cs.jsonl
    python3 -c "import json; d=json.loads(open('$OUT/bench_train_${cfg}_cs$cs.jsonl').read()); print('$cfg critic_stream=$cs ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
  done
done
