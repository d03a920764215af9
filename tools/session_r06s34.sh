set -o pipefail
OUT=gpurun_out/r06s34; mkdir -p $OUT
# side-stream OC2 step (critic step after the counterfactual pass): the OC2 graph tests 6 times, then the C5 A/B
for rep in 1 2 3 4 5 6; do
  SWARM_OC2_CRITIC_STREAM=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_step.py -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "oc2" > $OUT/rep${rep}.log 2>&1
  RC=$?
  echo "rep $rep rc=$RC $(tail -n 1 $OUT/rep${rep}.log)"; grep -E "\[graph\] oc2|^E .*Assertion|^FAILED" $OUT/rep${rep}.log | head -n 4
  if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then echo "abort/timeout: stopping"; exit 3; fi
done
for rep in 1 2; do
  for cs in 0 1; do
    SWARM_OC2_CRITIC_STREAM=$cs timeout -k 10 400 python3 bench.py --train --config C5 > $OUT/train_C5_cs${cs}_$rep.log 2>&1 || { tail -n 5 $OUT/train_C5_cs${cs}_$rep.log; exit 4; }
    grep '^{' $OUT/train_C5_cs${cs}_$rep.log | tail -n 1 > $OUT/bench_train_C5_cs${cs}_$rep.jsonl
    python3 -c "import json; d=json.loads(open('$OUT/bench_train_C5_cs${cs}_$rep.jsonl').read()); print('rep $rep critic_stream=$cs ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
  done
done
