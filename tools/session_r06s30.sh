set -o pipefail
OUT=gpurun_out/r06s30; mkdir -p $OUT
# OC2 device step with the critics' branch on a side stream: the trainer fixtures and graph tests, then the C5 A/B
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_oc2_trainer.py tests/test_gpu_graph_step.py tests/test_gpu_oc2terms.py tests/test_gpu_rccl_graph.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_oc2_streams.log 2>&1
RC=$?; tail -n 2 $OUT/pytest_oc2_streams.log; grep -E "^FAILED" $OUT/pytest_oc2_streams.log | head -3; [ $RC -ne 0 ] && exit 3
for rep in 1 2; do
  for cs in 0 1; do
    SWARM_OC2_CRITIC_STREAM=$cs timeout -k 10 400 python3 bench.py --train --config C5 > $OUT/train_C5_cs${cs}_$rep.log 2>&1 || { tail -n 5 $OUT/train_C5_cs${cs}_$rep.log; exit 4; }
    grep '^{' $OUT/train_C5_cs${cs}_$rep.log | tail -n 1 > $OUT/bench_train_C5_cs${cs}_$rep.jsonl
    python3 -c "import json; d=json.loads(open('$OUT/bench_train_C5_cs${cs}_$rep.jsonl').read()); print('rep $rep critic_stream=$cs ms/opt-step %.3f' % d['ms_per_optimizer_step'], d.get('step_path'))"
  done
done
