set -o pipefail
# HEAD records beside the step bench: the critic bench (frac on executed flops), the C3-C5 trainers'
# optimizer steps, the C3 collector with groups, and a two-rank rehearsal of the default (2-group) bench
OUT=gpurun_out/r06s15; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --critic > $OUT/critic.log 2>&1 || { tail -n 5 $OUT/critic.log; exit 3; }
grep '^{' $OUT/critic.log | tail -n 1 > $OUT/bench_critic.jsonl
for cfg in C5 C4 C3; do
  timeout -k 10 400 python3 bench.py --train --config $cfg > $OUT/train_$cfg.log 2>&1 || { echo "train $cfg failed"; tail -n 5 $OUT/train_$cfg.log; exit 4; }
  grep '^{' $OUT/train_$cfg.log | tail -n 1 > $OUT/bench_train_$cfg.jsonl
  python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
done
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --cpu-seconds 0 > $OUT/bench_gpus2_gloo_one_gpu.log 2>&1 || { tail -n 5 $OUT/bench_gpus2_gloo_one_gpu.log; exit 5; }
grep '^{' $OUT/bench_gpus2_gloo_one_gpu.log | tail -n 1 > $OUT/bench_gpus2_gloo_one_gpu.json
python3 -c "import json; d=json.load(open('$OUT/bench_gpus2_gloo_one_gpu.json')); print('2 ranks on one GPU', d['n_gpus'], d['ranks'], d['ranks_per_device'], '%.3g' % d['value'])"
