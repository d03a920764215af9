#!/bin/bash
# HEAD: the trainers' MFMA PMC tables (C3, C4, C5), then the multi-rank launcher rehearsed with
# gloo ranks sharing the one GPU (2 and 4 ranks; RCCL refuses a shared device).
set -u
TAG=r06s38 CFGS="C3 C4 C5" STEPS="pmctrain" bash tools/gpu_steps.sh || exit $?
OUT=gpurun_out/r06s38
for n in 2 4; do
  timeout -k 10 300 python3 bench.py --gpus $n --dist-backend gloo --cpu-seconds 0 > $OUT/bench_gpus${n}_gloo_one_gpu.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -n 5 $OUT/bench_gpus${n}_gloo_one_gpu.log; exit $rc; fi
  grep '^{' $OUT/bench_gpus${n}_gloo_one_gpu.log | tail -n 1 > $OUT/bench_gpus${n}_gloo_one_gpu.json
  python3 -c "import json; d=json.load(open('$OUT/bench_gpus${n}_gloo_one_gpu.json')); print('$n ranks on one GPU', d['n_gpus'], d['ranks'], d['ranks_per_device'], '%.3g' % d['value'])"
done
