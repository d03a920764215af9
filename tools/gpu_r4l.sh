#!/bin/bash
# Round-4 trainer study on one MI355X: the C5 OC2 optimizer step with and without the fused OC2
# term kernels (alternating twice), the LSTM sequence micro-benchmark, then the kernel count of an
# OC2 optimizer step and the GEMM shapes of the C3 decision loop (tools/gpu_r4b.sh prof part).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4l
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for terms in 1 0; do
    SWARM_FUSED_OC2_TERMS=$terms timeout -k 10 300 python3 bench.py --train --config C5 > $OUT/c5_terms${terms}_$rep.log 2>&1 \
      || { echo "C5 terms=$terms failed"; tail -5 $OUT/c5_terms${terms}_$rep.log; exit 3; }
    grep '^{' $OUT/c5_terms${terms}_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 fused_terms=$terms rep $rep ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
  done
done
timeout -k 10 300 python3 tools/lstm_micro.py > $OUT/lstm_micro.jsonl 2> $OUT/lstm_micro.err || { tail -5 $OUT/lstm_micro.err; exit 4; }
head -4 $OUT/lstm_micro.jsonl | cut -c1-300
CONFIGS= ITER_CONFIGS= bash tools/gpu_r4b.sh || exit 5
echo R4L_DONE
