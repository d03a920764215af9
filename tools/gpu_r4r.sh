#!/bin/bash
# Round-4: LSTM kernels with LDS-broadcast packed FMAs against the readlane build (bitwise + time,
# tools/lstm_ab.py), then the C5 LSTM launch trace (gpu_r4q.sh) and the HEAD validation (gpu_r4k.sh).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python3 -u tools/lstm_ab.py build/variants7/lib_lstm0.so build/variants7/lib_lstmpk.so \
  > $OUT/lstm_ab.jsonl 2>&1; RC=$?; cat $OUT/lstm_ab.jsonl | cut -c1-200
[ $RC -ne 0 ] && { echo "lstm_ab rc=$RC"; exit 3; }
bash tools/gpu_r4q.sh && bash tools/gpu_r4k.sh
