#!/bin/bash
# Round-4: torch.profiler of eager C5 / C3 optimizer steps: top device ops, by input shape, and the
# glue ops (fill / copy / add / cat) with their Python call sites (tools/prof_train.py --stack).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4x
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in C5 C3; do
  SWARM_GRAPHS=0 timeout -k 10 300 python3 -u tools/prof_train.py --config $cfg --steps 3 --stack > $OUT/prof_$cfg.txt 2>&1 \
    || { echo "prof $cfg failed"; tail -5 $OUT/prof_$cfg.txt; exit 3; }
  tail -3 $OUT/prof_$cfg.txt
done
echo R4X_DONE
