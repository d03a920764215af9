#!/bin/bash
# Round-4: SPLITK_MIN_ROWS 8192 (HEAD) vs 4096 on the C3 / C4 / C5 optimizer steps, alternating, twice.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4ab
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in C3 C4 C5; do
    for rows in 8192 4096; do
      timeout -k 10 300 python3 tools/splitk_rows_ab.py $rows --config $cfg > $OUT/${cfg}_${rows}_$rep.log 2>&1 \
        || { echo "$cfg $rows failed"; tail -5 $OUT/${cfg}_${rows}_$rep.log; exit 3; }
      grep '^{' $OUT/${cfg}_${rows}_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg rows $rows rep $rep ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
    done
  done
done
echo R4AB_DONE
