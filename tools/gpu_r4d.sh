#!/bin/bash
# Round-4 diagnosis of the sequence-length-128 trainer fixtures on one MI355X: per-gradient
# errors of the OC2 and POCA L128 teacher-forced updates with the fused paths on / off.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/l128_diag.py --which ${WHICH:-both} > $OUT/l128_diag.jsonl 2> $OUT/l128_diag.err \
  || { echo "l128 diag failed"; tail -5 $OUT/l128_diag.err; exit 3; }
cut -c1-700 $OUT/l128_diag.jsonl
echo R4D_DONE
