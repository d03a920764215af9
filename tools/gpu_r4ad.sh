#!/bin/bash
# Round-4 end: the whole GPU suite and smoke() at HEAD.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
RC=$?; tail -2 $OUT/pytest_gpu.log; grep '^FAILED' $OUT/pytest_gpu.log | head
[ $RC -ne 0 ] && exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 4; }
echo "smoke ok"
