#!/bin/bash
# One GPU session of variant timing + the GPU suite: bench each build/variants/lib_*.so
# (tools/variants.sh run), then pytest -m gpu and smoke() on the in-tree library.
# Every GPU step has its own time limit; a crash / abort / time-out ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if ls build/variants/lib_*.so > /dev/null 2>&1 && [ "${SKIP_VARIANTS:-0}" != 1 ]; then
  bash tools/variants.sh run || { echo "variants failed"; exit 2; }
fi
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_SEL:-} > gpurun_out/pytest_gpu.log 2>&1
  RC=$?
  tail -5 gpurun_out/pytest_gpu.log
  if [ $RC -ne 0 ]; then echo "pytest rc=$RC"; exit 3; fi
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 4; }
  echo "smoke ok"
fi
echo GPU_SESSION_DONE
