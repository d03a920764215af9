#!/bin/bash
# One GPU session: build, GPU parity tests, smoke, bench, rocprof kernel-trace stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
python3 -c "import torch; print('torch', torch.__version__, 'gpu', torch.cuda.get_device_name(0))" > gpurun_out/env.log 2>&1 || exit 1
make -C swarmacb-isaaclab_amd/csrc > gpurun_out/build.log 2>&1 && make -C oracle >> gpurun_out/build.log 2>&1 || exit 2
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 3; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 4; }
  tail -1 gpurun_out/smoke.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 5; }
  tail -1 gpurun_out/bench.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --steps 250 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 6; }
  find gpurun_out/prof -name "*stats*" | head
fi
echo GPU_ROUND_OK
