#!/bin/bash
# Round-3 end-of-round evidence at HEAD on one MI355X: the GPU suite + smoke, the bench of
# record (default and driver arguments) with rocprofv3 stats and PMC passes (tools/gpu_final.sh),
# the C3/C4/C5 optimizer-step bench and the critic bench. Each GPU step has its own time limit;
# the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SKIP_VARIANTS=1 bash tools/gpu_session.sh || exit 2
bash tools/gpu_final.sh || exit 3
SKIP_TESTS=1 PROF=0 NORMS=1 CONFIGS="C3 C4 C5" bash tools/gpu_train_session.sh || exit 4
timeout -k 10 300 python3 bench.py --critic > gpurun_out/final/bench_critic.log 2>&1 || { tail -5 gpurun_out/final/bench_critic.log; exit 5; }
tail -3 gpurun_out/final/bench_critic.log
echo R3_FINAL_DONE
