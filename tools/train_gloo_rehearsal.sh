#!/bin/bash
# World-2 rehearsal of the multi-GPU training entry point on ONE GPU: two ranks
# share cuda:0 (RCCL refuses two ranks per device, so the collectives run over
# gloo: SWARM_DIST_BACKEND=gloo), an odd global env count (65 -> shards of 33 and
# 32 envs), one update of each trainer kind. Every rank prints its parameter
# digest after training; TrainerBase.train() has already asserted them bitwise
# equal across the ranks.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/train_gloo
export PYTHONPATH="$PWD/swarmacb-isaaclab_amd:$PYTHONPATH" SWARM_DIST_BACKEND=gloo TMPDIR=/tmp
PORT=${PORT:-29533}
for NAME in Foraging_cyclamen OC_DirGate_cyclamen OC2_XOR_cyclamen; do
  python3 - "$NAME" > gpurun_out/train_gloo/$NAME.yaml <<'PY' || exit 2
import json, sys, yaml
raw = json.load(open("tests/golden/config/load_config.json"))[sys.argv[1] + ".yaml"]["raw"]
next(iter(raw["behaviors"].values()))["summary_freq"] = 1300
print(yaml.safe_dump(raw))
PY
  # 65 envs x 20 = 1300 experiences per decision; buffer_size 20480 -> 16 decisions
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $PORT -m SwarmACB_isaac.train --config gpurun_out/train_gloo/$NAME.yaml --num_envs 65 \
    --total_timesteps 20800 --log_dir gpurun_out/train_gloo/runs_$NAME --checkpoint_dir gpurun_out/train_gloo/ckpt_$NAME \
    --device cuda:0 > gpurun_out/train_gloo/$NAME.log 2>&1
  RC=$?
  grep "parameter digest" gpurun_out/train_gloo/$NAME.log
  if [ $RC -ne 0 ]; then echo "$NAME rc=$RC"; tail -30 gpurun_out/train_gloo/$NAME.log; exit 3; fi
  PORT=$((PORT + 1))
done
rm -rf gpurun_out/train_gloo/ckpt_*
echo TRAIN_GLOO_DONE
