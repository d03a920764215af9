set -o pipefail
mkdir -p gpurun_out/r06s3
OUT=gpurun_out/r06s3/groups REPS=2 KS="1 2 3 4 6" LAYOUTS="0 203" bash tools/groups_sweep.sh || exit 4
for k in 1 2 3 1 2 3; do timeout -k 10 180 python3 bench.py --collect --variant dandelion --envs 4096 --decisions 48 --groups $k 2>&1 | grep '^{' | tee -a gpurun_out/r06s3/collect_dandelion.jsonl || exit 5; done
