set -o pipefail
mkdir -p gpurun_out/r06s2
# (tests ran green: 15 passed)
: timeout -k 10 600 python3 -u -m pytest tests/test_gpu_philox.py tests/test_gpu_glue.py tests/test_gpu_oc2terms.py -k "streams or groups or collector or input_checks" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s2/pytest.log 2>&1
: 
OUT=gpurun_out/r06s2/groups REPS=2 KS="1 2 3" LAYOUTS="0 203" bash tools/groups_sweep.sh || exit 4
for k in 1 2 1 2; do timeout -k 10 180 python3 bench.py --collect --variant dandelion --envs 4096 --decisions 48 --groups $k 2>&1 | grep '^{' | tee -a gpurun_out/r06s2/collect_dandelion.jsonl || exit 5; done
