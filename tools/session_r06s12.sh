set -o pipefail
mkdir -p gpurun_out/r06s12
# heaviest-first dispatch order of the layout-203 launches: the bitwise tests, then the A/B
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s12/pytest_order.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s12/pytest_order.log; grep -E "^FAILED" gpurun_out/r06s12/pytest_order.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s12/order REPS=2 KS="2 3" LAYOUTS="0" ORDERS="0 6 10 14" bash tools/groups_sweep.sh || exit 4
