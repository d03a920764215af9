set -o pipefail
mkdir -p gpurun_out/r06s7
# the rebalanced pipeline (range-and-bearing on the physics wave): layout 203 == 103 bitwise, split steps
SWARMSTEP_LIB=$PWD/build/variants/lib_r6.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -k "pipe or streams or groups or production or c2" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s7/pytest_r6.log 2>&1
RC=$?; tail -2 gpurun_out/r06s7/pytest_r6.log; grep -E "^FAILED" gpurun_out/r06s7/pytest_r6.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s7/groups REPS=2 KS="2 3" LAYOUTS="0" VLIBS="product build/variants/lib_r5.so build/variants/lib_r6.so build/variants/lib_r7.so" bash tools/groups_sweep.sh || exit 4
