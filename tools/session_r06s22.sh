set -o pipefail
mkdir -p gpurun_out/r06s22
# layout 203 with sin / cos of the yaw handed from the physics wave to the observation wave (lib_sc)
SWARMSTEP_LIB=$PWD/build/variants/lib_sc.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s22/pytest_sc.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s22/pytest_sc.log; grep -E "^FAILED" gpurun_out/r06s22/pytest_sc.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s22/groups REPS=3 KS="2" LAYOUTS="0" VLIBS="product build/variants/lib_sc.so" bash tools/groups_sweep.sh || exit 4
