set -o pipefail
mkdir -p gpurun_out/r06s14
# serialised proximity rays (SWARM_PROX_SERIAL=1: the observation role fits 80 VGPRs) at 5 / 6 waves per SIMD
SWARMSTEP_LIB=$PWD/build/variants/lib_s6.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s14/pytest_s6.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s14/pytest_s6.log; grep -E "^FAILED" gpurun_out/r06s14/pytest_s6.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s14/groups REPS=2 KS="2 3" LAYOUTS="0" VLIBS="product build/variants/lib_s5.so build/variants/lib_s6.so build/variants/lib_p6.so" bash tools/groups_sweep.sh || exit 4
