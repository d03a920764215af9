set -o pipefail
mkdir -p gpurun_out/r06s8
# rebalanced layout-203 pipeline (SWARM_PIPE_RAB=1: range-and-bearing on the physics wave) at 5-8 waves per SIMD
# r6 (6 waves, 80 VGPRs, no spill): the pipelined layout / split-step / Philox parity suites
SWARMSTEP_LIB=$PWD/build/variants/lib_r6.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s8/pytest_r6.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s8/pytest_r6.log; grep -E "^FAILED" gpurun_out/r06s8/pytest_r6.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s8/groups REPS=2 KS="2 3" LAYOUTS="0" VLIBS="product build/variants/lib_r5.so build/variants/lib_r6.so build/variants/lib_r7.so" bash tools/groups_sweep.sh || exit 4
# r8 (64 VGPRs): one group of 4,096 arenas as 8,192 resident waves
OUT=gpurun_out/r06s8/groups1 REPS=1 KS="1" LAYOUTS="203" VLIBS="product build/variants/lib_r6.so build/variants/lib_r8.so" bash tools/groups_sweep.sh || exit 5
