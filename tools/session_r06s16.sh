set -o pipefail
mkdir -p gpurun_out/r06s16
# layout-203 wave priority: the observation wave mirrors the physics wave's level (pm1), or no bumps (pm2)
SWARMSTEP_LIB=$PWD/build/variants/lib_pm1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s16/pytest_pm1.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s16/pytest_pm1.log; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s16/groups REPS=3 KS="2" LAYOUTS="0" VLIBS="product build/variants/lib_pm1.so build/variants/lib_pm2.so" bash tools/groups_sweep.sh || exit 4
