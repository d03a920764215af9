set -o pipefail
mkdir -p gpurun_out/r06s25
# layout 203: the wall-segment proximity rays evaluated by the physics wave and handed over (pw1)
SWARMSTEP_LIB=$PWD/build/variants/lib_pw1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s25/pytest_pw1.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s25/pytest_pw1.log; grep -E "^FAILED" gpurun_out/r06s25/pytest_pw1.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s25/groups REPS=3 KS="2" LAYOUTS="0" VLIBS="product build/variants/lib_pw1.so" bash tools/groups_sweep.sh || exit 4
