set -o pipefail
mkdir -p gpurun_out/r06s23
# layout-203 hand-over of the inside flags (h1) and the ray directions (h2) from the physics wave
SWARMSTEP_LIB=$PWD/build/variants/lib_h3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s23/pytest_h3.log 2>&1
RC=$?; tail -n 2 gpurun_out/r06s23/pytest_h3.log; grep -E "^FAILED" gpurun_out/r06s23/pytest_h3.log | head -3; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s23/groups REPS=3 KS="2" LAYOUTS="0" VLIBS="product build/variants/lib_h1.so build/variants/lib_h2.so build/variants/lib_h3.so" bash tools/groups_sweep.sh || exit 4
