set -o pipefail
mkdir -p gpurun_out/r06s4
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_philox.py tests/test_gpu_glue.py -k "streams or groups or collector" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s4/pytest.log 2>&1
RC=$?; tail -3 gpurun_out/r06s4/pytest.log; [ $RC -ne 0 ] && exit 3
OUT=gpurun_out/r06s4/groups REPS=2 KS="1 2 3" LAYOUTS="0" VLIBS="product build/variants/lib_p5.so build/variants/lib_p6.so" bash tools/groups_sweep.sh || exit 4
