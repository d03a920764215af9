set -o pipefail
mkdir -p gpurun_out/r06s6
# product (layout 203 at 5 waves per SIMD): the pipelined layout, split steps and collector stay bitwise
# pair-compaction variant: the step parity suites against the oracle / reference fixtures
SWARMSTEP_LIB=$PWD/build/variants/lib_pc.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_philox.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06s6/pytest_pc.log 2>&1
RC=$?; tail -2 gpurun_out/r06s6/pytest_pc.log; grep -E "^FAILED" gpurun_out/r06s6/pytest_pc.log | head -3
OUT=gpurun_out/r06s6/groups REPS=3 KS="1 2" LAYOUTS="0" VLIBS="product build/variants/lib_pc.so" bash tools/groups_sweep.sh || exit 4
