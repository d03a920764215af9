set -o pipefail
OUT=gpurun_out/r06s32; mkdir -p $OUT
# repeated: the OC2 graphed-vs-eager test and the side-stream-vs-serial bitwise test, side stream on / off
for rep in 1 2 3 4; do
  for cs in 1 0; do
    SWARM_OC2_CRITIC_STREAM=$cs timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_step.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "oc2" > $OUT/rep${rep}_cs${cs}.log 2>&1
    echo "rep $rep cs $cs rc=$? $(tail -n 1 $OUT/rep${rep}_cs${cs}.log)"
    grep -E "^E .*Assertion|^FAILED" $OUT/rep${rep}_cs${cs}.log | head -n 3
  done
done
