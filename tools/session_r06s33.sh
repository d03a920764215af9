set -o pipefail
OUT=gpurun_out/r06s33; mkdir -p $OUT
# side-stream OC2 step with keep-alive instead of record_stream: repeated graph tests; stop at the first abort
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_step.py -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "oc2" > $OUT/rep${rep}.log 2>&1
  RC=$?
  echo "rep $rep rc=$RC $(tail -n 1 $OUT/rep${rep}.log)"; grep -E "side stream\]|^E .*Assertion|^FAILED" $OUT/rep${rep}.log | head -n 4
  if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then echo "abort/timeout: stopping"; exit 3; fi
done
