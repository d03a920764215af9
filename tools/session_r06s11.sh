set -o pipefail
# (1) step-kernel throughput at saturation: layouts 103 / 203 at 8,192 and 16,384 envs, 1-4 groups
mkdir -p gpurun_out/r06s11
for cfg in "16384 1 103" "16384 1 203" "16384 2 0" "16384 4 0" "8192 1 103" "8192 2 0" "8192 4 0"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --cpu-seconds 0 --envs $1 --groups $2 --layout $3 --steps 600 > gpurun_out/r06s11/sat_$1_$2_$3.log 2>&1 \
    || { echo "bench $cfg failed"; tail -n 5 gpurun_out/r06s11/sat_$1_$2_$3.log; exit 3; }
  grep '^{' gpurun_out/r06s11/sat_$1_$2_$3.log | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']
print(json.dumps({'envs': $1, 'groups': $2, 'layout_arg': $3, 'layout': r['layout'], 'value': d['value'], 'decision_us': r['kernel_avg_us'],
                  'ns_per_arena': r['kernel_avg_us'] * 1e3 / $1}))" | tee -a gpurun_out/r06s11/saturation.jsonl
done
# (2) the C5 optimizer step's kernel mix at HEAD (graphed steps, two step counts, rocprofv3 stats)
export TMPDIR=/tmp
for n in 4 12; do
  PROF_TRAIN_NOPROF=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06s11/mix_$n -o run --output-format csv \
    -- python3 tools/prof_train.py --config C5 --steps $n > gpurun_out/r06s11/mix_$n.log 2>&1 || { tail -n 5 gpurun_out/r06s11/mix_$n.log; exit 4; }
  find gpurun_out/r06s11/mix_$n -name "*kernel_trace*" -delete
done
python3 tools/step_kernel_diff.py $(find gpurun_out/r06s11/mix_4 -name "*kernel_stats.csv") 4 $(find gpurun_out/r06s11/mix_12 -name "*kernel_stats.csv") 12 90 > gpurun_out/r06s11/step_kernel_mix_C5.txt
head -n 3 gpurun_out/r06s11/step_kernel_mix_C5.txt
# (3) the glue ops of the eager C5 step by Python call site
SWARM_GRAPHS=0 timeout -k 10 400 python3 -u tools/prof_train.py --config C5 --steps 3 --stack > gpurun_out/r06s11/prof_stack_C5.txt 2>&1 || { tail -n 5 gpurun_out/r06s11/prof_stack_C5.txt; exit 5; }
tail -n 1 gpurun_out/r06s11/prof_stack_C5.txt
