#!/bin/bash
# One parameterised GPU session (it replaces the per-session gpu_r3* / gpu_r4* scripts of earlier
# rounds; those live in git history). Steps run in the order given; every GPU step has its own time
# limit, and the first failure (a test failure, a crash, an abort or a time-out) ends the script.
#
#   TAG=name STEPS="tests smoke bench prof pmc" tools/gpu_steps.sh
#
# steps:  tests      pytest (PYTEST_SEL, default "tests -m gpu")
#         smoke      __graft_entry__.smoke()
#         bench      bench.py with the default arguments and with the driver's (--steps 20 --warmup 5)
#         prof       rocprofv3 --kernel-trace --stats of both bench commands (summaries only)
#         pmc        the step kernel's PMC passes (tools/pmc.sh -> gpurun_out/pmc/pmc_traffic.json)
#         variants   bench every build/variants/lib_*.so (tools/variants.sh run)
#         wavetime   the wave-timing build's per-wave log (tools/wave_timing.py, WT_LIB)
#         train      bench.py --train --config c for c in CFGS (default "C5 C4 C3")
#         trainprof  tools/prof_train.py --config c (eager, torch profiler) for c in CFGS
#         pmctrain   tools/pmc_train.sh for c in CFGS (MFMA counters of the optimizer steps)
#         critic     bench.py --critic (the fused critic attention at C3)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-session}
mkdir -p $OUT
export TMPDIR=/tmp
test -f swarmacb-isaaclab_amd/SwarmACB_isaac/libswarmstep.so || { echo "libswarmstep.so missing: build first"; exit 2; }
last_json() { grep '^{' "$1" | tail -1; }
for step in ${STEPS:-tests smoke bench}; do
  case $step in
  tests)
    timeout -k 10 1200 python3 -u -m pytest ${PYTEST_SEL:-tests -m gpu} -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > $OUT/pytest.log 2>&1
    RC=$?; tail -3 $OUT/pytest.log; grep '^FAILED' $OUT/pytest.log | head
    [ $RC -ne 0 ] && { echo "tests rc=$RC"; exit 3; } ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
      || { tail -5 $OUT/smoke.log; exit 4; }
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 5; }
    last_json $OUT/bench_default.log > $OUT/bench_default.json
    timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_args.log 2>&1 \
      || { tail -20 $OUT/bench_driver_args.log; exit 5; }
    last_json $OUT/bench_driver_args.log > $OUT/bench_driver_args.json
    python3 -c "
import json
for k in ('default', 'driver_args'):
    d = json.load(open('$OUT/bench_%s.json' % k)); r = d['roofline']
    print(k, 'value %.4g' % d['value'], 'kernel_us %.2f' % r['kernel_avg_us'], 'valu_frac', r['frac'], r['pmc_status'])" ;;
  prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv \
      -- python3 bench.py --cpu-seconds 0 > $OUT/prof_default.log 2>&1 || { tail -20 $OUT/prof_default.log; exit 6; }
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv \
      -- python3 bench.py --cpu-seconds 0 --steps 20 --warmup 5 > $OUT/prof_driver.log 2>&1 \
      || { tail -20 $OUT/prof_driver.log; exit 6; }
    find $OUT/prof_default $OUT/prof_driver -name "*kernel_trace*" -delete
    find $OUT/prof_default $OUT/prof_driver -name "*kernel_stats*" -exec head -3 {} \; ;;
  pmc)
    bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 7; }
    find gpurun_out/pmc -name "*counter_collection*" -size +20M -delete
    tail -3 $OUT/pmc.log ;;
  variants)
    bash tools/variants.sh run > $OUT/variants.log 2>&1 || { tail -20 $OUT/variants.log; exit 8; }
    tail -20 $OUT/variants.log ;;
  wavetime)
    SWARMSTEP_LIB=$PWD/${WT_LIB:-build/variants/lib_wt.so} timeout -k 10 300 python3 tools/wave_timing.py ${WT_ARGS:-} \
      > $OUT/wave_timing.log 2>&1 || { tail -20 $OUT/wave_timing.log; exit 9; }
    tail -12 $OUT/wave_timing.log ;;
  train)
    for cfg in ${CFGS:-C5 C4 C3}; do
      timeout -k 10 300 python3 bench.py --train --config $cfg > $OUT/train_$cfg.log 2>&1 \
        || { echo "train $cfg failed"; tail -5 $OUT/train_$cfg.log; exit 10; }
      last_json $OUT/train_$cfg.log > $OUT/bench_train_$cfg.jsonl
      python3 -c "import json; d=json.loads(open('$OUT/bench_train_$cfg.jsonl').read()); print('$cfg ms/opt-step %.3f' % d['ms_per_optimizer_step'])"
    done ;;
  trainprof)
    for cfg in ${CFGS:-C5}; do
      SWARM_GRAPHS=0 timeout -k 10 300 python3 -u tools/prof_train.py --config $cfg --steps 3 ${PROF_ARGS:-} \
        > $OUT/prof_train_$cfg.txt 2>&1 || { tail -5 $OUT/prof_train_$cfg.txt; exit 11; }
      tail -1 $OUT/prof_train_$cfg.txt
    done ;;
  pmctrain)
    for cfg in ${CFGS:-C3 C5}; do
      CFG=$cfg bash tools/pmc_train.sh > $OUT/pmc_train_$cfg.log 2>&1 || { tail -20 $OUT/pmc_train_$cfg.log; exit 12; }
      rm -rf $OUT/pmc_train_$cfg && mv gpurun_out/pmc_train $OUT/pmc_train_$cfg
      find $OUT/pmc_train_$cfg -name "*counter_collection*" -size +20M -delete
      find $OUT/pmc_train_$cfg -name "*kernel_trace*" -delete
      tail -3 $OUT/pmc_train_$cfg.log
    done ;;
  critic)
    timeout -k 10 300 python3 bench.py --critic ${CRITIC_ARGS:-} > $OUT/critic.log 2>&1 || { tail -10 $OUT/critic.log; exit 13; }
    last_json $OUT/critic.log ;;
  *) echo "unknown step $step"; exit 1 ;;
  esac
done
echo "GPU_STEPS_DONE $OUT"
