set -o pipefail
mkdir -p gpurun_out/dp
for dp in 1 2 5 10 20; do
  timeout -k 10 120 python3 bench.py --cpu-seconds 0 --steps 600 --decision-period $dp > gpurun_out/dp/dp$dp.log 2>&1 || { tail -5 gpurun_out/dp/dp$dp.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dp/dp$dp.log').read().strip().splitlines()[-1]); print('dp=$dp', 'value %.4g' % d['value'], 'kernel_us %.2f' % d['roofline']['kernel_avg_us'], 'per_substep %.2f' % (d['roofline']['kernel_avg_us']/$dp))"
done
