#!/bin/bash
# Round-4: the C5 optimizer step's LSTM sequence launches (grid, duration, order) from a
# rocprofv3 kernel trace of bench.py --train --config C5; only the LSTM rows are kept.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv \
  -- python3 bench.py --train --config C5 --minibatches 2 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 3; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4q/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
keys = [k for k in rows[0] if "Grid" in k or "Workgroup" in k or "Size" in k]
print("columns", keys)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
with open("gpurun_out/r4q/lstm_rows.csv", "w") as o:
    w = csv.writer(o)
    w.writerow(["idx", "name", "dur_us"] + keys)
    for i, r in enumerate(rows):
        if "lstm" in r["Kernel_Name"] or "rsa_pool" in r["Kernel_Name"]:
            w.writerow([i, r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3]
                       + [r[k] for k in keys])
print(len(rows), "kernels")
PY
tail -40 $OUT/lstm_rows.csv
rm -rf $OUT/trace
echo R4Q_DONE
