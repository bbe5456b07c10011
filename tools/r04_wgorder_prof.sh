#!/bin/bash
# Grouped weight-gradient kernel per block order: rocprofv3 kernel durations and FETCH_SIZE (HBM
# reads) of the cfg3 step, order 1 (split-major) and 0 (member-major).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/wgorder
mkdir -p $O
for ord in 1 0; do
  ISR_WGRAD_GROUP_ORDER=$ord timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st$ord -o run -- python3 tools/bench_train.py --steps 2 --warmup 1 > $O/st$ord.log 2>&1 || { echo "stats $ord failed"; tail -5 $O/st$ord.log; exit 1; }
  ISR_WGRAD_GROUP_ORDER=$ord timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc$ord -o run -- python3 tools/bench_train.py --steps 2 --warmup 1 > $O/pmc$ord.log 2>&1 || { echo "pmc $ord failed"; tail -5 $O/pmc$ord.log; exit 1; }
  echo "order $ord done"
done
python3 - <<'PY'
import csv, glob, json
out = {}
for ord in ("1", "0"):
    st = glob.glob(f"gpurun_out/r04/wgorder/st{ord}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(st)):
        if "wgrad3x3_group_kernel" in r["Name"]:
            out[f"order{ord}_avg_us"] = float(r["AverageNs"]) / 1e3
            out[f"order{ord}_calls"] = int(r["Calls"])
    pc = glob.glob(f"gpurun_out/r04/wgorder/pmc{ord}/**/*counter_collection.csv", recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(pc))
         if "wgrad3x3_group_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    out[f"order{ord}_fetch_MB"] = sum(v) / max(1, len(v)) / 1024.0
print(json.dumps(out))
json.dump(out, open("gpurun_out/r04/wgorder/summary.json", "w"))
PY
