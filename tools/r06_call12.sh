#!/bin/bash
# Round 6: the trunk kernel's per-dispatch durations under rocprofv3 across one whole bench.py run
# (warm-up, timed steps, per-kernel timing rounds, parity, training leg), to place the profiled
# average against the live per-launch figure of the bench line.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
T=/tmp/isr_prof_dist
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $T -o bench -- \
  python3 bench.py > gpurun_out/r06/prof_dist_bench.json 2> gpurun_out/r06/prof_dist_bench.err || exit 1
python3 - "$T/bench_kernel_trace.csv" gpurun_out/r06/trunk_dispatches.json <<'EOF2'
import csv, json, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "trunk_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
out = [{"kernel": "fp16" if ", true>" in r["Kernel_Name"] else "bf16",
        "t_ms": round((int(r["Start_Timestamp"]) - t0) / 1e6, 2),
        "us": round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1)} for r in rows]
json.dump(out, open(sys.argv[2], "w"), indent=0)
print(len(out))
EOF2
