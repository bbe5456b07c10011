#!/bin/bash
# Produce the round's committed profiles (run on the GPU box from the repo root):
#   profiles/<R>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `python3 bench.py`
#   profiles/<R>_pmc_summary.json         per-kernel PMC summary (tools/pmc_summary.py)
#   profiles/<R>_pmc_traffic.json         HBM bytes per launch of the dominant kernel (read by bench.py)
#   profiles/<R>_bench.json               the bench line after the traffic file exists
#   profiles/<R>_train_kernel_stats.csv   rocprofv3 --kernel-trace --stats of tools/bench_train.py (cfg3 step)
# usage: tools/make_profiles.sh r02
set -eu
R=${1:-r01}
export TMPDIR=/tmp
P=gpurun_out/profiles_$R   # gpurun merges only gpurun_out/ back (<= 64 MiB); copy into profiles/ afterwards
T=/tmp/isr_prof_$R         # raw rocprofv3 output stays off gpurun_out/
mkdir -p $P $T
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof_bench -o bench -- \
  python3 bench.py --round $R > $P/prof_bench.json 2> $P/prof_bench.err
cp $T/prof_bench/bench_kernel_stats.csv $P/${R}_bench_kernel_stats.csv
# the dominant kernel (the persistent trunk kernel): its launches from the trace
python3 - "$T/prof_bench/bench_kernel_trace.csv" "$P/${R}_bench_dominant_by_grid.json" <<'EOF2'
import csv, json, sys
from collections import defaultdict
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "trunk_" in r["Kernel_Name"] and "prep" not in r["Kernel_Name"]]
by = defaultdict(list)  # per (instantiation, grid): the inference forward's fp16 trunk and the
for r in rows:          # training leg's bf16 trunk are different kernels of one bench run
    by[(r["Kernel_Name"], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(
        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = [{"kernel": k, "blocks": b, "dispatches": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 3),
        "min_us": round(min(v) / 1e3, 3), "median_us": round(sorted(v)[len(v) // 2] / 1e3, 3),
        "durations_us_in_launch_order": [round(x / 1e3, 1) for x in v],
        "role": "persistent trunk kernel (trunk.hip), one launch per forward"
                + (" (inference, fp16 storage)" if ", true>" in k else " (bf16: the bench's training leg)")}
       for (k, b), v in sorted(by.items())]
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
EOF2
bash tools/profile_pmc.sh $T/pmc_bench bench.py --no-cpu-baseline --no-storage-ab --steps 5 --warmup 2 --train-steps 0 --round $R
python3 tools/pmc_summary.py $T/pmc_bench --json $P/${R}_pmc_summary.json > /dev/null
python3 - "$R" "$P" <<'EOF'
import json, sys
R, P = sys.argv[1], sys.argv[2]
rows = json.load(open(f"{P}/{R}_pmc_summary.json"))
# kernel families bench.py reports a roofline for (bench.py load_traffic): the persistent
# trunk kernel, the per-conv growth (V_G0) and final (V_F0) templates, the 9x9 tail
fam = {"chain": "trunk_", "growth": "C3<4, 4, 1, 16, 2, 0, 0, 2",
       "final": "C3<4, 4, 2, 16, 2, 192", "tail": "tail9x9_"}
out = {"families": {},
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, KiB -> bytes, FETCH_SIZE x2 "
                 "(gfx950 wide-load correction, MI355X_MICROARCH.md §HBM); mean over dispatches of the "
                 "largest grid of the family; Infinity-Cache hits are included in these counters"}
for k, sub in fam.items():
    dom = [r for r in rows if sub in r["kernel"] and (k != "growth" or "chain" not in r["kernel"])]
    if not dom:
        continue
    g = max(int(r["grid"]) for r in dom)
    sel = [r for r in dom if int(r["grid"]) == g]
    nd = sum(r["dispatches"] for r in sel)
    avg = lambda key: sum(r[key] * r["dispatches"] for r in sel) / nd
    out["families"][k] = {"kernel": sel[0]["kernel"], "grid": g, "dispatches": nd,
                          "hbm_bytes_per_launch": avg("hbm_bytes"), "hbm_read_bytes": avg("hbm_read_bytes"),
                          "hbm_write_bytes": avg("hbm_write_bytes")}
    print("traffic", k, out["families"][k]["hbm_bytes_per_launch"])
json.dump(out, open(f"{P}/{R}_pmc_traffic.json", "w"), indent=1)
EOF
cp $P/${R}_pmc_traffic.json profiles/ 2>/dev/null || true
timeout -k 10 600 python3 bench.py --round $R > $P/${R}_bench.json 2> $P/bench_final.err
cat $P/${R}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/prof_train -o train -- \
  python3 tools/bench_train.py --steps 3 --warmup 2 > $P/${R}_train_bench.json 2> $P/prof_train.err
cp $T/prof_train/train_kernel_stats.csv $P/${R}_train_kernel_stats.csv
