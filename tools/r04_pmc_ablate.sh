#!/bin/bash
# Per-cause HBM traffic of the pair-form trunk kernel: the tuning build's
# ablations (1 no halo DMA, 8 no weight DMA, 4 no epilogue stores, 16 no dependency waits) under
# rocprofv3 FETCH_SIZE and WRITE_SIZE, one counter per pass; traffic(all) - traffic(cause off)
# attributes the bytes.  Summaries: tools/pmc_summary.py per ablation.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04/pmc_ablate
T=/tmp/isr_pmc_ablate
mkdir -p $O $T
export ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
for A in 0 1 8 4 16; do
  i=0
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $T/abl$A/pass$i -o run -- \
      python3 tools/ab_trunk.py --configs $A:0 --rounds 1 --reps 3 > $O/abl${A}_pass$i.log 2>&1
    rc=$?
    echo "ablate $A $C rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    i=$((i+1))
  done
  python3 tools/pmc_summary.py $T/abl$A --json $O/abl$A.json --match trunk_kernel > /dev/null || exit 1
done
python3 - <<'PY'
import json
out = {}
for a in (0, 1, 8, 4, 16):
    rows = json.load(open(f"gpurun_out/r04/pmc_ablate/abl{a}.json"))
    r = max(rows, key=lambda r: r["dispatches"])
    out[a] = {"read_gb": round(r["hbm_read_bytes"] / 1e9, 3), "write_gb": round(r["hbm_write_bytes"] / 1e9, 3),
              "dispatches": r["dispatches"]}
print(json.dumps(out))
json.dump(out, open("gpurun_out/r04/pmc_ablate/summary.json", "w"), indent=1)
PY
