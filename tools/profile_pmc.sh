#!/bin/bash
# Collect rocprofv3 PMC counters for a command, one counter group per pass
# (MI355X_MICROARCH.md: TCC FETCH_SIZE and WRITE_SIZE cannot share a pass;
# never combine --pmc with sys/runtime tracing).
# usage: tools/profile_pmc.sh <outdir> <python args...>
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT TCC_MISS TA_TA_BUSY"
)
i=0
for P in "${PASSES[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/pass$i" -o run -- python3 "$@" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i ($P): rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
