#!/bin/bash
# Round 6: production trunk vs the same trunk with the XCD-aware tile deal (lib/libisr_xcd.so,
# -DISR_TRUNK_XCD=1), whole fp16 forwards of the bench workload under sustained load, alternating
# processes (4 each).  Outputs must be bit-identical (checksum).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
L=$PWD/image_super_resolution_amd/lib
for i in 1 2 3 4; do
  for lib in libisr.so libisr_xcd.so; do
    ISR_LIB=$L/$lib timeout -k 10 120 python -u tools/time_forward.py --rounds 5 --steps 20 >> gpurun_out/r06/t22_xcd_ab.jsonl 2>> gpurun_out/r06/t22_xcd_ab.err
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc ($lib)"; exit $rc; fi
  done
done
echo done
