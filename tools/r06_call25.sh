#!/bin/bash
# Round 6: the dependency-wait sleep of the trunk kernel (s_sleep 1 = production vs 3 vs 8 between
# polls), whole fp16 forwards of the bench workload under sustained load, alternating processes.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
L=$PWD/image_super_resolution_amd/lib
for i in 1 2 3; do
  for lib in libisr.so libisr_spin3.so libisr_spin8.so; do
    ISR_LIB=$L/$lib timeout -k 10 120 python -u tools/time_forward.py --rounds 5 --steps 20 >> gpurun_out/r06/t25_spin_ab.jsonl 2>> gpurun_out/r06/t25_spin_ab.err
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc ($lib)"; exit $rc; fi
  done
done
echo done
