#!/bin/bash
# Inference-only kernel trace of bench.py (no train leg, no CPU baseline): per-kernel durations of
# one forward and the gaps between them on the graph replay.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/inftrace -o inf -- python3 bench.py --steps 10 --warmup 3 --train-steps 0 --no-cpu-baseline > $O/infer_prof_bench.json 2> $O/infer_prof_err.txt || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('/tmp/inftrace/**/inf_kernel_trace.csv', recursive=True) + glob.glob('/tmp/inftrace/inf_kernel_trace.csv')
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
tr = [i for i, r in enumerate(rows) if 'trunk_kernel' in r['Kernel_Name']]
sel = rows[max(0, tr[4] - 12):tr[6] + 12] if len(tr) >= 7 else rows[-400:]
with open('gpurun_out/r05/infer_trace.csv', 'w') as o:
    o.write('start_ns,dur_ns,queue,grid,wg,name\n')
    for r in sel:
        o.write('%d,%d,%s,%s,%s,"%s"\n' % (int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - int(r['Start_Timestamp']),
                                          r.get('Queue_Id', ''), r['Grid_Size_X'], r['Workgroup_Size_X'], r['Kernel_Name'][:120]))
print(len(rows))
PY
