#!/bin/bash
# Kernel trace (order + stream) of two cfg3 training steps, to attribute the torch glue kernels
# (fills, copies, elementwise) to the phases that launch them.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/trtrace -o tr -- python3 tools/bench_train.py --steps 2 --warmup 1 > $O/train_trace_bench.json 2> $O/train_trace_err.txt || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('/tmp/trtrace/**/tr_kernel_trace.csv', recursive=True) + glob.glob('/tmp/trtrace/tr_kernel_trace.csv')
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
with open('gpurun_out/r05/train_trace.csv', 'w') as o:
    o.write('start_ns,dur_ns,queue,grid,wg,name\n')
    t0 = int(rows[0]['Start_Timestamp'])
    for r in rows:
        o.write('%d,%d,%s,%s,%s,"%s"\n' % (int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - int(r['Start_Timestamp']),
                                          r.get('Queue_Id', r.get('Stream_Id', '')), r['Grid_Size_X'], r['Workgroup_Size_X'], r['Kernel_Name'][:120]))
print(len(rows))
PY
