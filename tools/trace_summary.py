"""Summarise a rocprofv3 kernel trace for the LAST objective eval (dev tool)."""
import csv, collections, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
nev = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = rows[len(rows) - len(rows) // nev:]
t0 = int(rows[0]['Start_Timestamp']); t1 = int(rows[-1]['End_Timestamp'])
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows)
print('eval wall ms %.2f busy ms %.2f kernels %d' % ((t1 - t0) / 1e6, busy / 1e6, len(rows)))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    nm = r['Kernel_Name'].split('(')[0][-32:]
    g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
    key = (nm, 'g<=64' if g <= 64 else ('g<=512' if g <= 512 else 'g>512'))
    agg[key][0] += 1; agg[key][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print('%-34s %-7s n=%4d  %8.2f ms' % (k[0], k[1], v[0], v[1]))
