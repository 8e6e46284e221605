"""Per-launch timeline of the last objective evaluation in a rocprofv3 kernel trace (dev tool):
every launch after the last K-build with its grid and start/duration in us.
usage: python tools/step_timeline.py kernel_trace.csv"""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
NB = 128
starts = [i + 1 for i, r in enumerate(rows) if 'k_pairs' in r['Kernel_Name']]
i0 = starts[-1]
seq = rows[i0:]
t0 = int(seq[0]['Start_Timestamp'])
for i, r in enumerate(seq[:160]):
    nm = r['Kernel_Name'].split('(')[0][-30:]
    wg = int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])
    print('%3d %-30s %6d WG start %8.1f dur %7.1f' % (i, nm, wg, (int(r['Start_Timestamp'])-t0)/1e3, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3))
