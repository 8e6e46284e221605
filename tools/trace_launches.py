"""Per-launch listing of the last objective eval in a rocprofv3 trace (dev tool)."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = rows[len(rows) - len(rows) // int(sys.argv[2]):]
flt = sys.argv[3] if len(sys.argv) > 3 else ''
for r in rows:
    nm = r['Kernel_Name'].split('(')[0]
    if flt and flt not in nm: continue
    g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
    print('%-40s grid %6d  %9.1f us' % (nm[-40:], g, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
