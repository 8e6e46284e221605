"""Check stream overlap in a rocprofv3 kernel trace (dev tool)."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = rows[len(rows) - len(rows) // int(sys.argv[2]):]
t0 = int(rows[0]['Start_Timestamp'])
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    nm = r['Kernel_Name'].split('(')[0][-28:]
    g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
    print('q%-3s %-28s g=%5d  start %9.1f  end %9.1f us' % (r['Queue_Id'], nm, g, (int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - t0) / 1e3))
