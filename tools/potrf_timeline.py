"""Per-step Cholesky timeline from a rocprofv3 kernel trace (dev tool)."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = rows[len(rows) - len(rows) // int(sys.argv[2]):]
t0 = None
steps = []
cur = None
for r in rows:
    nm = r['Kernel_Name']
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
    if 'potrf_diag' in nm:
        if t0 is None: t0 = s
        cur = {'diag': (s, e), 'gemm': []}
        steps.append(cur)
    elif 'k_gemm' in nm and cur is not None and len(steps) <= 128:
        cur['gemm'].append((g, s, e, r['Queue_Id']))
tot_diag = sum(st['diag'][1] - st['diag'][0] for st in steps)
print('steps', len(steps), 'sum diag ms %.2f' % (tot_diag / 1e6))
end = steps[-1]['diag'][1]
print('potrf span ms %.2f' % ((end - t0) / 1e6))
for k in list(range(0, 6)) + list(range(60, 64)) + list(range(120, 128)):
    if k >= len(steps): break
    st = steps[k]
    d = st['diag']
    parts = ' '.join('g%d[q%s]%.0f@%.0f' % (g, q, (e - s) / 1e3, (s - t0) / 1e3) for g, s, e, q in st['gemm'])
    print('k=%3d diag %.0fus @%.0f | %s' % (k, (d[1] - d[0]) / 1e3, (d[0] - t0) / 1e3, parts))
