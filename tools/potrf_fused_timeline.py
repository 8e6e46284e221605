"""Per-step timeline of the fused Cholesky schedule from a rocprofv3 kernel trace
(dev tool): launch 0 = diag(0) + panel(0), then one launch per step kt.
usage: potrf_fused_timeline.py kernel_trace.csv [NB]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 128
starts = [i + 1 for i, r in enumerate(rows) if 'k_pairs' in r['Kernel_Name']]
i0 = starts[-1]            # last eval's first Cholesky launch follows its K-build
seq = rows[i0:i0 + NB]
t0 = int(seq[0]['Start_Timestamp'])
dur = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
print('launch0 %.1f us' % dur(seq[0]))
fsum = gsum = 0.0
prev_end = int(seq[0]['End_Timestamp'])
lines = []
for kt in range(NB - 1):
    f = seq[1 + kt]
    gap = (int(f['Start_Timestamp']) - prev_end) / 1e3
    prev_end = int(f['End_Timestamp'])
    fsum += dur(f)
    gsum += gap
    wg = int(f['Grid_Size_X']) // int(f['Workgroup_Size_X'])
    lines.append('kt=%3d m=%3d fused %7.1f (%5d WG) gap %5.1f' % (kt, NB - 1 - kt, dur(f), wg, gap))
for ln in lines[:4] + lines[40:44] + lines[80:84] + lines[100:104] + lines[-10:]:
    print(ln)
print('span %.2f ms: launches %.2f gaps %.2f' % ((prev_end - t0) / 1e6, fsum / 1e3, gsum / 1e3))
