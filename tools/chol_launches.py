"""Per-launch timeline of the last objective evaluation in a rocprofv3 kernel trace
(dev tool).  usage: python tools/chol_launches.py <kernel_trace.csv>

Finds the last K-build (k_pairs) and prints every launch after it up to the next
K-build: index, kernel, workgroups, duration, gap to the previous launch's end.
Summarises the Cholesky (the fused k_gemm<false,false> launches right after the
K-build), the TRTRI and LAUUM launches, and the idle time between launches."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
kb = [i for i, r in enumerate(rows) if "k_pairs" in r["Kernel_Name"]]
if len(kb) < 2:
    sys.exit("need two evaluations in the trace")
seg = rows[kb[-2]:kb[-1]]


def short(nm):
    nm = nm.split("(")[0].replace("void ", "").replace("gpe::", "")
    return nm[:28]


prev_end = None
phase = {}
chol = []
for i, r in enumerate(seg):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    nm = short(r["Kernel_Name"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e
    other_gemm = "gemm_other" in phase
    if nm.startswith("k_gemm<false, false, true") and not other_gemm:   # FUSED (either C form)
        key = "chol"
        chol.append((wg, (e - s) / 1e3, gap))
    elif nm.startswith("k_gemm"):
        key = "gemm_other"
    else:
        key = nm
    p = phase.setdefault(key, [0, 0.0, 0.0])
    p[0] += 1
    p[1] += (e - s) / 1e3
    p[2] += gap
    if "-v" in sys.argv:
        print("%4d %-28s wg %6d  %9.1f us  gap %6.1f" % (i, nm, wg, (e - s) / 1e3, gap))
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
print("evaluation span %.2f ms" % (span / 1e3))
for k, (cnt, dur, gap) in phase.items():
    print("  %-28s launches %4d  busy %8.2f ms  gaps %6.2f ms" % (k, cnt, dur / 1e3, gap / 1e3))
print("cholesky steps (t: workgroups, us, gap):")
for t, (wg, d, g) in enumerate(chol):
    if t % 4 == 0 or t >= 88:
        print("  t=%3d wg %5d  %7.1f us  gap %5.1f" % (t, wg, d, g))
