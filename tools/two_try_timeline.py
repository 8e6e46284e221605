"""Which phases of the two tries in flight overlap, and for how long (dev tool; run on the
GPU box).  Traces tools/concurrent_evals.py (2 contexts, `reps` evaluations each) with
rocprofv3 --kernel-trace and sweeps the concurrent part: for every interval, the set of
phases running (Cb/Cm/Ct = Cholesky steps 0-47 / 48-87 / 88-127, T = TRTRI levels,
L = LAUUM, o = the rest), and the share of time each set holds.
usage: python tools/two_try_timeline.py [reps]  -> gpurun_out/two_try_timeline.json"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
odir = os.path.join(root, "gpurun_out", "two_try_trace")
if "--analyze" not in sys.argv:
    subprocess.run(["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", odir, "-o", "run", "--",
                    sys.executable, os.path.join(root, "tools", "concurrent_evals.py"), "16384", "2", str(reps)],
                   check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"), timeout=300)
files = glob.glob(os.path.join(odir, "**", "*kernel_trace.csv"), recursive=True)
rows = []
for f in files:
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def cls(name):
    if "k_gemm<false, false, true" in name:
        return "C"
    if "k_gemm<true, true, false, false>" in name:
        return "L"
    if "k_gemm" in name:
        return "T"
    return "o"


qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
cnt = defaultdict(int)
ev = []
fused_seen = 0
t_start = t_stop = None
for r in rows:
    c = cls(r["Kernel_Name"])
    if c == "C":
        q = r[qkey]
        i = cnt[q] % 128
        cnt[q] += 1
        fused_seen += 1
        c = "Cb" if i < 48 else ("Cm" if i < 88 else "Ct")
        if fused_seen == 2 * 128 + 1:   # the first concurrent evaluation starts
            t_start = int(r["Start_Timestamp"])
        if fused_seen == 2 * 128 + 2 * 2 * reps * 128 + 1:   # the sequential part starts
            t_stop = int(r["Start_Timestamp"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), (c, r[qkey])))
assert t_start is not None, "fewer than three Cholesky sweeps in the trace"
ev = [e for e in ev if e[0] >= t_start and (t_stop is None or e[0] < t_stop)]
t_end = max(e[1] for e in ev)
points = sorted({e[0] for e in ev} | {e[1] for e in ev})
share = defaultdict(float)
active = defaultdict(int)
starts = defaultdict(list)
for e in ev:
    starts[e[0]].append(e)
ends = defaultdict(list)
for e in ev:
    ends[e[1]].append(e)
prev = points[0]
for p in points:
    if p > prev:
        key = "+".join(sorted(k[0] for k in active)) or "idle"   # one entry per (phase, queue)
        share[key] += (p - prev) / 1e6
    for e in ends[p]:
        active[e[2]] -= 1
        if active[e[2]] == 0:
            del active[e[2]]
    for e in starts[p]:
        active[e[2]] += 1
    prev = p
total = (t_end - t_start) / 1e6
out = {"reps": reps, "window_ms": total, "evals_in_window": 2 * 2 * reps,
       "ms_per_eval": total / (2 * 2 * reps),
       "share": {k: {"ms": round(v, 2), "frac": round(v / total, 4)} for k, v in sorted(share.items(), key=lambda x: -x[1]) if v / total >= 0.002}}
json.dump(out, open(os.path.join(root, "gpurun_out", "two_try_timeline.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
