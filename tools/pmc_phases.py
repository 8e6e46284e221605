"""Per-launch PMC picture of one objective evaluation, grouped by phase (dev tool,
run on the GPU box): shader clock and MFMA busy, L2 hit rate, HBM bytes.

Separate rocprofv3 --pmc passes (counter-block limits; FETCH_SIZE and WRITE_SIZE
apart), each over one evaluation at (n, d) (tools/prof_objective.py).  Launches are
matched across passes by their order.  Per MI355X_MICROARCH.md: clock = GRBM_GUI_ACTIVE
/ 8 / wall time, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs),
FETCH_SIZE doubled on gfx950 (KiB).
Phases: the Cholesky launches (one per step or one per column group) by steps 0/1-47 /
48-87 / 88-127, the TRTRI launches, the LAUUM.
usage: python tools/pmc_phases.py [n] [d]"""
import csv
import glob
import json
import os
import subprocess
import sys

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 10
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
passes = [["GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"],
          ["TCC_HIT_sum", "TCC_MISS_sum"],
          ["FETCH_SIZE"],
          ["WRITE_SIZE"]]
launches = None
for i, counters in enumerate(passes):
    odir = os.path.join(root, "gpurun_out", f"pmc_phase{i}")
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "-d", odir, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.join(root, "tools", "prof_objective.py"),
           str(n), str(d), "1"]
    subprocess.run(cmd, check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL)
    rows = {}
    for f in glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_gemm" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            e = rows.setdefault(k, {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                    "kind": r["Kernel_Name"].split("(")[0].replace("void gpe::", "")})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [rows[k] for k in sorted(rows)]
    if launches is None:
        launches = seq
    else:
        assert len(seq) == len(launches), (len(seq), len(launches))
        for a, b in zip(launches, seq):
            for key, v in b.items():
                if key not in ("ns", "kind"):
                    a[key] = v
# 14 TRTRI + 1 LAUUM after the Cholesky's launches: one per step (GPEMU_POTRF=fused), or
# one per column group of width >= 2 and one per width-1 step (the default for a lone
# evaluation); the widths as the library's (GPEMU_POTRF_W, default 4 while more than 48
# tile columns remain, then 2 while more than 24).  Phases by each launch's first step.
nb = -(-n // 128)
widths = [(4, 48), (2, 24)]
if os.environ.get("GPEMU_POTRF_W"):
    widths = [tuple(int(v) for v in e.split(":")) for e in os.environ["GPEMU_POTRF_W"].split(",")]
starts, g = [], 0
while g < nb:
    starts.append(g)
    w = next((a for a, m in widths if nb - g > m), 1)
    g += max(1, min(w, nb - g))
nch = len(launches) - 15
first = list(range(nb)) if nch == nb else starts
if len(first) != nch:
    groups = {"chol": launches[:nch]}
else:
    groups = {"chol 0-47": [], "chol 48-87": [], "chol 88-127": []}
    for f, e in zip(first, launches[:nch]):
        groups["chol 0-47" if f < 48 else ("chol 48-87" if f < 88 else "chol 88-127")].append(e)
groups.update({"trtri": launches[nch:nch + 14], "lauum": launches[nch + 14:nch + 15]})
out = {"n": n, "d": d, "schedule": os.environ.get("GPEMU_POTRF", "auto"), "phases": {}}
for name, ls in groups.items():
    ns = sum(e["ns"] for e in ls)
    gui = sum(e.get("GRBM_GUI_ACTIVE", 0.0) for e in ls)
    clk = gui / 8 / (ns * 1e-9)
    busy = sum(e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for e in ls) / (clk * ns * 1e-9 * 1024)
    hit = sum(e.get("TCC_HIT_sum", 0.0) for e in ls)
    miss = sum(e.get("TCC_MISS_sum", 0.0) for e in ls)
    fetch = 2.0 * 1024.0 * sum(e.get("FETCH_SIZE", 0.0) for e in ls)
    write = 1024.0 * sum(e.get("WRITE_SIZE", 0.0) for e in ls)
    out["phases"][name] = {"launches": len(ls), "ms": ns / 1e6, "clock_ghz": clk / 1e9, "mfma_busy": busy,
                           "l2_hit": hit / max(hit + miss, 1.0), "hbm_read_gb": fetch / 1e9,
                           "hbm_write_gb": write / 1e9, "hbm_tb_s": (fetch + write) / (ns * 1e-9) / 1e12}
print(json.dumps(out, indent=1))
