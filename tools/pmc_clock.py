"""Effective shader clock and MFMA busy fraction of the GEMM launches of one
objective evaluation (rocprofv3 --pmc, one pass; run on the GPU box).
Per MI355X_MICROARCH.md (DVFS give-back): clock ~= GRBM_GUI_ACTIVE / 8 / wall time
(summed over the 8 XCDs), trustworthy on dispatches >= 0.3 ms.
SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs) = MFMA pipe busy fraction.
usage: python tools/pmc_clock.py [n] [d]"""
import csv
import glob
import json
import os
import subprocess
import sys

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 10
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
odir = os.path.join(root, "gpurun_out", "pmc_clock")
cmd = ["rocprofv3", "--pmc", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "-d", odir, "-o", "run",
       "--output-format", "csv", "--", sys.executable, os.path.join(root, "tools", "prof_objective.py"),
       str(n), str(d), "1"]
subprocess.run(cmd, check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"), timeout=180)
rows = {}
for f in glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gemm" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = rows.setdefault(k, {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                "name": r["Kernel_Name"].split("(")[0]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = []
for k in sorted(rows):
    e = rows[k]
    if e["ns"] < 300000:
        continue
    clk = e.get("GRBM_GUI_ACTIVE", 0.0) / 8 / (e["ns"] * 1e-9)
    busy = e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (clk * e["ns"] * 1e-9 * 1024) if clk else 0.0
    out.append({"dispatch": k, "kernel": e["name"], "ms": e["ns"] / 1e6, "clock_ghz": clk / 1e9,
                "mfma_busy": busy})
with open(os.path.join(root, "gpurun_out", "pmc_clock_all.jsonl"), "w") as fh:
    for o in out:
        fh.write(json.dumps(o) + "\n")
for o in out[:6] + out[-8:]:
    print(json.dumps(o))
big = [o for o in out if o["ms"] > 5]
print(json.dumps({"n": n, "long_launches": len(big),
                  "clock_ghz_mean_long": sum(o["clock_ghz"] for o in big) / max(len(big), 1)}))
