"""HBM traffic of the GEMM launches from rocprofv3 PMC counters (run on the box).

Two separate --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on
gfx950), each over ONE objective evaluation at (n, d).  Per MI355X_MICROARCH.md
(HBM section): FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming
reads on gfx950, so it is doubled; WRITE_SIZE is read as is; both are in KiB.
Writes profiles/pmc_gemm_<tag>.json with bytes per launch (mean) of the fp64 GEMM (k_gemm)
and of the int8 products of the emulated A^-1 / top TRTRI level (k_oz_gemm).
"""
import csv
import glob
import json
import os
import subprocess
import sys

n, d, tag = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    odir = os.path.join(root, "gpurun_out", f"pmc_{counter}")
    cmd = ["rocprofv3", "--pmc", counter, "-d", odir, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(root, "tools", "prof_objective.py"), str(n), str(d), "1"]
    subprocess.run(cmd, check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"), timeout=180)
    files = glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True)
    for kern in ("k_gemm", "k_oz_gemm"):
        tot, launches = 0.0, set()
        for f in files:
            for r in csv.DictReader(open(f)):
                if ("::" + kern) in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                    tot += float(r["Counter_Value"])
                    launches.add(r.get("Dispatch_Id"))
        out[(counter, kern)] = {"kib_total": tot, "launches": len(launches)}
rec = {"n": n, "d": d, "note": "FETCH_SIZE doubled per the gfx950 correction; values in bytes"}
for kern, key in (("k_gemm", "gemm"), ("k_oz_gemm", "ozaki")):
    fetch = 2.0 * out[("FETCH_SIZE", kern)]["kib_total"] * 1024.0
    write = out[("WRITE_SIZE", kern)]["kib_total"] * 1024.0
    nl = max(out[("FETCH_SIZE", kern)]["launches"], 1)
    rec[key] = {"fetch_bytes_corrected": fetch, "write_bytes": write, "launches": nl}
    rec[f"bytes_per_{key}_launch" if key == "ozaki" else "bytes_per_gemm_launch"] = (fetch + write) / nl
rec["gemm_launches"] = rec["gemm"]["launches"]
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(rec, open(os.path.join(root, "profiles", f"pmc_gemm_{tag}.json"), "w"), indent=1)
print(json.dumps(rec))
