"""Combined k_gemm row of a rocprofv3 --stats kernel summary (dev tool): the GEMM has
ten instances (layout x fused x CDEF), bench.py's roofline averages over all of them.
usage: python tools/kgemm_combined.py <kernel_stats.csv> [bench_line.json]"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_gemm<" in r["Name"]]
calls = sum(int(r["Calls"]) for r in rows)
total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
out = {"kernel": "k_gemm (all instances)", "calls": calls, "total_ms": total_ns / 1e6,
       "mean_us": total_ns / calls / 1e3,
       "instances": {r["Name"].split("(")[0].replace("void gpe::", ""): {"calls": int(r["Calls"]),
                     "mean_us": float(r["AverageNs"]) / 1e3} for r in rows}}
if len(sys.argv) > 2:
    line = [ln for ln in open(sys.argv[2]) if ln.startswith("{")][-1]
    rf = json.loads(line)["roofline"]
    out["bench_ms_per_launch"] = rf["ms_per_launch"]
    out["bench_vs_rocprof"] = rf["ms_per_launch"] * 1e3 / out["mean_us"]
print(json.dumps(out, indent=1))
