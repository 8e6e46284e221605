"""Does the GEMM's HBM traffic cost shader clock?  (dev tool, run on the GPU box; VERDICT r4
item 2.)  One plain NN k_gemm configuration (128 x 128 tiles, beta = 1, as the Cholesky's
bulk) run three ways by gpe_bench_gemm:
  cold   operands streamed from HBM (every tile its own A / B panels, as in the sweep);
  hot1   GPEMU_BENCH_HOT=1: every k re-reads the same 128 values (L1-resident, but the
         MFMA inputs repeat, so they also toggle less);
  hot2   GPEMU_BENCH_HOT=2: operands from a (tiles + K) x 128-double window (L2-resident,
         the MFMA inputs as varied as when cold).
For each: un-profiled ms per launch (HIP events, 20 launches), then separate rocprofv3
--pmc passes (GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES; FETCH_SIZE; WRITE_SIZE) over the
same launches, per launch: clock = GRBM_GUI_ACTIVE / 8 / wall, MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs), HBM bytes = 2 FETCH_SIZE (gfx950)
+ WRITE_SIZE (KiB); and amd-smi power / clock samples during a ~3 s un-profiled run.
usage: python tools/clock_traffic.py [mt] [K ...]   -> gpurun_out/clock_traffic.json"""
import csv
import glob
import json
import os
import re
import subprocess
import sys
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
mt = int(sys.argv[1]) if len(sys.argv) > 1 else 96
Ks = [int(k) for k in sys.argv[2:]] or [512, 4096]
MODES = {"cold": None, "hot1": "1", "hot2": "2"}
PASSES = [["GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"], ["FETCH_SIZE"], ["WRITE_SIZE"]]


def env_for(mode):
    e = dict(os.environ, TMPDIR="/tmp")
    e.pop("GPEMU_BENCH_HOT", None)
    if MODES[mode]:
        e["GPEMU_BENCH_HOT"] = MODES[mode]
    return e


def gemm_cmd(K, reps):
    return [sys.executable, os.path.join(root, "tools", "gemm_one.py"), str(mt), str(mt), str(K), "0", "0", str(reps)]


def smi_sample():
    try:
        out = subprocess.run(["amd-smi", "metric", "-g", "0", "--clock", "--power"], capture_output=True,
                             text=True, timeout=20).stdout
    except Exception:
        return None
    w = re.search(r"SOCKET_POWER:\s*(\d+) W", out)
    clks = [int(m) for m in re.findall(r"^\s+CLK: (\d+) MHz", out, re.M)][:8]
    return {"w": int(w.group(1)) if w else None, "gfx_mhz": sum(clks) / len(clks) if clks else None}


res = {"mt": mt, "nt": mt, "beta": 1.0, "layout": "NN", "configs": []}
for K in Ks:
    flops = 2.0 * (mt * 128) ** 2 * K
    for mode in MODES:
        row = {"K": K, "mode": mode}
        r = subprocess.run(gemm_cmd(K, 20), capture_output=True, text=True, cwd=root, env=env_for(mode), timeout=120)
        m = re.search(r": ([0-9.]+) ms ([0-9.]+) TF/s", r.stdout)
        row["ms"], row["tflops"] = (float(m.group(1)), float(m.group(2))) if m else (None, None)
        # power / clock while the same launches run back to back for ~3 s
        reps = max(20, int(3000.0 / max(row["ms"] or 1.0, 0.05)))
        p = subprocess.Popen(gemm_cmd(K, reps), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=root,
                             env=env_for(mode))
        samples = []
        time.sleep(1.5)
        while p.poll() is None and len(samples) < 6:
            s = smi_sample()
            if s:
                samples.append(s)
            time.sleep(0.2)
        p.wait(timeout=120)
        row["smi"] = samples
        per = {}
        for i, counters in enumerate(PASSES):
            odir = os.path.join(root, "gpurun_out", f"ct_{K}_{mode}_{i}")
            cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *counters, "-d", odir, "-o", "run",
                   "--output-format", "csv", "--"] + gemm_cmd(K, 10)
            subprocess.run(cmd, check=True, cwd=root, env=env_for(mode), stdout=subprocess.DEVNULL)
            rows = {}
            for f in glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True):
                for rr in csv.DictReader(open(f)):
                    if "k_gemm" not in rr["Kernel_Name"]:
                        continue
                    k = int(rr["Dispatch_Id"])
                    e = rows.setdefault(k, {"ns": int(rr["End_Timestamp"]) - int(rr["Start_Timestamp"])})
                    e[rr["Counter_Name"]] = e.get(rr["Counter_Name"], 0.0) + float(rr["Counter_Value"])
            seq = [rows[k] for k in sorted(rows)][1:]   # the warm-up launch left out
            for key in counters + ["ns"]:
                vals = [e.get(key, 0.0) for e in seq]
                per.setdefault(key, []).append(sum(vals) / max(len(vals), 1))
        ns = sum(per["ns"]) / len(per["ns"])
        clk = per["GRBM_GUI_ACTIVE"][0] / 8 / (per["ns"][0] * 1e-9)
        row.update({"prof_ms": ns / 1e6, "clock_ghz": clk / 1e9,
                    "mfma_busy": per["SQ_VALU_MFMA_BUSY_CYCLES"][0] / (clk * per["ns"][0] * 1e-9 * 1024),
                    "hbm_read_gb": 2.0 * 1024.0 * per["FETCH_SIZE"][0] / 1e9,
                    "hbm_write_gb": 1024.0 * per["WRITE_SIZE"][0] / 1e9,
                    "algorithmic_gb": (2 * mt * 128 * K + 2 * (mt * 128) ** 2) * 8 / 1e9,
                    "prof_tflops": flops / (ns * 1e-9) / 1e12})
        row["hbm_tb_s"] = (row["hbm_read_gb"] + row["hbm_write_gb"]) / (row["prof_ms"] * 1e-3) / 1e3
        res["configs"].append(row)
        print(json.dumps(row), flush=True)
with open(os.path.join(root, "gpurun_out", "clock_traffic.json"), "w") as fh:
    json.dump(res, fh, indent=1)
