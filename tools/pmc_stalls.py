"""Where the Cholesky's short-K bulk loses against the long-K LAUUM (dev tool, run on the
GPU box): per-phase sums of SQ wave-state, LDS, vector-memory and TA/TCP stall counters
over one objective evaluation (tools/prof_objective.py), one rocprofv3 --pmc pass per
counter set (gfx950 block limits: <= 8 SQ, 2 TA, 4 TCP, 2 GRBM per pass).  Ratios are
per wave-cycle (SQ_* / SQ_WAVE_CYCLES) or per GUI-active cycle; phases as
tools/pmc_phases.py.  usage: python tools/pmc_stalls.py [n] [d]"""
import csv
import glob
import json
import os
import subprocess
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if len(args) > 0 else 16384
d = int(args[1]) if len(args) > 1 else 10
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
passes = [["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
           "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"],
          ["SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VALU_MFMA_F64",
           "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INST_LEVEL_VMEM", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"],
          ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
           "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum", "TCP_TCC_WRITE_REQ_sum", "GRBM_GUI_ACTIVE"]]
analyze_only = "--analyze" in sys.argv   # re-read gpurun_out/pmc_stall*/ without collecting
launches = None
for i, counters in enumerate(passes):
    odir = os.path.join(root, "gpurun_out", f"pmc_stall{i}")
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "-d", odir, "-o", "run",
           "--output-format", "csv", "--", sys.executable, os.path.join(root, "tools", "prof_objective.py"),
           str(n), str(d), "1"]
    if not analyze_only:
        subprocess.run(cmd, check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"))
    rows = {}
    for f in glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_gemm" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            e = rows.setdefault(k, {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [rows[k] for k in sorted(rows)]
    if launches is None:
        launches = seq
    else:
        assert len(seq) == len(launches), (len(seq), len(launches))
        for a, b in zip(launches, seq):
            for key, v in b.items():
                if key != "ns":
                    a[key] = v
assert len(launches) == 143, len(launches)
groups = {"chol 1-47": launches[1:48], "chol 48-87": launches[48:88], "chol 88-127": launches[88:128],
          "trtri": launches[128:142], "lauum": launches[142:143]}
out = {"n": n, "d": d, "phases": {}}
for name, ls in groups.items():
    s = {}
    for e in ls:
        for k, v in e.items():
            s[k] = s.get(k, 0.0) + v
    wc = max(s.get("SQ_WAVE_CYCLES", 1.0), 1.0)
    gui = max(s.get("GRBM_GUI_ACTIVE", 1.0), 1.0)
    rec = {"ms": s["ns"] / 1e6, "raw": {k: v for k, v in s.items() if k != "ns"}}
    for k in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
        rec[k + "/wave_cycle"] = s.get(k, 0.0) / wc
    rec["lds_conflict_per_lds_inst"] = s.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(s.get("SQ_INSTS_LDS", 1.0), 1.0)
    rec["vmem_rd_per_mfma"] = s.get("SQ_INSTS_VMEM_RD", 0.0) / max(s.get("SQ_INSTS_VALU_MFMA_F64", 1.0), 1.0)
    rec["vmem_wr_per_mfma"] = s.get("SQ_INSTS_VMEM_WR", 0.0) / max(s.get("SQ_INSTS_VALU_MFMA_F64", 1.0), 1.0)
    rec["tcp_read_latency_avg"] = s.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / max(s.get("TCP_TCC_READ_REQ_sum", 1.0), 1.0)
    rec["ta_busy_per_gui"] = s.get("TA_TA_BUSY_sum", 0.0) / gui
    rec["tcp_pending_stall_per_gui"] = s.get("TCP_PENDING_STALL_CYCLES_sum", 0.0) / gui
    out["phases"][name] = rec
print(json.dumps(out, indent=1))
