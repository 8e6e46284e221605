"""SQ counters for one GEMM configuration (dev tool; run on the box):
python tools/gemm_pmc.py mt nt K ta tb -- one rocprofv3 --pmc pass per counter group."""
import csv, glob, os, subprocess, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:6]
groups = [["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
          ["SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"],
          ["SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS"],
          ["SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_MFMA", "SQ_INSTS_VMEM_RD"]]
for gi, g in enumerate(groups):
    odir = os.path.join(root, "gpurun_out", f"gpmc{gi}")
    cmd = ["rocprofv3", "--pmc", *g, "-d", odir, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(root, "tools", "gemm_one.py"), *args, "1"]
    subprocess.run(cmd, check=True, cwd=root, env=dict(os.environ, TMPDIR="/tmp"), timeout=240)
    vals = {}
    for f in glob.glob(os.path.join(odir, "**", "*counter_collection*.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "k_gemm" in r.get("Kernel_Name", "")]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(gi, {k: f"{v:.4g}" for k, v in vals.items()}, flush=True)
