"""GEMM rate of the loaded library (GPEMU_LIB) for each operand layout and a few K
(dev tool, 64x64 tiles, beta = 1)."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
for ta, tb in ((0, 0), (1, 0), (1, 1), (0, 1)):
    row = []
    for K in (128, 512, 4096):
        reps = 3 if K >= 4096 else 10
        ctx.bench_gemm(64, 64, K, ta, tb, False, 1.0, 1)
        ms = ctx.bench_gemm(64, 64, K, ta, tb, False, 1.0, reps)
        row.append("K=%d %.2f" % (K, 2.0 * 64 * 64 * 128 * 128 * K / ms / 1e9))
    print("ta=%d tb=%d: %s TF/s" % (ta, tb, "  ".join(row)), flush=True)
