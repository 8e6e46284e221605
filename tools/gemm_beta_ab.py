"""Plain GEMM at short K with and without C (beta 1 / 0), 64x64 tiles, NN (dev tool):
how much of the short-K rate goes to reading and writing C."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
for K in (256, 512, 1024, 4096):
    row = []
    for beta in (1.0, 0.0):
        ctx.bench_gemm(64, 64, K, 0, 0, False, beta, 2)
        ms = min(ctx.bench_gemm(64, 64, K, 0, 0, False, beta, 6 if K >= 2048 else 12) for _ in range(3))
        row.append("beta %.0f: %.1f TF/s" % (beta, 2.0 * 64 * 64 * 128 * 128 * K / ms / 1e9))
    print("K=%d  %s" % (K, "  ".join(row)), flush=True)
