"""GEMM rate against K (dev tool): 64x64 tiles of the plain kernel, every layout, warm
(one untimed launch per configuration, then `reps`), K = 256 ... 4096."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
ks = (256, 512, 768, 1024, 1536, 2048, 3072, 4096)
for ta, tb in ((0, 0), (1, 1), (1, 0)):
    row = []
    for K in ks:
        ctx.bench_gemm(64, 64, K, ta, tb, False, 1.0, 2)
        ms = ctx.bench_gemm(64, 64, K, ta, tb, False, 1.0, 6 if K >= 2048 else 12)
        row.append("%d:%.1f" % (K, 2.0 * 64 * 64 * 128 * 128 * K / ms / 1e9))
    print("ta=%d tb=%d  %s" % (ta, tb, "  ".join(row)), flush=True)
