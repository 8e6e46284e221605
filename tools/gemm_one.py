"""One GEMM configuration for counter collection (dev tool): mt nt K ta tb reps."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
mt, nt, K, ta, tb, reps = (int(a) for a in sys.argv[1:7])
ctx = native.Context(0)
ms = ctx.bench_gemm(mt, nt, K, ta, tb, False, 1.0, reps)
print(f"{mt}x{nt}x{K} ta={ta} tb={tb}: {ms:.3f} ms {2.0 * mt * nt * 128 * 128 * K / ms / 1e9:.2f} TF/s")
