"""Per-tile fixed cost of k_gemm (dev tool): time per tile slot (2 workgroups per CU, 512 slots)
against K, with and without the C preload (beta)."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
def run(mt, nt, K, ta=0, tb=0, lower=False, beta=1.0, reps=10):
    ms = ctx.bench_gemm(mt, nt, K, ta, tb, lower, beta, reps)
    tiles = mt * (mt + 1) // 2 if lower else mt * nt
    fl = 2.0 * tiles * 128 * 128 * K
    print(f"mt={mt:4d} nt={nt:4d} K={K:6d} ta={ta} tb={tb} beta={beta}: {ms:8.3f} ms {fl/ms/1e9:7.2f} TF/s  us/tile-slot {ms*1e3*512/tiles:7.1f}", flush=True)
for K in (256, 512, 1024, 2048, 4096):
    for beta in (1.0, 0.0):
        run(64, 64, K, beta=beta)
run(64, 72, 512)
run(64, 80, 512)
run(32, 32, 512)
