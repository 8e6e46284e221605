"""GEMM building-block sweep (dev tool): TF/s vs K, layout, beta."""
import sys
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
def run(mt, nt, K, ta=0, tb=0, lower=False, beta=1.0, reps=5):
    ms = ctx.bench_gemm(mt, nt, K, ta, tb, lower, beta, reps)
    tiles = mt * (mt + 1) // 2 if lower else mt * nt
    fl = 2.0 * tiles * 128 * 128 * K
    print(f"mt={mt:4d} nt={nt:4d} K={K:6d} ta={ta} tb={tb} lower={int(lower)} beta={beta}: {ms:9.3f} ms  {fl/ms/1e9:7.2f} TF/s  per-tile-CU {ms*1e3*256/tiles:7.1f} us", flush=True)
for K in (128, 256, 512, 1024, 4096):
    run(64, 64, K)
for K in (128, 256, 512):
    run(127, 127, K, lower=True)
run(64, 64, 128, beta=0.0)
run(64, 64, 1024, 1, 1)
run(64, 64, 1024, 1, 0)
run(64, 64, 1024, 0, 1)
