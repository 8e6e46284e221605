"""Run gpe_cholesky on 128x128 SPD tiles (diag kernel timing under rocprof)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from gp_emu_uqsa_amd import native
ctx = native.Context(0)
rs = np.random.RandomState(0)
G = rs.standard_normal((128, 128))
A = G @ G.T / 128 + np.eye(128)
for _ in range(5):
    ctx.cholesky(A, want=("L",))
print("ok")
