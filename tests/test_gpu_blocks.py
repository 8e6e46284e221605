"""GPU parity of the building blocks: MFMA GEMM forms and the blocked Cholesky."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


# K = 144: 9 K stages, C preloaded; K = 160 (10 stages, the shortest) and 512: the CDEF
# instances, C added chunk by chunk inside the K loop (csrc/gpemu_kernels.hpp, c_chunk_load)
@pytest.mark.parametrize("K", [144, 160, 512])
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0), (1, 1), (0, 1)])
def test_gemm_forms(ctx, ta, tb, K):
    rs = np.random.RandomState(ta * 2 + tb + K)
    M, N = 256, 384
    A = rs.standard_normal((M, K))
    B = rs.standard_normal((K, N))
    C = rs.standard_normal((M, N))
    out = ctx.test_gemm(A, B, C, alpha=-0.7, beta=0.3, trans_a=ta, trans_b=tb)
    ref = -0.7 * A @ B + 0.3 * C
    assert np.max(np.abs(out - ref)) < 1e-12 * np.max(np.abs(ref)) * K


def test_gemm_exact_integer_layout(ctx):
    # A = I, asymmetric integer B: catches any row/column swap in the MFMA map
    M = N = 128
    K = 128
    A = np.eye(M)
    B = np.arange(K * N, dtype=float).reshape(K, N) % 97
    out = ctx.test_gemm(A, B, np.zeros((M, N)))
    assert np.array_equal(out, B)


@pytest.mark.parametrize("m", [1, 100, 128, 300, 700])
def test_cholesky_inverse(ctx, m):
    rs = np.random.RandomState(m)
    G = rs.standard_normal((m, m))
    A = G @ G.T / m + np.eye(m)
    out = ctx.cholesky(A, want=("L", "Linv", "Ainv"))
    L = np.linalg.cholesky(A)
    assert np.max(np.abs(out["L"] - L)) < 1e-12 * np.max(np.abs(L)) * 10
    assert np.max(np.abs(out["Linv"] - np.linalg.inv(L))) < 1e-10
    assert np.max(np.abs(out["Ainv"] - np.linalg.inv(A))) < 1e-10
    assert abs(out["logdet"] - np.linalg.slogdet(A)[1]) < 1e-10 * m


def test_cholesky_not_pd(ctx):
    from gp_emu_uqsa_amd import native
    A = np.ones((200, 200))
    with pytest.raises(native.NotPositiveDefinite):
        ctx.cholesky(A)
