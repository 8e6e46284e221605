"""ctypes binding of libgpemu.so (the HIP/gfx950 hot path, include/gpemu.h).

There is no CPU fallback: if the library cannot be loaded, or no GPU is
visible, every entry point raises ``NativeUnavailable``.  The reference's
arithmetic (NumPy/SciPy, _emulatorkernels.py / _emulatoroptimise.py /
_emulatorclasses.py) is replaced here, not mirrored.
"""
from __future__ import annotations

import ctypes as _ct
import hashlib as _hashlib
import os as _os
import threading as _threading

import numpy as _np

_HERE = _os.path.dirname(_os.path.abspath(__file__))
_DEFAULT_LIB = _os.path.join(_HERE, "libgpemu.so")
LIB_PATH = _os.environ.get("GPEMU_LIB", _DEFAULT_LIB)

GPE_OK = 0
GPE_NOT_PD = 1
KERNEL_STD = 0
KERNEL_ALT_NUG = 1
GP4ML = 0
MUCM = 1

_D = _ct.POINTER(_ct.c_double)
_VP = _ct.c_void_p

# name -> (restype, argtypes); the full exported surface of include/gpemu.h
SIGNATURES = {
    "gpe_abi_version": (_ct.c_int, []),
    "gpe_build_id": (_ct.c_char_p, []),
    "gpe_device_count": (_ct.c_int, []),
    "gpe_device_synchronize": (_ct.c_int, [_ct.c_int32]),
    "gpe_create": (_VP, [_ct.c_int32]),
    "gpe_destroy": (None, [_VP]),
    "gpe_last_error": (_ct.c_char_p, [_VP]),
    "gpe_set_data": (_ct.c_int, [_VP, _ct.c_int64, _ct.c_int32, _ct.c_int32, _D, _D, _D, _D]),
    "gpe_objective": (_ct.c_int, [_VP, _ct.c_int32, _ct.c_int32, _D, _ct.c_int32, _ct.c_double,
                                  _ct.c_int32, _D, _D, _D]),
    "gpe_factor": (_ct.c_int, [_VP, _ct.c_int32, _D, _ct.c_double, _ct.c_double, _ct.c_double]),
    "gpe_beta": (_ct.c_int, [_VP, _D]),
    "gpe_posterior": (_ct.c_int, [_VP, _ct.c_int64, _D, _D, _D, _ct.c_double, _ct.c_int32, _ct.c_int32,
                                  _D, _D]),
    "gpe_noise_sample": (_ct.c_int, [_VP, _ct.c_int64, _D, _D, _D, _ct.c_double, _D, _ct.c_double,
                                     _D, _ct.c_int32, _D, _D, _D]),
    "gpe_solve": (_ct.c_int, [_VP, _ct.c_int32, _D, _D]),
    "gpe_sense_pairs": (_ct.c_int, [_VP, _ct.c_int32, _D, _D, _ct.c_int32, _D, _D, _D]),
    "gpe_gauss_transform": (_ct.c_int, [_VP, _ct.c_int64, _ct.c_int32, _ct.POINTER(_ct.c_int32), _D, _D, _D,
                                        _D]),
    "gpe_kernel_var": (_ct.c_int, [_VP, _ct.c_int32, _D, _ct.c_int32, _ct.c_double, _ct.c_int32,
                                   _ct.c_int64, _D, _D, _ct.c_double, _D]),
    "gpe_kernel_covar": (_ct.c_int, [_VP, _ct.c_int32, _D, _ct.c_int32, _ct.c_double, _ct.c_int64,
                                     _D, _ct.c_int64, _D, _D]),
    "gpe_kernel_grad": (_ct.c_int, [_VP, _D, _ct.c_int32, _ct.c_int64, _D, _D, _ct.c_double, _ct.c_double, _D]),
    "gpe_lhc_maximin": (_ct.c_int, [_VP, _ct.c_int32, _ct.c_int64, _ct.c_int32, _D, _ct.c_int64, _D,
                                    _ct.POINTER(_ct.c_int64)]),
    "gpe_cholesky": (_ct.c_int, [_VP, _ct.c_int64, _D, _D, _D, _D, _D]),
    "gpe_test_gemm": (_ct.c_int, [_VP, _ct.c_int32, _ct.c_int32, _ct.c_int64, _ct.c_int64,
                                  _ct.c_int64, _D, _D, _D, _ct.c_double, _ct.c_double]),
    "gpe_bench_gemm": (_ct.c_int, [_VP, _ct.c_int32, _ct.c_int32, _ct.c_int32, _ct.c_int32,
                                   _ct.c_int32, _ct.c_int32, _ct.c_double, _ct.c_int32, _D]),
    "gpe_set_profiling": (_ct.c_int, [_VP, _ct.c_int32]),
    "gpe_phase_times": (_ct.c_int, [_VP, _D, _ct.c_int32]),
    "gpe_gemm_stats": (_ct.c_int, [_VP, _D, _D, _D]),
    "gpe_ozaki_stats": (_ct.c_int, [_VP, _D, _D, _D, _D]),
    # include/gpemu_dist.h: row-block distributed value objective (RCCL / loopback)
    "gpe_dist_unique_id": (_ct.c_int, [_ct.c_char_p, _ct.c_int32]),
    "gpe_dist_create": (_VP, [_ct.c_int32, _ct.c_int32, _ct.c_int32, _ct.c_char_p]),
    "gpe_dist_destroy": (None, [_VP]),
    "gpe_dist_last_error": (_ct.c_char_p, [_VP]),
    "gpe_dist_set_data": (_ct.c_int, [_VP, _ct.c_int64, _ct.c_int32, _ct.c_int32, _D, _D, _D, _D]),
    "gpe_dist_objective": (_ct.c_int, [_VP, _ct.c_int32, _ct.c_int32, _D, _ct.c_int32, _ct.c_double,
                                       _ct.c_int32, _D, _D, _D]),
    "gpe_dist_owner": (_ct.c_int32, [_ct.c_int32, _ct.c_int32]),
    "gpe_dist_local_rows": (_ct.c_int32, [_ct.c_int64, _ct.c_int32, _ct.c_int32, _ct.c_int32]),
    "gpe_dist_times": (_ct.c_int, [_VP, _D, _D]),
    "gpe_dist_rank_bytes": (_ct.c_int, [_VP, _ct.c_int32, _ct.POINTER(_ct.c_int64)]),
}

UNIQUE_ID_BYTES = 128


class NativeUnavailable(RuntimeError):
    """libgpemu.so is missing or no HIP device is visible (no CPU fallback)."""


class NotPositiveDefinite(ArithmeticError):
    """Cholesky met a non-positive / NaN pivot (the reference's LinAlgError)."""


_lib = None
_lib_lock = _threading.Lock()


def load_library(path: str | None = None):
    """Load and type the shared library (idempotent)."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not _os.path.exists(p):
            raise NativeUnavailable(
                f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = _ct.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        # provenance: the in-tree library must be built from the sources beside it (a
        # probe build named by GPEMU_LIB or `path` is the caller's choice)
        from . import buildinfo
        want = buildinfo.source_hash() if p == _DEFAULT_LIB else None
        have = lib.gpe_build_id().decode()
        if want is not None and have != want:
            raise NativeUnavailable(
                f"{p} was built from other sources (build id {have[:12]}, sources {want[:12]}): "
                "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")
        if path is None:
            _lib = lib
        return lib


def build_id() -> str:
    """SHA-256 of the sources the loaded library was built from."""
    return load_library().gpe_build_id().decode()


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(_D)


def _f64(a, shape=None):
    arr = _np.ascontiguousarray(a, dtype=_np.float64)
    if shape is not None:
        arr = arr.reshape(shape)
    return arr


class Context:
    """One GPU, one HIP stream, resident training data (gpe_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        if self.lib.gpe_device_count() <= 0:
            raise NativeUnavailable("no HIP device visible to libgpemu.so")
        h = self.lib.gpe_create(int(device))
        if not h:
            raise NativeUnavailable("gpe_create failed: " + self.lib.gpe_last_error(None).decode())
        self._h = h
        self.device = device
        self.n = self.d = self.q = 0
        self._data_key = None
        self._factor_key = None

    # -- lifetime
    def close(self):
        if getattr(self, "_h", None):
            self.lib.gpe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc == GPE_OK:
            return
        msg = self.lib.gpe_last_error(self._h).decode()
        if rc == GPE_NOT_PD:
            raise NotPositiveDefinite(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")

    # -- data
    def set_data(self, X, f, H, r=None):
        X = _f64(X)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        n, d = X.shape
        f = _f64(f, (n,))
        H = _f64(H)
        if H.ndim == 1:
            H = H.reshape(n, -1)
        q = H.shape[1]
        rr = None if r is None or _np.isscalar(r) else _f64(r, (n,))
        self._keep = (X, f, H, rr)
        self._data_key = None
        self._factor_key = None
        self._check(self.lib.gpe_set_data(self._h, n, d, q, _ptr(X), _ptr(f), _ptr(H), _ptr(rr)),
                    "gpe_set_data")
        self.n, self.d, self.q = n, d, q

    @staticmethod
    def _digest(*arrays):
        h = _hashlib.blake2b(digest_size=16)
        for a in arrays:
            if a is None:
                h.update(b"-")
            else:
                a = _np.ascontiguousarray(a, dtype=_np.float64)
                h.update(str(a.shape).encode())
                h.update(a.tobytes())
        return h.hexdigest()

    def ensure_data(self, X, f, H, r=None):
        """set_data unless this exact (X, f, H, r) is already resident."""
        key = self._digest(X, f, H, r)
        if key != self._data_key:
            self.set_data(X, f, H, r)
            self._data_key = key

    def ensure_factor(self, kernel, delta, nu, s2=1.0, r_scale=0.0):
        """factor() unless the same factor of the resident data is already held."""
        key = (int(kernel), tuple(_np.asarray(delta, float).ravel().tolist()), float(nu), float(s2),
               float(r_scale), self._data_key)
        if key != self._factor_key or self._data_key is None:
            self._factor_key = None
            self.factor(kernel, delta, nu, s2, r_scale)
            self._factor_key = key

    # -- objective
    def objective(self, variant, kernel, hp, nu_fixed=0.0, want_grad=True):
        """Returns (llh, grad or None, sigma2); raises NotPositiveDefinite."""
        hp = _f64(hp).ravel()
        llh = _ct.c_double(0.0)
        s2 = _ct.c_double(0.0)
        grad = _np.zeros(hp.size) if want_grad else None
        self._factor_key = None            # the objective reuses the factor buffers
        rc = self.lib.gpe_objective(self._h, int(variant), int(kernel), _ptr(hp), hp.size,
                                    float(nu_fixed), 1 if want_grad else 0, _ct.byref(llh),
                                    _ptr(grad), _ct.byref(s2))
        self._check(rc, "gpe_objective")
        return llh.value, grad, s2.value

    def factor(self, kernel, delta, nu, s2=1.0, r_scale=0.0):
        self._factor_key = None
        delta = _f64(delta).ravel()
        self._check(self.lib.gpe_factor(self._h, int(kernel), _ptr(delta), float(nu), float(s2),
                                        float(r_scale)), "gpe_factor")

    def beta(self):
        out = _np.zeros(self.q)
        self._check(self.lib.gpe_beta(self._h, _ptr(out)), "gpe_beta")
        return out

    def posterior(self, Xs, Hs, beta, sigma, full_var=True, precision=64):
        """(mean, var): var is m x m when full_var, else its diagonal.  The L^-1 K* product
        runs as exact int8 products (4096 <= n_pad <= 32768): of 53-bit operands at precision
        64, of 24-bit ones at precision=32 (diagonal variance only; fp32 MFMA outside that
        range or with GPEMU_OZAKI=0)."""
        if precision not in (32, 64):
            raise ValueError("precision must be 32 or 64")
        Xs = _f64(Xs)
        if Xs.ndim == 1:
            Xs = Xs.reshape(-1, 1)
        m = Xs.shape[0]
        Hs = _f64(Hs, (m, self.q))
        beta = _f64(beta).ravel()
        mean = _np.zeros(m)
        var = _np.zeros((m, m)) if full_var else _np.zeros(m)
        self._check(self.lib.gpe_posterior(self._h, m, _ptr(Xs), _ptr(Hs), _ptr(beta), float(sigma),
                                           1 if full_var else 0, int(precision), _ptr(mean), _ptr(var)),
                    "gpe_posterior")
        return mean, var

    def noise_sample(self, Xs, Hs, beta, sigma, t, U, r_new=None, r_scale=0.0):
        """noise_fit's estimation step for the resident factor: the posterior at Xs
        (full covariance V, plus r_scale * r_new on its diagonal), L = chol(V) and
        sum_j 0.5 (t - mean - L U[j])^2 over the rows of U (s x m).  Returns
        (mean, that sum).  NotPositiveDefinite when V is not."""
        Xs = _f64(Xs)
        if Xs.ndim == 1:
            Xs = Xs.reshape(-1, 1)
        m = Xs.shape[0]
        Hs = _f64(Hs, (m, self.q))
        beta = _f64(beta).ravel()
        t = _f64(t, (m,))
        U = _f64(U)
        U = U.reshape(-1, m)
        rn = None if r_new is None else _f64(r_new, (m,))
        mean = _np.zeros(m)
        z = _np.zeros(m)
        self._check(self.lib.gpe_noise_sample(self._h, m, _ptr(Xs), _ptr(Hs), _ptr(beta), float(sigma),
                                              _ptr(rn), float(r_scale), _ptr(t), U.shape[0], _ptr(U),
                                              _ptr(mean), _ptr(z)), "gpe_noise_sample")
        return mean, z

    # -- sensitivity building blocks (resident factor)
    def solve(self, B):
        """A^-1 B for the resident factor (B: n or n x k)."""
        B = _f64(B)
        vec = B.ndim == 1
        B2 = B.reshape(self.n, -1)
        B2 = _np.ascontiguousarray(B2)
        X = _np.zeros_like(B2)
        self._check(self.lib.gpe_solve(self._h, B2.shape[1], _ptr(B2), _ptr(X)), "gpe_solve")
        return X.ravel() if vec else X

    def sense_pairs(self, w, u, Z):
        """For K_j(k,l) = u[j,k] u[j,l] exp(-sum_i w[j,i] (x_ki - x_li)^2):
        (tr(A^-1 K_j) for each j, Z^T K_j Z for each j)."""
        w = _np.ascontiguousarray(_f64(w).reshape(-1, self.d))
        J = w.shape[0]
        u = _np.ascontiguousarray(_f64(u).reshape(J, self.n))
        Z = _np.ascontiguousarray(_f64(Z).reshape(self.n, -1))
        p = Z.shape[1]
        tr = _np.zeros(J)
        quad = _np.zeros((J, p, p))
        self._check(self.lib.gpe_sense_pairs(self._h, J, _ptr(w), _ptr(u), p, _ptr(Z), _ptr(tr), _ptr(quad)),
                    "gpe_sense_pairs")
        return tr, quad

    def gauss_transform(self, dims, c, Y, a):
        """out[t] = sum_k a[k] exp(-sum_s c[s] (Y[t,s] - x[k, dims[s]])^2)."""
        dims_a = _np.ascontiguousarray(_np.asarray(dims, dtype=_np.int32).ravel())
        ns = dims_a.size
        c = _np.ascontiguousarray(_f64(c).ravel())
        Y = _np.ascontiguousarray(_f64(Y).reshape(-1, ns))
        a = _np.ascontiguousarray(_f64(a).ravel())
        if a.size != self.n or c.size != ns:
            raise ValueError("gauss_transform: a must have n entries and c one per dimension")
        out = _np.zeros(Y.shape[0])
        self._check(self.lib.gpe_gauss_transform(self._h, Y.shape[0], ns,
                                                 dims_a.ctypes.data_as(_ct.POINTER(_ct.c_int32)), _ptr(c),
                                                 _ptr(Y), _ptr(a), _ptr(out)), "gpe_gauss_transform")
        return out

    def kernel_var(self, kernel, delta, nu, X, predict=True, r=None, r_scale=0.0):
        X = _f64(X)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        m, d = X.shape
        delta = _f64(delta).ravel()
        rr = None if r is None or _np.isscalar(r) else _f64(r, (m,))
        out = _np.zeros((m, m))
        self._check(self.lib.gpe_kernel_var(self._h, int(kernel), _ptr(delta), d, float(nu),
                                            1 if predict else 0, m, _ptr(X), _ptr(rr),
                                            float(r_scale), _ptr(out)), "gpe_kernel_var")
        return out

    def kernel_covar(self, kernel, delta, nu, XT, XV):
        XT = _f64(XT)
        XV = _f64(XV)
        if XT.ndim == 1:
            XT = XT.reshape(-1, 1)
        if XV.ndim == 1:
            XV = XV.reshape(-1, 1)
        n, d = XT.shape
        m = XV.shape[0]
        delta = _f64(delta).ravel()
        out = _np.zeros((n, m))
        self._check(self.lib.gpe_kernel_covar(self._h, int(kernel), _ptr(delta), d, float(nu), n,
                                              _ptr(XT), m, _ptr(XV), _ptr(out)), "gpe_kernel_covar")
        return out

    def kernel_grad(self, delta, X, col, col_scale, pre):
        """pre * ((col_k - col_l) col_scale)^2 * exp(-|(x_k - x_l)/delta|^2), zero
        diagonal (col None: no squared factor); m x m."""
        X = _f64(X)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        m, d = X.shape
        delta = _f64(delta).ravel()
        cc = None if col is None else _f64(col, (m,))
        out = _np.zeros((m, m))
        self._check(self.lib.gpe_kernel_grad(self._h, _ptr(delta), d, m, _ptr(X), _ptr(cc),
                                             float(col_scale), float(pre), _ptr(out)), "gpe_kernel_grad")
        return out

    def lhc_maximin(self, designs, fextra=None):
        """np.argmin(pdist([designs[k]; fextra], 'sqeuclidean')) for every candidate
        design k (designs: N x n x dim) -> int64 array of N condensed indices."""
        designs = _f64(designs)
        N, n, dim = designs.shape
        fe = None if fextra is None else _f64(fextra).reshape(-1, dim)
        ne = 0 if fe is None else fe.shape[0]
        out = _np.zeros(N, dtype=_np.int64)
        self._check(self.lib.gpe_lhc_maximin(self._h, N, n, dim, _ptr(designs), ne, _ptr(fe),
                                             out.ctypes.data_as(_ct.POINTER(_ct.c_int64))), "gpe_lhc_maximin")
        return out

    def cholesky(self, A, want=("L",)):
        A = _f64(A)
        m = A.shape[0]
        outs = {k: _np.zeros((m, m)) for k in want if k in ("L", "Linv", "Ainv")}
        ld = _ct.c_double(0.0)
        self._check(self.lib.gpe_cholesky(self._h, m, _ptr(A), _ptr(outs.get("L")),
                                          _ptr(outs.get("Linv")), _ptr(outs.get("Ainv")),
                                          _ct.byref(ld)), "gpe_cholesky")
        outs["logdet"] = ld.value
        return outs

    def test_gemm(self, A, B, C, alpha=1.0, beta=0.0, trans_a=0, trans_b=0):
        A = _f64(A)
        B = _f64(B)
        C = _f64(C).copy()
        M, K = A.shape
        N = B.shape[1]
        self._check(self.lib.gpe_test_gemm(self._h, int(trans_a), int(trans_b), M, N, K, _ptr(A),
                                           _ptr(B), _ptr(C), float(alpha), float(beta)),
                    "gpe_test_gemm")
        return C

    def bench_gemm(self, mt, nt, K, trans_a=0, trans_b=0, lower=False, beta=1.0, reps=5):
        ms = _ct.c_double()
        self._check(self.lib.gpe_bench_gemm(self._h, int(trans_a), int(trans_b), int(mt), int(nt),
                                            int(K), 1 if lower else 0, float(beta), int(reps),
                                            _ct.byref(ms)), "gpe_bench_gemm")
        return ms.value

    # -- profiling
    def set_profiling(self, on=True):
        self._check(self.lib.gpe_set_profiling(self._h, 1 if on else 0), "gpe_set_profiling")

    def phase_times(self):
        out = _np.zeros(8)
        self._check(self.lib.gpe_phase_times(self._h, _ptr(out), 8), "gpe_phase_times")
        keys = ["kbuild", "cholesky", "trtri", "inverse", "skinny", "contract", "total"]
        return dict(zip(keys, out[:7].tolist()))

    def gemm_stats(self):
        ms, nl, fl = _ct.c_double(), _ct.c_double(), _ct.c_double()
        self._check(self.lib.gpe_gemm_stats(self._h, _ct.byref(ms), _ct.byref(nl), _ct.byref(fl)),
                    "gpe_gemm_stats")
        return {"ms": ms.value, "launches": nl.value, "flops": fl.value}

    def ozaki_stats(self):
        """k_oz_gemm launches of the most recent objective (profiling on): ms, launches,
        int8 ops and the fp64 flops of the products they emulate."""
        ms, nl, ops, fl = _ct.c_double(), _ct.c_double(), _ct.c_double(), _ct.c_double()
        self._check(self.lib.gpe_ozaki_stats(self._h, _ct.byref(ms), _ct.byref(nl), _ct.byref(ops), _ct.byref(fl)),
                    "gpe_ozaki_stats")
        return {"ms": ms.value, "launches": nl.value, "int8_ops": ops.value, "fp64_flops": fl.value}


_default_ctx = None
_ctx_lock = _threading.Lock()


_tls = _threading.local()
_extra_ctxs: list = []


def default_context() -> Context:
    """The calling thread's bound context (bind_context), else the process-wide
    context on the GPU chosen by GPEMU_DEVICE / LOCAL_RANK (or 0)."""
    bound = getattr(_tls, "ctx", None)
    if bound is not None:
        return bound
    global _default_ctx
    with _ctx_lock:
        if _default_ctx is None:
            dev = int(_os.environ.get("GPEMU_DEVICE", _os.environ.get("LOCAL_RANK", "0")))
            _default_ctx = Context(dev)
        return _default_ctx


class bind_context:
    """Route default_context() of the current thread to `ctx` inside the block
    (worker threads of concurrent multistart tries, optimize.py)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def __enter__(self):
        self.prev = getattr(_tls, "ctx", None)
        _tls.ctx = self.ctx
        return self.ctx

    def __exit__(self, *exc):
        _tls.ctx = self.prev
        return False


def worker_contexts(k: int) -> list:
    """k contexts on the default context's GPU: the default one plus k-1 extra,
    created once and kept (each has its own HIP stream and workspaces)."""
    base = default_context()
    with _ctx_lock:
        while len(_extra_ctxs) < k - 1:
            _extra_ctxs.append(Context(base.device))
        return [base] + _extra_ctxs[:k - 1]


class DistContext:
    """Row-block distributed objective and gradient over P GPUs (include/gpemu_dist.h).

    unique_id=None selects the in-process loopback transport: all `nranks`
    logical ranks run in this process on `device` (same partition and schedule,
    device copies instead of RCCL).  With a unique id (bytes from
    ``dist_unique_id()`` on rank 0, shared by the host, see distributed.py) this
    process is rank `rank` of an RCCL communicator of `nranks` GPUs.
    """

    def __init__(self, device: int, nranks: int, rank: int = 0, unique_id: bytes | None = None):
        self.lib = load_library()
        if self.lib.gpe_device_count() <= 0:
            raise NativeUnavailable("no HIP device visible to libgpemu.so")
        if unique_id is not None and len(unique_id) != UNIQUE_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        h = self.lib.gpe_dist_create(int(device), int(nranks), int(rank), unique_id)
        if not h:
            raise NativeUnavailable("gpe_dist_create failed")
        self._h = h
        self.nranks, self.rank, self.loopback = nranks, rank, unique_id is None

    def close(self):
        if getattr(self, "_h", None):
            self.lib.gpe_dist_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc == GPE_OK:
            return
        msg = self.lib.gpe_dist_last_error(self._h).decode()
        if rc == GPE_NOT_PD:
            raise NotPositiveDefinite(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")

    def set_data(self, X, f, H, r=None):
        X = _f64(X)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        n, d = X.shape
        f = _f64(f, (n,))
        H = _f64(H)
        if H.ndim == 1:
            H = H.reshape(n, -1)
        rr = None if r is None or _np.isscalar(r) else _f64(r, (n,))
        self._keep = (X, f, H, rr)
        self._check(self.lib.gpe_dist_set_data(self._h, n, d, H.shape[1], _ptr(X), _ptr(f), _ptr(H),
                                               _ptr(rr)), "gpe_dist_set_data")

    def objective(self, variant, kernel, hp, nu_fixed=0.0, want_grad=False):
        """Objective (collective over all ranks): (llh, sigma2), or (llh, grad, sigma2)
        with want_grad."""
        hp = _f64(hp).ravel()
        llh, s2 = _ct.c_double(0.0), _ct.c_double(0.0)
        grad = _np.zeros(hp.size) if want_grad else None
        self._check(self.lib.gpe_dist_objective(self._h, int(variant), int(kernel), _ptr(hp), hp.size,
                                                float(nu_fixed), int(bool(want_grad)), _ct.byref(llh),
                                                _ptr(grad), _ct.byref(s2)),
                    "gpe_dist_objective")
        if want_grad:
            return llh.value, grad, s2.value
        return llh.value, s2.value

    def times(self):
        tot, comm = _ct.c_double(0.0), _ct.c_double(0.0)
        self._check(self.lib.gpe_dist_times(self._h, _ct.byref(tot), _ct.byref(comm)), "gpe_dist_times")
        return {"total_ms": tot.value, "comm_ms": comm.value}

    def rank_bytes(self, rank: int | None = None) -> int:
        """Device bytes held for `rank` (default: this process's rank; any logical
        rank in loopback)."""
        b = _ct.c_int64(0)
        r = self.rank if rank is None else int(rank)
        self._check(self.lib.gpe_dist_rank_bytes(self._h, r, _ct.byref(b)), "gpe_dist_rank_bytes")
        return int(b.value)


def device_synchronize(device: int) -> None:
    """Wait for all work on GPU `device` (no PyTorch in the process)."""
    rc = load_library().gpe_device_synchronize(int(device))
    if rc != GPE_OK:
        raise RuntimeError(f"gpe_device_synchronize({device}) failed ({rc})")


def dist_unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 only)."""
    lib = load_library()
    buf = _ct.create_string_buffer(UNIQUE_ID_BYTES)
    rc = lib.gpe_dist_unique_id(buf, UNIQUE_ID_BYTES)
    if rc != GPE_OK:
        raise RuntimeError(f"gpe_dist_unique_id failed ({rc})")
    return buf.raw


def dist_owner(nranks: int, tile_row: int) -> int:
    """Rank that stores 128-row tile row `tile_row` (pure; no GPU)."""
    return int(load_library().gpe_dist_owner(int(nranks), int(tile_row)))


def dist_local_rows(n: int, nranks: int, rank: int, q: int = 0) -> int:
    """Tile rows rank `rank` stores for n points and q basis columns, including its
    share of the ceil((q+1)/128) augmented [f H]^T rows (pure; no GPU)."""
    return int(load_library().gpe_dist_local_rows(int(n), int(q), int(nranks), int(rank)))
