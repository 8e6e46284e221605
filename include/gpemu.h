/*
 * gpemu.h -- C-ABI of libgpemu.so, the MI355X (gfx950) GP-emulator hot path.
 *
 * The reference (MathThyMod/GP_emu_UQSA) is pure Python and has no FFI: its
 * seams are duck-typed Python objects.  Each entry point below
 * replaces one of them; the reference interface it stands in for is cited.
 * The library is bound by the package's own ctypes layer
 * (gp_emu_uqsa_amd/native.py); INTEGRATION.md shows the binding a reference
 * maintainer would add.
 *
 * Conventions
 *  - All host buffers are caller-owned, C-contiguous (row-major) fp64 and are
 *    only read/written during the call.  Device buffers belong to the context.
 *  - Calls are synchronous: the context's HIP stream is drained before return.
 *  - One context per host thread, one GPU per context.  No callbacks.
 *  - Return codes: GPE_OK (0); GPE_NOT_PD (1) = Cholesky met a non-positive or
 *    NaN pivot, or a length scale is zero / NaN (the reference's covariance is NaN
 *    there) -- the host maps it to the reference's `return None`
 *    (_emulatoroptimise.py:374-376, :489-491); negative = error, text in
 *    gpe_last_error().
 *  - Hyperparameters are UNtransformed (delta, nu, sigma); transform /
 *    untransform x = 2 log(hp) stays on the host (_emulatorkernels.py:31-36).
 */
#ifndef GPEMU_H
#define GPEMU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPE_ABI_VERSION 10  /* 3: gpe_dist_objective gained want_grad / grad_out; 4: sensitivity;
                                5: gpe_noise_sample (noise_fit); 6: gpe_kernel_grad;
                                7: gpe_lhc_maximin; 8: gpe_dist_rank_bytes,
                                gpe_device_synchronize, gpe_build_id;
                                9: gpe_dist_local_rows takes the basis width q;
                                10: gpe_ozaki_stats */

enum gpe_status {
    GPE_OK = 0,
    GPE_NOT_PD = 1,
    GPE_ERR_ARG = -1,
    GPE_ERR_HIP = -2,
    GPE_ERR_ALLOC = -3,
    GPE_ERR_STATE = -4,
    GPE_ERR_UNSUPPORTED = -5
};

/* kernel family: _emulatorkernels.py:10 (kernel) and :83 (kernel_alt_nug) */
enum gpe_kernel { GPE_KERNEL_STD = 0, GPE_KERNEL_ALT_NUG = 1 };
/* objective: _emulatoroptimise.py:412 (gp4ml) and :305 (mucm) */
enum gpe_variant { GPE_GP4ML = 0, GPE_MUCM = 1 };

/* Input dimensions d and columns q + 1 of [f H] (the reference's linear mean has
 * q = d + 1) take any value, as in the reference (_emulatorkernels.py:39-50): the
 * kernels for d <= 32 and q + 1 <= 33 keep coordinates and basis rows in registers,
 * beyond that they stage them through LDS in chunks of 32.  The two constants below
 * are only the sizes a context's small per-dimension / per-column buffers start at
 * (they grow with the data); they are no longer limits (ABI version 8 and later). */
#define GPE_MAX_DIMS 128
#define GPE_MAX_COLS 128

typedef struct gpe_ctx gpe_ctx;

int gpe_abi_version(void);
/* SHA-256 (hex) of the sources the library was built from (gp_emu_uqsa_amd/buildinfo.py). */
const char* gpe_build_id(void);
int gpe_device_count(void);
/* Wait for all work on GPU `device` (the timed-region bracket of bench.py). */
int gpe_device_synchronize(int32_t device);

/* Create a context on one GPU (device index as HIP sees it). NULL on failure;
 * the reason is then available from gpe_last_error(NULL). */
gpe_ctx* gpe_create(int32_t device);
void gpe_destroy(gpe_ctx* ctx);
const char* gpe_last_error(const gpe_ctx* ctx);

/* Training data: replaces Data.inputs/.outputs/.H/.r (_emulatorclasses.py:540-550,
 * :577-584).  X n x d (already active-column-selected and [0,1]-scaled, as
 * All_Data leaves it), f n, H n x q, r n or NULL (r = 0).  Copies to HBM. */
int gpe_set_data(gpe_ctx* ctx, int64_t n, int32_t d, int32_t q,
                 const double* X, const double* f, const double* H, const double* r);

/* Objective: replaces Optimize.loglikelihood_gp4ml (_emulatoroptimise.py:412-493)
 * and Optimize.loglikelihood_mucm (:305-378).
 * hp = untransformed [delta(d), nu (if fitted), sigma (gp4ml only)], n_hp its
 * length; the nugget is fitted iff n_hp == d+2 (gp4ml) / d+1 (mucm), exactly the
 * reference's `x.size` test (:463, :360).  nu_fixed is used otherwise.
 * Outputs: *llh_out = the reference's LLH (negative log marginal likelihood);
 * grad_out (n_hp, may be NULL when want_grad == 0) = its gradient w.r.t.
 * x = 2 log(hp), including the MUCM sigma-hat^2 scaling the reference applies;
 * *sigma2_out = sigma^2 (gp4ml) or the analytic sigma-hat^2 (mucm, :324-327).
 * want_grad == 0 (sigma_analytic_mucm, :382-408) runs K-build, Cholesky and a forward
 * substitution for L^-1 [f H] only: no triangular inverse and no A^-1. */
int gpe_objective(gpe_ctx* ctx, int32_t variant, int32_t kernel,
                  const double* hp, int32_t n_hp, double nu_fixed, int32_t want_grad,
                  double* llh_out, double* grad_out, double* sigma2_out);

/* Factor A = s2 * K.var(X_train, predict=True) + r_scale * diag(r) and keep the
 * Cholesky factor and its inverse resident for gpe_beta / gpe_posterior.
 * Replaces the factorisations inside Optimize.optimalbeta (:497-504) and the
 * three scipy.linalg.solve(A, .) LU solves of Posterior (_emulatorclasses.py:613,
 * :623, :628).  r_scale is 1/s2 after training's make_A(s2) and 1 after remake(). */
int gpe_factor(gpe_ctx* ctx, int32_t kernel, const double* delta, double nu,
               double s2, double r_scale);

/* GLS beta = Q^-1 H^T A^-1 f with the resident factor (optimalbeta, :497-504).  Needs
 * only L: L^-1 [f H] by forward substitution with the Cholesky's diagonal-tile inverses
 * (no n^3/3 triangular inverse; that runs on demand for the posterior-side entries). */
int gpe_beta(gpe_ctx* ctx, double* beta_out);

/* Posterior at m points: replaces Posterior.make_covar/make_mean/make_var
 * (_emulatorclasses.py:607-631) with the resident factor.  Xs m x d, Hs m x q.
 * mean_out m; var_out m x m (row-major) when full_var != 0, else its diagonal
 * (m values); any m, in chunks of 16384 points (full: blocks of the m x m result
 * formed on the device and written to the host).  sigma is par.sigma.
 * precision 64: fp64 accuracy; for 4096 <= n_pad <= 32768 the dominant product
 * L^-1 K* (n^2 m flops) runs as exact int8 products of 53-bit operands (16 moduli).
 * precision 32 (diagonal only; SURVEY 8b/8d, BASELINE config C5): that product from
 * 24-bit operands (8 moduli; GPEMU_OZAKI=0 or n_pad outside that range: fp32 MFMA on
 * fp32 copies of L^-1 and K*); the mean and the q x q terms stay fp64. */
int gpe_posterior(gpe_ctx* ctx, int64_t m, const double* Xs, const double* Hs,
                  const double* beta, double sigma, int32_t full_var, int32_t precision,
                  double* mean_out, double* var_out);

/* ---- Sensitivity / UQ building blocks, resident factor --------
 * Replace the O(n^2) parts of sensitivity/_sensitivityclasses.py (case2): the
 * solves with emul.training.A (:40-44, :187-189, :436-441, :451-454) and the n x n
 * pair matrices Rtt (:90-102) and Pw (:599-626), which are never formed here.
 * Host arrays are row-major; x below is the resident raw training inputs (n x d). */

/* X = A^-1 B  (B, X: n x ncols). */
int gpe_solve(gpe_ctx* ctx, int32_t ncols, const double* B, double* X);

/* J Gaussian pair kernels K_j(k,l) = u[j,k] u[j,l] exp(-sum_i w[j,i] (x_ki - x_li)^2)
 * (w: J x d, u: J x n).  trace_out[j] = sum_kl (A^-1)_kl K_j(k,l) = tr(A^-1 K_j);
 * quad_out[j] = Z^T K_j Z (p x p; Z: n x p).  Any p (Z columns in chunks of 32, one
 * launch each) and any d the context holds (d > 32: coordinates staged through LDS in
 * chunks of 32 dimensions), as the reference's Pw / Rtt loops (:90-102, :599-626). */
int gpe_sense_pairs(gpe_ctx* ctx, int32_t J, const double* w, const double* u, int32_t p,
                    const double* Z, double* trace_out, double* quad_out);

/* out[t] = sum_k a[k] exp(-sum_s c[s] (Y[t,s] - x[k, dims[s]])^2), t < m, ns <= 4
 * (Y: m x ns): the Tw . e sums of main effects (:277-285, ns = 1) and interaction
 * effects (:353-373, ns = 2).  Needs set_data only. */
int gpe_gauss_transform(gpe_ctx* ctx, int64_t m, int32_t ns, const int32_t* dims,
                        const double* c, const double* Y, const double* a, double* out);

/* K.var(X, predict) materialised (m x m, symmetric): _emulatorkernels.py:39-50 /
 * :112-123, plus make_A's r/s2 diagonal (r_scale * r, r may be NULL). */
int gpe_kernel_var(gpe_ctx* ctx, int32_t kernel, const double* delta, int32_t d,
                   double nu, int32_t predict, int64_t m, const double* X,
                   const double* r, double r_scale, double* A_out);

/* The reference's dense derivative matrices, m x m row-major, zero diagonal:
 *   G(k,l) = pre * ((col_k - col_l) * col_scale)^2 * exp(-sum_i ((X_ki - X_li)/delta_i)^2)
 * (col NULL: the squared factor is 1).  kernel.grad_delta_A(X[:,i], i, s2)
 * (_emulatorkernels.py:53-63, alt :126-136): col = X[:,i], col_scale = 1/delta_i,
 * pre = s2 (1 - nu) (alt: s2), delta / X those of the preceding var() (its exp_save).
 * kernel.grad_nugget_A (std :66-71): col NULL, pre = -nu s2 / 2.  (The alt-nugget
 * form, s2 nu^2 I, is diagonal and built by the host.) */
int gpe_kernel_grad(gpe_ctx* ctx, const double* delta, int32_t d, int64_t m, const double* X,
                    const double* col, double col_scale, double pre, double* G_out);

/* The oLHC generator's selection statistic (design_inputs.py:54-64): for each of the N
 * candidate designs (designs: N x n x dim row-major, design k at k*n*dim),
 * idx_out[k] = np.argmin(scipy pdist(xt, 'sqeuclidean')) with xt = [design k; fextra]
 * (fextra: ne x dim row-major, ne may be 0 / NULL): the condensed index of the closest
 * pair, first occurrence on ties, NaN distances count as the minimum.  Distances are
 * summed over dimensions in order without FMA, bit-identical to pdist's.  The caller
 * keeps the reference's rule (largest index wins, :62-67).  n + ne >= 2. */
int gpe_lhc_maximin(gpe_ctx* ctx, int32_t N, int64_t n, int32_t dim, const double* designs,
                    int64_t ne, const double* fextra, int64_t* idx_out);

/* K.covar(XT, XV) -> n x m row-major: _emulatorkernels.py:75-79 / :148-152. */
int gpe_kernel_covar(gpe_ctx* ctx, int32_t kernel, const double* delta, int32_t d,
                     double nu, int64_t n, const double* XT, int64_t m,
                     const double* XV, double* C_out);

/* Cholesky factor, inverse factor and inverse of an arbitrary SPD matrix
 * (row-major m x m, lower triangle read).  Replaces the np.linalg.cholesky of the
 * posterior covariance in posterior_sample (emulatorfunctions.py:283) and serves
 * as the unit-test entry of the blocked factorisation.  Any output may be NULL.
 * L_out / Linv_out are lower-triangular with zero upper part. */
int gpe_cholesky(gpe_ctx* ctx, int64_t m, const double* A, double* L_out,
                 double* Linv_out, double* Ainv_out, double* logdet_out);

/* Test hook for the grouped MFMA GEMM building block on one problem:
 * C = alpha * opA x opB + beta * C with opA M x K, opB K x N (row-major host
 * arrays A (M x K), B (K x N), C (M x N)); trans_a / trans_b choose the device
 * storage orientation exercised (0: M-/N-contiguous, 1: K-contiguous).
 * M, N multiples of 128, K multiple of 16. */
int gpe_test_gemm(gpe_ctx* ctx, int32_t trans_a, int32_t trans_b, int64_t M, int64_t N,
                  int64_t K, const double* A, const double* B, double* C,
                  double alpha, double beta);

/* Benchmark hook: time `reps` launches of the grouped GEMM on device-resident
 * random operands: C (mt*128 x nt*128, lower tiles only if lower) += -A B^T-style
 * update with K, in storage orientation (trans_a, trans_b).  Returns average
 * ms per launch in *ms_out.  Uses its own device buffers. */
int gpe_bench_gemm(gpe_ctx* ctx, int32_t trans_a, int32_t trans_b, int32_t mt, int32_t nt,
                   int32_t K, int32_t lower, double beta, int32_t reps, double* ms_out);

/* noise_fit's noise-estimation step (noise_fit/noise_fit.py:130-139, :142-150):
 * the posterior at Xs (m x d, Hs m x q; full m x m covariance V, built on the
 * device with Dnew's own r/s2 diagonal: r_new (m, or NULL) times r_scale, as in
 * Dnew.make_A(s2) after Dnew.set_r, _emulatorclasses.py:572-575), L = chol(V),
 * and for the s draws u_j = U[j, :] (U row-major s x m: the reference's successive
 * np.random.randn(m) calls) z_out[i] = sum_j 0.5 (t_i - mean_i - (L u_j)_i)^2
 * (the caller divides by s and applies the log transform).  mean_out (m) is the
 * posterior mean.  Needs the resident factor of gpe_factor.  Any m up to 2^20 (the
 * reference has no bound): m <= 16384 forms V in one chunk, beyond it V is formed
 * chunk pair by chunk pair straight into the factorisation workspace (V and its
 * factor take 2 x m_pad^2 x 8 bytes of HBM: 2 x 8.6 GB at m = 32768).
 * GPE_NOT_PD when V is not positive definite (np.linalg.cholesky's LinAlgError). */
int gpe_noise_sample(gpe_ctx* ctx, int64_t m, const double* Xs, const double* Hs,
                     const double* beta, double sigma, const double* r_new, double r_scale,
                     const double* t, int32_t s, const double* U, double* mean_out,
                     double* z_out);

/* Per-phase device time of the most recent gpe_objective call, in ms:
 * [0] K-build, [1] Cholesky, [2] triangular inverse, [3] A^-1 (L^-T L^-1),
 * [4] skinny solves / small algebra, [5] gradient contraction, [6] total.
 * Only filled when profiling is on. */
int gpe_set_profiling(gpe_ctx* ctx, int32_t on);
int gpe_phase_times(gpe_ctx* ctx, double* ms_out, int32_t n);

/* Aggregate device time (ms) and call count of the MFMA GEMM launches of the most
 * recent objective (profiling on), and their algorithmic flop count. */
int gpe_gemm_stats(gpe_ctx* ctx, double* ms_out, double* launches_out,
                   double* flops_out);

/* The same for the int8 products of the objective's A^-1 and of the top TRTRI level
 * (gpemu_ozaki.hpp: the fp64 products emulated exactly on the i8 MFMA, N moduli): their
 * device time (ms), launch count, int8 multiply-add ops (2 per multiply-add, every modulus)
 * and the fp64 flops of the products they replace.  Internal instrumentation for bench.py;
 * the reference has no counterpart. */
int gpe_ozaki_stats(gpe_ctx* ctx, double* ms_out, double* launches_out, double* int8_ops_out,
                    double* fp64_flops_out);

#ifdef __cplusplus
}
#endif

#endif /* GPEMU_H */
