/*
 * gpemu_dist.h -- C-ABI of the row-block distributed objective in libgpemu.so
 * (BASELINE configs[3]: n = 65536, d = 20 on 8 x MI355X).
 *
 * Replaces, for one evaluation spread over P GPUs, Optimize.loglikelihood_gp4ml /
 * _mucm and their gradients (_emulatoroptimise.py:412-493, :305-378, the same
 * functions gpe_objective replaces on one GPU): K-build + blocked right-looking
 * Cholesky + log|A| + L^-1 [f H], and for the gradient L^-1, A^-1 and the
 * contraction <M, dA/dtheta>.  The n x n covariance is partitioned by 128-row
 * tile rows, dealt cyclically (tile row i on rank i mod P); each rank stores only
 * its tile rows of the lower triangle.  Per column step the owner factors the
 * diagonal tile in-kernel, RCCL broadcasts its inverse (128 KB), every rank forms
 * its panel tiles, RCCL all-gathers the panel column, and every rank applies the
 * trailing update to its own rows.  [f H] is carried as ceil((q+1)/128) extra tile
 * rows under the matrix (dealt like the others), so L^-1 [f H] and its Gram matrix
 * fall out of the same sweep.
 *
 * Gradient: X = L^-1 by the recursive TRTRI on the same partition: per level of
 * block pairs, RCCL all-gathers the rows of X11 and, after each rank's columns of
 * (L21 X11)^T, those columns; every rank then finishes its rows of X21 = -X22 L21 X11.
 * Each rank forms its partial X_r^T X_r of A^-1 slab by slab (so per-rank memory
 * stays O(n^2 / P)) and contracts it locally, so the only other collectives are an
 * all-reduce of the n x (q+1) matrix [sqrt(c) alpha, W] and of the d+3 contraction
 * sums.
 *
 * Processes: one per GPU.  Rank 0 calls gpe_dist_unique_id, the host shares the
 * 128 bytes (by default through the job's native file rendezvous,
 * gp_emu_uqsa_amd/rendezvous.py init_from_env(); a torch.distributed group is the
 * alternative, distributed.share_unique_id), every rank calls gpe_dist_create with it.  unique_id == NULL selects the in-process
 * loopback transport: all P logical ranks live in this process on one GPU, each
 * with its own buffers, running the same partition, schedule and device code
 * (pack, all-gather buffers, unpermute, all-reduced partials);
 * only the collective calls become device copies (used to test P = 2..8 on one
 * GPU).
 *
 * Same conventions and status codes as gpemu.h.
 */
#ifndef GPEMU_DIST_H
#define GPEMU_DIST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gpe_dist gpe_dist;

/* RCCL unique id for a new communicator (len >= 128); rank 0 only. */
int gpe_dist_unique_id(uint8_t* out, int32_t len);

/* device: GPU of this process; nranks: P; rank: this process's rank (ignored in
 * loopback); unique_id: 128 bytes from gpe_dist_unique_id, or NULL = loopback. */
gpe_dist* gpe_dist_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* unique_id);
void gpe_dist_destroy(gpe_dist* h);
const char* gpe_dist_last_error(gpe_dist* h);

/* Replicated inputs, as gpe_set_data (every rank passes the same arrays). */
int gpe_dist_set_data(gpe_dist* h, int64_t n, int32_t d, int32_t q, const double* X,
                      const double* f, const double* H, const double* r);

/* Objective (and gradient when want_grad != 0), arguments and outputs as
 * gpe_objective.  All ranks call it collectively and all receive the same llh,
 * gradient and sigma2.  The gradient buffers (this rank's rows of L^-1 and a slab
 * of its partial of A^-1: 512 MiB, or 1/P of the triangle's tile rows when that is
 * more and the triangle takes at most 2 GiB) are allocated on the first want_grad
 * call. */
int gpe_dist_objective(gpe_dist* h, int32_t variant, int32_t kernel, const double* hp,
                       int32_t n_hp, double nu_fixed, int32_t want_grad, double* llh_out,
                       double* grad_out, double* sigma2_out);

/* Partition map (pure functions, no GPU): owner rank of tile row t and the number
 * of tile rows rank `rank` stores for n points and q basis columns, including its
 * share of the ceil((q+1)/128) augmented [f H]^T tile rows. */
int32_t gpe_dist_owner(int32_t nranks, int32_t tile_row);
int32_t gpe_dist_local_rows(int64_t n, int32_t q, int32_t nranks, int32_t rank);

/* Time of the last gpe_dist_objective: total and the part spent in collectives
 * (RCCL or loopback copies), ms, measured with HIP events on this rank. */
int gpe_dist_times(gpe_dist* h, double* total_ms, double* comm_ms);

/* Device bytes held for rank `rank` (this process's rank over RCCL, any logical
 * rank in loopback): its own buffers plus the replicated inputs and schedules. */
int gpe_dist_rank_bytes(gpe_dist* h, int32_t rank, int64_t* bytes_out);

#ifdef __cplusplus
}
#endif

#endif /* GPEMU_DIST_H */
