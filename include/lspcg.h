/*
 * lspcg.h -- C ABI of the MI355X-native PCG hot path (liblspcg_hip.so, gfx950).
 *
 * This is the drop-in boundary for the reference's native solver and GNN kernels.
 * Every entry point names the reference interface it replaces:
 *
 *   pymathprim.linalg.PreconditionedConjugateGradient(A, device, preconditioner, dtype)
 *       (unvendored; call sites neural_cg/utils/validate.py:73,79-80,110,116-117,145,151-156)
 *       -> lspcg_solver_create / lspcg_solver_set_spai / lspcg_solver_solve
 *   scipy csr_matvec inside the PCG (validate.py:102, 182)      -> lspcg_spmv
 *   neural_cg/utils/validate.py:22-51 to_csr_cpu
 *       + neural_cg/data.py:134-170 (make_bsr_from_coo_inds, apply_dbc_masking)
 *                                                                -> lspcg_assemble
 *   csr_matrix(spai.T) (validate.py:176)                         -> lspcg_mat_transpose
 *   A.diagonal() (validate.py:243, 280)                          -> lspcg_mat_diagonal
 *   csr @ diags(rsqrt_diag) (scaled_workspace.py:210-211)        -> lspcg_mat_scale_columns
 *   neural_cg/nn/gnns.py:77-97 NodeEdgeProcessing.forward
 *       (+ basic_layers.py:73-109 FeedForward, :145-225 MPLayer) -> lspcg_gnn_forward
 *   neural_cg/nn/basic_layers.py:112-142 GraphSpmv.forward        -> lspcg_graph_spmv
 *   neural_cg/nn/basic_layers.py:228-261 AATPE.forward            -> lspcg_graph_aatpe
 *       (edge lists prepared once by lspcg_graph_create)
 *
 * Conventions: plain pointers and sizes only.  Vector arguments of compute calls are
 * DEVICE pointers; matrix/weight uploads accept host or device pointers.  All work is
 * issued on the context's stream.  Every call returns LSPCG_OK (0), LSPCG_NOT_CONVERGED
 * (1, solve only) or a negative error code; lspcg_last_error() describes the last error
 * of the calling thread.
 */
#ifndef LSPCG_H_
#define LSPCG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSPCG_OK 0
#define LSPCG_NOT_CONVERGED 1
#define LSPCG_ERR_ARG (-1)
#define LSPCG_ERR_HIP (-2)
#define LSPCG_ERR_UNSUPPORTED (-3)
#define LSPCG_ERR_FORMAT (-4)
#define LSPCG_ERR_BREAKDOWN (-5) /* incomplete factorization hit a non-positive pivot */
#define LSPCG_ERR_SINGULAR (-6)  /* a given triangular factor has a zero diagonal entry */

#define LSPCG_F32 0
#define LSPCG_F64 1

/* preconditioner kinds (pymathprim names: none / diagonal / ext_spai / ext_spai_scaled) */
#define LSPCG_PRECOND_NONE 0
#define LSPCG_PRECOND_DIAGONAL 1
#define LSPCG_PRECOND_EXT_SPAI 2
#define LSPCG_PRECOND_EXT_SPAI_SCALED 3
/* IC(0) of A, applied by two sync-free triangular solves (pymathprim "ic") */
#define LSPCG_PRECOND_IC 4

/* dot-product summation order of the PCG loop (lspcg_solver_set_dot_order) */
#define LSPCG_DOT_COMPENSATED 0 /* default: compensated (Dot2) dots in a fixed tree, ~correctly rounded */
#define LSPCG_DOT_OPENBLAS 1    /* parity mode: numpy's ddot as recorded (OpenBLAS 0.3.29 SkylakeX) */

typedef struct lspcg_ctx lspcg_ctx;
typedef struct lspcg_mat lspcg_mat;
typedef struct lspcg_solver lspcg_solver;
typedef struct lspcg_gnn lspcg_gnn;
typedef struct lspcg_graph lspcg_graph;

const char* lspcg_last_error(void);
int lspcg_version(void);
/* provenance: hash of the sources, headers, compiler flags and arch this library was built from
 * (learningsparsepreconditioner4gpu_amd/_build.py tree_hash) */
const char* lspcg_build_id(void);

/* ---- context: one per GPU per host thread; stream NULL = the default (null) stream ---- */
int lspcg_ctx_create(int device, void* stream, lspcg_ctx** out);
int lspcg_ctx_destroy(lspcg_ctx* ctx);
int lspcg_ctx_synchronize(lspcg_ctx* ctx);

/* ---- sparse matrices (device copies owned by the handle) ---- */
/* scalar CSR, n x n, int32 indptr[n+1] / indices[nnz], vals[nnz] of dtype */
int lspcg_mat_create_csr(lspcg_ctx* ctx, int64_t n, int64_t nnz, const int32_t* indptr,
                         const int32_t* indices, const void* vals, int dtype, lspcg_mat** out);
/* block CSR, nb x nb blocks of bs x bs (bs in {1,3}), vals[nnzb][bs][bs] row-major */
int lspcg_mat_create_bsr(lspcg_ctx* ctx, int64_t nb, int64_t nnzb, int bs, const int32_t* indptr,
                         const int32_t* indices, const void* vals, int dtype, lspcg_mat** out);
int lspcg_mat_destroy(lspcg_mat* A);
/* n = scalar rows, nnzb = stored blocks (= scalar nnz when bs == 1) */
int lspcg_mat_info(const lspcg_mat* A, int64_t* n, int64_t* nnzb, int* bs, int* dtype);
/* copy the handle's arrays out (host or device destinations; NULL skips an array) */
int lspcg_mat_copy_out(const lspcg_mat* A, int32_t* indptr, int32_t* indices, void* vals);
/* explicit transpose (sorted), replaces csr_matrix(spai.T) of validate.py:176 */
int lspcg_mat_transpose(const lspcg_mat* A, lspcg_mat** out);
/* d[i] = A[i,i] (0 where absent), device pointer of the matrix dtype, length n */
int lspcg_mat_diagonal(const lspcg_mat* A, void* d);
/* A <- A diag(d): column scaling, d device pointer of the matrix dtype, length n */
int lspcg_mat_scale_columns(lspcg_mat* A, const void* d);
/* The solver's reordering analysis on its own (DESIGN.md §2 "Reordering"): perm (device int32,
 * one entry per block row) <- the reverse Cuthill-McKee order of A's block graph, new row i' = old row
 * perm[i'] (isolated rows -- empty or diagonal-only -- last, each component from a pseudo-peripheral
 * node, children by (row length, index)); *applied = 0 and perm untouched when the graph is left in
 * its order (more than 256 non-trivial components, a row longer than 1024 blocks, or a row whose
 * columns are not strictly increasing).  Mean |col -
 * row| before / after (either pointer may be NULL). */
int lspcg_mat_rcm(const lspcg_mat* A, int32_t* perm, int* applied, double* mean_offset_before,
                  double* mean_offset_after);

/* ---- kernels ---- */
/* y = A x (scipy csr_matvec bit pattern: per-row sequential sum in index order).  x and y must not
 * overlap.  After a reordering lspcg_mat_prepare_spmv (lspcg_mat_spmv_reorder_info) the call gathers x
 * into a scratch vector owned by A, so calls on one matrix must run on one stream at a time. */
int lspcg_spmv(lspcg_ctx* ctx, const lspcg_mat* A, const void* x, void* y);
/* analysis step (cf. rocSPARSE csrmv_analysis): attach a SELL-64 copy of a scalar CSR matrix, or
 * the BSELL-64 block copy of a BSR 3x3 (one column per block, block values in 16-B lane chunks), with the
 * same values and dtype and 16-bit column offsets where they fit, that lspcg_spmv then uses -- the
 * results keep the same bits.  *kind (nullable) = the column storage: 1 (SELL-DIA: a sorted scalar
 * CSR whose 64-row slices have <= 16 distinct row-relative offsets col - row, one value slot per
 * offset and a row mask, no column array), 16 (16-bit offsets from the slice's first row), 17
 * (SELL-64J: lanes sorted by row length, each 4-entry group stored for its active lanes only), 18
 * (SELL-64X: SELL-64J reading x from an LDS copy of each 256-row tile's blocks), 32 (int32
 * columns), or 0 when the matrix stays on the CSR / BSR kernel (irregular row lengths).  A numbering
 * far from banded (the solver's rule: mean |col - row| > 4 n^(2/3), n >= 16384, env LSPCG_REORDER) is
 * analysed on P A P^T, P the device reverse Cuthill-McKee permutation, every row's entries in their
 * original order; lspcg_spmv then gathers x into that numbering and scatters y back (same bits).
 * lspcg_mat_scale_columns drops it. */
int lspcg_mat_prepare_spmv(lspcg_mat* A, int* kind);
/* the analysis step's reordering (lspcg_mat_prepare_spmv): *applied = 1 when the SpMV runs on
 * P A P^T; mean |col - row| before / after (either pointer may be NULL).  Replaces nothing in the
 * reference (its SpMV is scipy's, on the caller's numbering). */
int lspcg_mat_spmv_reorder_info(const lspcg_mat* A, int* applied, double* mean_offset_before,
                                double* mean_offset_after);
/* average device ms of one SpMV launch, HIP events on the ctx stream.  flush_bytes == 0:
 * reps back-to-back launches (warm caches); > 0: before every launch a read of a flush_bytes
 * buffer evicts the 256 MiB Infinity Cache (cold); the launch time is (reps x (flush + SpMV)
 * - reps x flush) / reps, i.e. the in-stream duration without per-event overhead. */
int lspcg_spmv_timed(lspcg_ctx* ctx, const lspcg_mat* A, const void* x, void* y, int reps,
                     int64_t flush_bytes, double* avg_ms);
/* diagnostics: time SpMV launch configuration `variant` (fp64 scalar CSR; see csrc/lspcg_core.hip
 * kSpmvVariants) exactly like lspcg_spmv_timed; variant < 0 returns the number of variants */
int lspcg_spmv_variant_timed(lspcg_ctx* ctx, const lspcg_mat* A, int variant, const void* x, void* y,
                             int reps, int64_t flush_bytes, double* avg_ms);
/* diagnostics: the same timing for the SELL-64 kernel the PCG loop uses (csrc/lspcg_sell.hpp) on a
 * SELL copy of A built inside the call (fp64 scalar CSR).  flags bit 0: store the values as fp32
 * (lossless only when every value is fp32-representable); bit 1: 16-bit column offsets where they
 * fit; bit 3: SELL-DIA where it fits (tried before bit 1); bit 2 (experiment): gather x from an
 * interleaved (x, x) pair array with one 16-B load per entry, the cost model of a fused update
 * evaluated in the gather.  y = A x, same bits as lspcg_spmv */
int lspcg_spmv_sell_timed(lspcg_ctx* ctx, const lspcg_mat* A, int flags, const void* x, void* y,
                          int reps, int64_t flush_bytes, double* avg_ms);
/* calibration: the same cold / warm timing for a plain streaming read of `bytes` (16-B loads, 8
 * workgroups per CU): the achievable bandwidth an SpMV of that many bytes is compared against */
int lspcg_read_timed(lspcg_ctx* ctx, int64_t bytes, int reps, int64_t flush_bytes, double* avg_ms);
/* ---- baseline preconditioners (pymathprim "ic" / "ainv", infer.py:310-321; algorithms and
 * operation order: oracle/precond.py; scalar CSR, sorted rows, stored diagonal) ---- */
/* IC(0): *L = lower-triangular factor with the pattern of tril(A), A ~ L L^T */
int lspcg_ic0(const lspcg_mat* A, lspcg_mat** L, double* t_ms);
/* AINV(0): *L = Z D^{-1/2} (Z unit upper, pattern triu(A)) so that L L^T = Z D^{-1} Z^T ~ A^{-1};
 * use it as an ext_spai factor with epsilon = 0 */
int lspcg_ainv0(const lspcg_mat* A, lspcg_mat** L, double* t_ms);
/* x = T^{-1} b, T triangular (lower != 0: diagonal stored last in each row; else first), in the
 * arithmetic of scipy's spsolve_triangular on csc(T) -- the reference's IC apply
 * (validate.py:359-365): column-scaled unit solve, updates in SuperLU's column order, diagonal
 * scaling after; one sync-free launch over the level-ordered rows; b, x device vectors of T's
 * dtype */
int lspcg_trsv(const lspcg_mat* T, int lower, const void* b, void* x);
/* compensated, deterministic dot product of two device vectors; result to host */
int lspcg_dot(lspcg_ctx* ctx, int64_t n, int dtype, const void* x, const void* y, double* out);

/* ---- PCG solver (pymathprim.linalg.PreconditionedConjugateGradient) ---- */
int lspcg_solver_create(lspcg_ctx* ctx, const lspcg_mat* A, int precond, lspcg_solver** out);
/* ext_spai=(L, eps): builds Lᵀ (and diag(A) for the scaled variant) on device.
 * t_prec_ms (nullable) receives the device time of that setup. L must outlive solves. */
int lspcg_solver_set_spai(lspcg_solver* s, const lspcg_mat* L, double epsilon, double* t_prec_ms);
/* LSPCG_PRECOND_IC solvers: IC(0) factorization of A on the device (pymathprim "ic" setup;
 * the reference's scipy twin is validate.py:344-429); t_prec_ms = setup time */
int lspcg_solver_set_ic(lspcg_solver* s, double* t_prec_ms);
/* LSPCG_PRECOND_IC solvers: install a given lower-triangular factor L (scalar CSR of the solver's
 * size and dtype, sorted rows, diagonal stored last) and apply M^-1 = L^-T L^-1 -- the
 * reference's IncompleteCholeskyPreconditioner(L) of get_pcg_iter_time_scipy_ichol
 * (validate.py:344-419, which takes an external L).  L is copied. */
int lspcg_solver_set_ic_factor(lspcg_solver* s, const lspcg_mat* L, double* t_prec_ms);
/* Solve A x = b from x (x0, in/out).  Semantics of scipy.sparse.linalg.cg (iterative.py
 * 359-418): atol = rtol*||b||, ||r|| checked at the top of each iteration, iters = number
 * of completed iterations, max_iter <= 0 means n.  res_hist (host, nullable, length
 * max_iter+2) receives ||r_k|| for k = 0..iters.  t_solve_ms = device time of the solve.
 * Returns LSPCG_OK when converged, LSPCG_NOT_CONVERGED when max_iter was reached.
 * Scalar systems with n <= LSPCG_SMALL_N (env read at solver creation; default 3072, 0 = off;
 * at most 3 rows per thread of 1024 and 3 vectors in 60 KiB of LDS: 2560 in fp64; IC excluded)
 * run the whole loop in one single-workgroup launch -- same bits as the multi-kernel schedule. */
int lspcg_solver_solve(lspcg_solver* s, const void* b, void* x, double rtol, int64_t max_iter,
                       int64_t* iters, double* res_hist, double* t_solve_ms);
/* Measurement only (bench.py): `iters` iterations of the split ext_spai schedule from x0 = 0,
 * each of the five launches bracketed by HIP events on the solver stream (no graph, no
 * convergence stop); kernel_ms[0..4] = mean device time of KA (t = Lᵀr), KB (z = Lt + εr, ρ),
 * UP (p, x), KC (q = Ap, π), UR (r); *nk = 5.  LSPCG_ERR_UNSUPPORTED for other schedules. */
int lspcg_solver_time_kernels(lspcg_solver* s, const void* b, int64_t iters, double* kernel_ms, int* nk);
/* Summation order of every dot / norm of the loop (scipy cg's np.dot / np.linalg.norm,
 * iterative.py:398-418).  LSPCG_DOT_COMPENSATED (default): split / one-workgroup schedules,
 * ~correctly rounded.  LSPCG_DOT_OPENBLAS: parity mode, fp64 only -- each dot is recomputed in
 * the order of numpy's cblas_ddot in the container that recorded the reference's trajectories
 * (OpenBLAS 0.3.29 SkylakeX kernel, split over `threads` (1..16) OpenBLAS threads when n > 10000;
 * restated in oracle/openblas_ddot.c) by one extra single-workgroup launch after each reducing
 * launch, on the last-arriver multi-kernel schedule: the solve then reproduces the reference's
 * recorded count, ||r_k|| history and x bit for bit.  Measurement: DESIGN.md §3. */
int lspcg_solver_set_dot_order(lspcg_solver* s, int order, int threads);
/* Bandwidth-reducing analysis step (no reference counterpart; cf. scipy's reverse_cuthill_mckee
 * before a solve): a solver whose A is numbered far from banded (mean |col - row| > 4 n^(2/3),
 * n above the one-workgroup bound) runs the loop on P A Pᵀ, P Lᵀ Pᵀ, P L Pᵀ with P a reverse
 * Cuthill-McKee permutation, every row's entries kept in their original order -- the same row
 * sums bit for bit -- with b / x permuted on the device around the loop.  Environment
 * LSPCG_REORDER = 0 (never) / 1 (always) / auto.  Not for IC, batches or the OpenBLAS dot order
 * (which switches a reordered solver back).  *applied = 1 if the solver runs permuted;
 * mean |col - row| before / after (either pointer may be NULL). */
/* The iteration views the solver built for A (0), L (1), Lᵀ (2): col_kind[w] = 0 (staged CSR kernel),
 * 1 (SELL-DIA: no column array), 16 / 32 (SELL-64 with 16-bit / int32 columns), 8 (SELL-64C: one-byte
 * codes into per-slice dictionaries of <= 64 row-relative offsets, 16-bit columns for slices with
 * more; unstructured orderings, LSPCG_SELLC=0 turns it off), 17 (SELL-64J: unstructured meshes, each
 * slice's rows sorted by length, no padded slots), 18 (SELL-64X: SELL-64J reading x through the row
 * tile's LDS-staged blocks); value_bytes[w] = 8 (fp64), 4 (fp64 matrix stored exactly as fp32),
 * 0 (no view).  Same bits in every case. */
int lspcg_solver_views(const lspcg_solver* s, int* col_kind, int* value_bytes);
int lspcg_solver_reorder_info(const lspcg_solver* s, int* applied, double* mean_offset_before,
                              double* mean_offset_after);
int lspcg_solver_destroy(lspcg_solver* s);

/* ---- batched lockstep ext_spai PCG over independent systems (infer.py:278-331 solves its samples
 * one after another, each a get_pcg_iter_time call, validate.py:89-121; this solves a window of
 * them with every launch covering all systems -- DESIGN.md §6).  Each system keeps scipy cg's
 * recurrence, its own scalars, top-of-loop test and iteration count: the result per system is
 * what lspcg_solver_solve returns for it alone (count and history equal; iterate within the
 * compensated dots' rounding, same bits in practice).  A[k], L[k]: nsys >= 1 matrices of one
 * dtype and block size (L[k] the ext_spai factor of A[k]); the handles must outlive the batch
 * only until lspcg_batch_create returns (their entries are copied into a block-diagonal system
 * whose per-system row ranges are padded to whole 256-row workgroup tiles).
 * Windows whose systems all fit the one-workgroup solve (n <= 2560 in fp64) run it with one
 * workgroup per system in one launch; others run the five phases in lockstep.
 * LSPCG_ERR_UNSUPPORTED when a SELL view cannot be built (irregular rows): solve one by one. */
typedef struct lspcg_batch lspcg_batch;
int lspcg_batch_create(lspcg_ctx* ctx, int nsys, const lspcg_mat* const* A, const lspcg_mat* const* L,
                       double epsilon, lspcg_batch** out);
/* b[k], x[k]: device vectors of system k (x in: x0, out: solution).  max_iter <= 0: each
 * system's own n.  iters[k], status[k] (LSPCG_OK converged / LSPCG_NOT_CONVERGED) per system;
 * res_hist (nullable): per-system host arrays of length max_iter_k + 2 (or NULL entries);
 * t_solve_ms = device time of the whole batch.  Returns LSPCG_OK when every system converged. */
int lspcg_batch_solve(lspcg_batch* bt, const void* const* b, void* const* x, double rtol, int64_t max_iter,
                      int64_t* iters, int32_t* status, double* const* res_hist, double* t_solve_ms);
int lspcg_batch_destroy(lspcg_batch* bt);

/* ---- CSR assembly with Dirichlet masking (to_csr_cpu on device) ----
 * edge_index: device int64 [2,E] (row-major sorted, duplicate free -- checked);
 * blocks: device [E,bs,bs] of in_dtype; mask: device [nb*bs] of mask_dtype or NULL.
 * out_block = 0: scalar CSR exactly as to_csr_cpu (zeros dropped, sorted);
 * out_block = 1: BSR (bs x bs blocks, masking applied, zeros kept) for the block kernels. */
int lspcg_assemble(lspcg_ctx* ctx, int64_t nb, int64_t E, int bs, const int64_t* edge_index,
                   const void* blocks, int in_dtype, const void* mask, int mask_dtype,
                   int out_dtype, int out_block, lspcg_mat** out);

/* ---- GNN (NodeEdgeProcessing, F = hidden = 16, FeedForward num_layers = 2) ---- */
typedef struct lspcg_gnn_desc {
  int node_in;        /* node input features (x.shape[1]) */
  int edge_in;        /* edge input features (edge_attr.shape[1]) */
  int hidden;         /* node_features = edge_features = MLP hidden channels (16) */
  int mlp_layers;     /* FeedForward num_layers (2 -> three Linear layers) */
  int num_mp_layers;  /* MPLayer count (4) */
  int edge_out;       /* block_size * block_size */
  int node_residual;  /* gnn.yaml node_residual */
  int edge_residual;  /* gnn.yaml edge_residual */
} lspcg_gnn_desc;

/* weights: packed fp32 blob in the order documented in learningsparsepreconditioner4gpu_amd/nn.py
 * (pack_weights); host or device pointer.  The MLP products run as fp32-accurate split-f16 GEMMs
 * (raw edge features of any magnitude are scaled per edge inside); weights whose LayerNorm-fed MLPs
 * bound their hidden activations at 2^15 or more -- past f16's range -- select the fp32-MFMA
 * kernels instead (environment LSPCG_GNN_F32=1 forces them).  Any weights run. */
int lspcg_gnn_create(lspcg_ctx* ctx, const lspcg_gnn_desc* desc, const float* weights,
                     int64_t nweights, lspcg_gnn** out);
/* Structure analysis of a graph (its CSC by destination), like a sparse library's analysis step:
 * lspcg_gnn_forward reuses it while it is called with the same (edge_index pointer, N, E) -- the
 * reference runs `repeat` forwards of one sample (infer.py:290-293) -- and rebuilds it for any
 * other graph.  Call it again after changing edge_index's contents in place. */
int lspcg_gnn_set_graph(lspcg_gnn* g, int64_t N, int64_t E, const int64_t* edge_index);
/* x [N,node_in], edge_index device int64 [2,E], edge_attr [E,edge_in] -> out [E,edge_out]
 * (all fp32 device).  Message aggregation order is deterministic. */
int lspcg_gnn_forward(lspcg_gnn* g, int64_t N, int64_t E, const float* x, const int64_t* edge_index,
                      const float* edge_attr, float* out);
/* Which kernels lspcg_gnn_create chose: *f32 = 1 for the fp32-MFMA ones, 0 for the split-f16 GEMMs;
 * *hidden_bound (may be NULL) = the weights' hidden-activation bound that decided it (2^15). */
int lspcg_gnn_precision(const lspcg_gnn* g, int* f32, double* hidden_bound);
int lspcg_gnn_destroy(lspcg_gnn* g);

/* ---- block SpMV over an edge list (GraphSpmv / AATPE, basic_layers.py:112-142, 228-261) ----
 * edge_index: device int64 [2,E], any order, duplicates summed (PyG scatter-add semantics);
 * N nodes of bs (1 or 3) components.  Values [E,bs,bs], x / y / mask / diag [N*bs], all of
 * `dtype`, device pointers; mask and diag nullable. */
int lspcg_graph_create(lspcg_ctx* ctx, int64_t N, int64_t E, int bs, const int64_t* edge_index, lspcg_graph** out);
int lspcg_graph_destroy(lspcg_graph* g);
/* GraphSpmv(use_transpose).forward: y = A x (transpose = 0: block (ei[0], ei[1]) multiplies
 * x[ei[1]], summed at ei[0]) or y = Aᵀ x (transpose = 1), then y *= mask */
int lspcg_graph_spmv(lspcg_graph* g, const void* vals, int dtype, int transpose, const void* x, const void* mask,
                     void* y);
/* AATPE(epsilon).forward: t = (mask ⊙ Aᵀx) ⊙ diag ; y = mask ⊙ (A t) + (ε x) ⊙ diag
 * (t: caller-provided [N*bs] scratch that receives AᵀX, the reference's AT_x) */
int lspcg_graph_aatpe(lspcg_graph* g, const void* vals, int dtype, double epsilon, const void* x, const void* mask,
                      const void* diag, void* t, void* y);

/* ---- one system row-partitioned over ranks (NOT in the reference,
 * whose systems each fit one process -- it replaces no reference interface).  The host driver
 * (learningsparsepreconditioner4gpu_amd/dist_pcg.py) owns the halo all-to-alls, the all-gathers
 * of dot partials (torch.distributed: RCCL over xGMI) and scipy cg's scalar recurrence
 * (iterative.py:359-418, as restated at validate.py:163-201); these calls enqueue the rank-local
 * device phases on the context's stream.  A, L, LT: the rank's rows of the global matrices as
 * square n_ext x n_ext scalar CSR over its extended vector [n_own own rows | halo] (rows >= n_own
 * empty; L and LT may both be NULL for plain CG).  send_idx (host or device, n_send entries):
 * own-row indices packed for the other ranks, grouped by destination.  red: a device buffer of
 * 64 x 2 x 2 doubles receiving per-group compensated (sum, correction) pairs of the launch's dots
 * (zeroed by the call; the host sums every rank's groups). */
typedef struct lspcg_part lspcg_part;
int lspcg_part_create(lspcg_ctx* ctx, const lspcg_mat* A, const lspcg_mat* L, const lspcg_mat* LT, int64_t n_own,
                      const int32_t* send_idx, int64_t n_send, lspcg_part** out);
int lspcg_part_destroy(lspcg_part* p);
/* sendbuf[k] = v[send_idx[k]] */
int lspcg_part_pack(lspcg_part* p, const void* v, void* sendbuf);
/* red <- groups of a·a, b·b over the own rows */
int lspcg_part_norms(lspcg_part* p, const void* a, const void* b, double* red);
/* t[i] = (LT r)_i, i < n_own */
int lspcg_part_lt(lspcg_part* p, const void* r_ext, void* t_ext);
/* z = L t + eps r ; red <- groups of r·z, r·r */
int lspcg_part_l(lspcg_part* p, const void* t_ext, const void* r, double eps, void* z, double* red);
/* q = A p ; red <- groups of p·q */
int lspcg_part_a(lspcg_part* p, const void* p_ext, void* q, double* red);
/* p = z (first != 0) or p*beta + z */
int lspcg_part_update_p(lspcg_part* p, const void* z, void* p_ext, double beta, int first);
/* x += alpha p ; r -= alpha q */
int lspcg_part_update_xr(lspcg_part* p, double alpha, const void* p_ext, const void* q, void* x, void* r_ext);
/* Device-side scalar recurrence (no host round trip per iteration; dist_pcg.DistributedPCG):
 * the part's device state holds scipy cg's scalars (rtol, atol, ‖r‖², ρ, ρ_prev, π, α, β, the
 * iteration count and a done code: 1 converged, 2 max_iter, 3 non-finite, 4 ‖b‖ = 0).
 * state_init: reset it (hist: device buffer of max_iter + 2 doubles receiving ‖r_k‖, or NULL).
 * scalars: one single-thread launch summing the all-gathered [world][64][nd][2] group pairs
 * rank-major and applying phase 0 init (nd 2: ‖r_0‖², ‖b‖²), 1 after part_l (nd 2: ρ, ‖r_k‖²;
 * then the top-of-loop test and β), 2 the same for plain CG (no gathered data), 3 after part_a
 * (nd 1: π; α), 4 plain CG after part_norms of r (nd 2: ‖r_{k+1}‖²).  update_p_dev /
 * update_xr_dev: update_p / update_xr with β, α from the state, skipped once done (update_xr_dev
 * also advances the iteration).  status: the iteration count and done code (synchronises). */
int lspcg_part_state_init(lspcg_part* p, double rtol, int64_t max_iter, double* hist);
int lspcg_part_scalars(lspcg_part* p, const double* gathered, int world, int phase);
int lspcg_part_update_p_dev(lspcg_part* p, const void* z, void* p_ext);
int lspcg_part_update_xr_dev(lspcg_part* p, const void* p_ext, const void* q, void* x, void* r_ext);
int lspcg_part_status(lspcg_part* p, int64_t* iter, int* done);
/* The SpMV phases (lt / l / a) of this part store and reduce own rows [r0, n_own) only (default 0):
 * dist_pcg keeps one part for the interior rows (every column owned: computed while the halo
 * exchange is in flight) and one with r0 = the first boundary row (after it). */
int lspcg_part_set_rows(lspcg_part* p, int64_t r0);
/* lspcg_part_status plus the state's ‖r_k‖² and atol: the host sizes the next chunk of enqueued
 * iterations from the residual's decay (as lspcg_solver_solve does), so few iterations are enqueued
 * past convergence -- each would still run its halo exchanges and all-gathers. */
int lspcg_part_progress(lspcg_part* p, int64_t* iter, int* done, double* rr, double* atol);

#ifdef __cplusplus
}
#endif

#endif /* LSPCG_H_ */
