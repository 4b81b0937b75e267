// Rank-local phases of ONE system row-partitioned over ranks (not in the
// reference, whose systems each fit one process).  The host driver (dist_pcg.py) owns the
// exchange -- halo all-to-alls and all-gathers of dot partials over torch.distributed (RCCL over
// xGMI) -- and the scalar recurrence of scipy's cg (iterative.py:359-418, the reference's CPU
// restatement validate.py:163-201); each call here enqueues one device phase on the ctx stream.
//
// Rank layout: the rank owns n_own consecutive global rows.  Its rows of A, L and Lᵀ are stored
// as square n_ext x n_ext matrices (rows >= n_own empty) over the rank's EXTENDED vector
// [own rows | halo], the halo ordered by owner rank, so one all-to-all lands every received
// entry in place (no unpack).  The SpMVs are the library's (SELL-64 copy when prepared, else
// staged CSR) with epilogues that write own rows only and pre-reduce their compensated dot
// partials per group of workgroups (grid_partial_groups) into a 64-group DD buffer the host
// gathers across ranks: every expression is the single-GPU solver's (lspcg_pcg.hip), the dot
// totals are compensated sums in a different (rank-major) order.
#include <hip/hip_runtime.h>

#include <memory>
#include <string>

#include "lspcg_internal.hpp"
#include "lspcg_sell.hpp"
#include "lspcg_spmv.hpp"

namespace lspcg {

constexpr int kPartGroups = 64;  // group slots of a reduction buffer (kMaxGroups)

// own-row store (rows >= n_own of the extended matrix are empty and skipped; so are rows < r0, the
// part's first row -- lspcg_part_set_rows: a part that runs the boundary rows only)
template <typename T>
struct EpiOwn {
  static constexpr int NDOT = 0;
  T* y;
  int64_t n_own;
  double* partials = nullptr;
  unsigned* ticket = nullptr;
  int64_t r0 = 0;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD*) const {
    if (i >= r0 && i < n_own) gst(y + i, s);
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

// group size from the launch's own grid: <= kPartGroups groups, the buffer zeroed beforehand
__device__ __forceinline__ int part_gsz() { return int((gridDim.x + kPartGroups - 1) / kPartGroups); }

// z = L t + ε r (EpiZ's expression); groups of r·z and r·r
template <typename T>
struct EpiZPart {
  static constexpr int NDOT = 2;
  static constexpr bool GROUPS = true;
  T* z;
  const T* r;
  T eps;
  int64_t n_own;
  double* partials;
  unsigned* ticket;
  double* group_out;
  int gsz;
  int64_t r0 = 0;
  __device__ __forceinline__ void prepare() { gsz = part_gsz(); }
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    if (i < r0 || i >= n_own) return;
    const T ri = gld(r + i);
    const T zi = s + eps * ri;
    gst(z + i, zi);
    dd_fma(dots[0], double(ri), double(zi));
    dd_fma(dots[1], double(ri), double(ri));
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

// q = A p; groups of p·q (EpiQG's expression)
template <typename T>
struct EpiQPart {
  static constexpr int NDOT = 1;
  static constexpr bool GROUPS = true;
  T* q;
  const T* p;
  int64_t n_own;
  double* partials;
  unsigned* ticket;
  double* group_out;
  int gsz;
  int64_t r0 = 0;
  __device__ __forceinline__ void prepare() { gsz = part_gsz(); }
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    if (i < r0 || i >= n_own) return;
    gst(q + i, s);
    dd_fma(dots[0], double(gld(p + i)), double(s));
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_pack(int64_t m, const int32_t* __restrict__ idx,
                                                        const T* __restrict__ v, T* __restrict__ out) {
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += int64_t(gridDim.x) * blockDim.x)
    out[k] = v[idx[k]];
}

// p = z (first) or p β + z  (scipy `p *= beta; p += z`, k_update_p's expression)
template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_update_p(int64_t n, const T* __restrict__ z, T* __restrict__ p,
                                                            T beta, int first) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = first ? z[i] : (p[i] * beta) + z[i];
}

// x += α p ; r -= α q
template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_update_xr(int64_t n, T alpha, const T* __restrict__ p,
                                                             const T* __restrict__ q, T* __restrict__ x,
                                                             T* __restrict__ r) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    x[i] = x[i] + alpha * p[i];
    r[i] = r[i] - alpha * q[i];
  }
}

// groups of a·a and b·b over the own rows (the init's ‖r_0‖², ‖b‖²)
template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_norms(int64_t n, const T* __restrict__ a, const T* __restrict__ b,
                                                         double* partials, unsigned* ticket, double* group_out) {
  DD d[2] = {dd_zero(), dd_zero()};
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const T ai = a[i], bi = b[i];
    dd_fma(d[0], double(ai), double(ai));
    dd_fma(d[1], double(bi), double(bi));
  }
  grid_partial_groups<2>(d, partials, ticket, part_gsz(), group_out);
}

// ---- device-side scalar recurrence (round 4): the dot totals, scipy's scalars and its top-of-loop
// test computed on the device from the all-gathered group pairs, so an iteration needs no host
// round trip (the host polls the state once per chunk of iterations).  One thread sums every
// rank's 64 group pairs in rank-major order with dd_add -- dist_pcg.sum_groups' order, so the
// scalars are the host recurrence's bits -- and every later kernel of the iteration reads them.
struct PartState {
  double rtol, atol, rr, rho, rho_prev, pq, alpha, beta, bb;
  int64_t iter, max_iter;
  int32_t done;  // 0 running, 1 converged, 2 max_iter, 3 non-finite residual, 4 ‖b‖ = 0
  int32_t pad;
  double* hist;  // ‖r_k‖, k = 0 .. iter (device, caller-owned; may be NULL)
};

template <typename T>
__device__ __forceinline__ T part_sqrt(T v) { return sqrt(v); }

// total j of the gathered [world][64 groups][nd][2] pairs, rank-major (sum_groups' order)
__device__ double part_total(const double* g, int world, int nd, int j) {
  DD acc = dd_zero();
  for (int r = 0; r < world; ++r)
    for (int k = 0; k < kPartGroups; ++k) {
      const double* e = g + (size_t(r) * kPartGroups * nd + size_t(k) * nd + j) * 2;
      acc = dd_add(acc, DD{e[0], e[1]});
    }
  return acc.s + acc.c;
}

// top-of-loop test (k_update_p_g's): sets done, returns true when the loop stops here
template <typename T>
__device__ __forceinline__ bool part_test(PartState* S) {
  int code = 0;
  if (S->iter >= S->max_iter) {
    code = 2;
  } else {
    const double rn = double(part_sqrt<T>(T(S->rr)));
    if (rn < S->atol) code = 1;
    else if (!(rn == rn) || rn == INFINITY) code = 3;
  }
  if (code) S->done = code;
  return code != 0;
}

enum PartPhase { kPartInit = 0, kPartZ = 1, kPartZcg = 2, kPartQ = 3, kPartR = 4 };

template <typename T>
__global__ void k_part_scalars(PartState* S, const double* __restrict__ g, int world, int phase) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (phase == kPartInit) {  // rr0 = r·r, bb = b·b (r = b); atol = max(0, rtol ‖b‖)
    const double rr0 = round_to<T>(part_total(g, world, 2, 0));
    const double bb = round_to<T>(part_total(g, world, 2, 1));
    const double bn = double(part_sqrt<T>(T(bb)));
    S->rr = rr0;
    S->bb = bb;
    S->atol = fmax(0.0, S->rtol * bn);
    S->iter = 0;
    S->done = bn == 0.0 ? 4 : 0;
    if (S->hist) S->hist[0] = double(part_sqrt<T>(T(rr0)));
    return;
  }
  if (S->done) return;
  if (phase == kPartZ || phase == kPartZcg) {
    const int64_t k = S->iter;
    double rho;
    if (phase == kPartZ) {  // ρ = r·z and ‖r_k‖² from L's launch
      rho = round_to<T>(part_total(g, world, 2, 0));
      const double rr_k = round_to<T>(part_total(g, world, 2, 1));
      if (k > 0) S->rr = rr_k;
    } else {  // CG: z = r, ρ = ‖r_k‖² (from the init or the previous kPartR)
      rho = S->rr;
    }
    if (k > 0 && S->hist) S->hist[k] = double(part_sqrt<T>(T(S->rr)));
    S->rho = rho;
    if (part_test<T>(S)) return;
    S->beta = k == 0 ? 0.0 : double(T(rho) / T(S->rho_prev));
  } else if (phase == kPartQ) {  // π = p·q ; α = ρ/π
    const double pq = round_to<T>(part_total(g, world, 1, 0));
    S->pq = pq;
    S->alpha = double(T(S->rho) / T(pq));
  } else {  // kPartR (CG): ‖r_{k+1}‖² for the next test
    S->rr = round_to<T>(part_total(g, world, 2, 0));
  }
}

// p = z (k = 0) or p β + z, scalars from the device state
template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_update_p_dev(int64_t n, const PartState* S, const T* __restrict__ z,
                                                                T* __restrict__ p) {
  if (S->done) return;
  const bool first = S->iter == 0;
  const T beta = T(S->beta);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = first ? z[i] : (p[i] * beta) + z[i];
}

// x += α p ; r -= α q ; then ρ_prev = ρ and the iteration count (workgroup 0, thread 0: the
// other workgroups read only α and done, which it does not write)
template <typename T>
__global__ void __launch_bounds__(kThreads) k_part_update_xr_dev(int64_t n, PartState* S, const T* __restrict__ p,
                                                                 const T* __restrict__ q, T* __restrict__ x,
                                                                 T* __restrict__ r) {
  if (S->done) return;
  const T alpha = T(S->alpha);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    x[i] = x[i] + alpha * p[i];
    r[i] = r[i] - alpha * q[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->rho_prev = S->rho;
    S->iter = S->iter + 1;
  }
}

static int part_grid(int64_t n) {
  const int64_t g = (n + kThreads - 1) / kThreads;
  return int(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

}  // namespace lspcg

using namespace lspcg;

struct lspcg_part {
  lspcg_ctx* ctx = nullptr;
  const lspcg_mat* A = nullptr;
  const lspcg_mat* L = nullptr;
  const lspcg_mat* LT = nullptr;
  int dtype = LSPCG_F64;
  int64_t n_own = 0, n_ext = 0, n_send = 0;
  int64_t r0 = 0;               // first own row of the SpMV phases (lspcg_part_set_rows)
  int32_t* send_idx = nullptr;  // owned device copy
  double* partials = nullptr;
  unsigned* ticket = nullptr;
  PartState* S = nullptr;  // device state of the device-side recurrence
};

namespace {

// SpMV of an extended matrix with a fused epilogue: the SELL copy when prepared, else staged CSR
template <typename T, class Epi>
int part_spmv(lspcg_part* p, const lspcg_mat* M, const void* x, Epi epi) {
  hipStream_t st = p->ctx->stream;
  const T* xv = static_cast<const T*>(x);
  if (const SellCopy* c = M->sell; c && !c->ro.perm) {  // (a reordered copy is of P M Pᵀ: the row epilogues
    launch_spmv_sell_cfg<T, T>(c->P, c->vals, GatherVec<T>{xv}, ProNone{}, epi, st);  // need M's rows)
    return LSPCG_OK;
  }
  return launch_spmv_any<T>(M, xv, ProNone{}, epi, st);
}

int check_mat(const lspcg_part* p, const lspcg_mat* M, const char* what) {
  LSPCG_CHECK(M && M->n == p->n_ext && M->dtype == p->dtype, LSPCG_ERR_ARG,
              std::string("part_create: ") + what + " must be n_ext x n_ext in the dtype of A");
  return LSPCG_OK;
}

}  // namespace

extern "C" {

int lspcg_part_create(lspcg_ctx* ctx, const lspcg_mat* A, const lspcg_mat* L, const lspcg_mat* LT, int64_t n_own,
                      const int32_t* send_idx, int64_t n_send, lspcg_part** out) {
  LSPCG_CHECK(ctx && A && out && (n_send == 0 || send_idx), LSPCG_ERR_ARG, "part_create: NULL argument");
  LSPCG_CHECK(n_own >= 0 && n_own <= A->n && n_send >= 0, LSPCG_ERR_ARG, "part_create: bad sizes");
  LSPCG_CHECK(A->dtype == LSPCG_F64 || A->dtype == LSPCG_F32, LSPCG_ERR_ARG, "part_create: dtype");
  LSPCG_CHECK(A->block_size == 1 && (!L || L->block_size == 1) && (!LT || LT->block_size == 1), LSPCG_ERR_UNSUPPORTED,
              "part_create: scalar CSR matrices only");
  LSPCG_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<lspcg_part> p(new lspcg_part());
  p->ctx = ctx;
  p->A = A;
  p->L = L;
  p->LT = LT;
  p->dtype = A->dtype;
  p->n_own = n_own;
  p->n_ext = A->n;
  p->n_send = n_send;
  if (L && check_mat(p.get(), L, "L")) return LSPCG_ERR_ARG;
  if (LT && check_mat(p.get(), LT, "LT")) return LSPCG_ERR_ARG;
  LSPCG_CHECK((L == nullptr) == (LT == nullptr), LSPCG_ERR_ARG, "part_create: give both L and LT or neither");
  hipStream_t st = ctx->stream;
  if (n_send) {
    LSPCG_HIP(hipMalloc(&p->send_idx, sizeof(int32_t) * n_send));
    LSPCG_HIP(hipMemcpyAsync(p->send_idx, send_idx, sizeof(int32_t) * n_send, hipMemcpyDefault, st));
  }
  LSPCG_HIP(hipMalloc(&p->partials, sizeof(double) * 2 * 2 * (kReduceBlocksMax + 1)));
  LSPCG_HIP(hipMalloc(&p->ticket, sizeof(unsigned) * kTicketWords));
  LSPCG_HIP(hipMemsetAsync(p->ticket, 0, sizeof(unsigned) * kTicketWords, st));
  LSPCG_HIP(hipMalloc(&p->S, sizeof(PartState)));
  LSPCG_HIP(hipMemsetAsync(p->S, 0, sizeof(PartState), st));
  LSPCG_HIP(hipStreamSynchronize(st));
  *out = p.release();
  return LSPCG_OK;
}

int lspcg_part_destroy(lspcg_part* p) {
  if (!p) return LSPCG_OK;
  (void)hipSetDevice(p->ctx->device);
  (void)hipStreamSynchronize(p->ctx->stream);
  for (void* v : {(void*)p->send_idx, (void*)p->partials, (void*)p->ticket, (void*)p->S}) (void)hipFree(v);
  delete p;
  return LSPCG_OK;
}

int lspcg_part_pack(lspcg_part* p, const void* v, void* sendbuf) {
  LSPCG_CHECK(p && v && (p->n_send == 0 || sendbuf), LSPCG_ERR_ARG, "part_pack: NULL argument");
  if (!p->n_send) return LSPCG_OK;
  hipStream_t st = p->ctx->stream;
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_pack<double>, dim3(part_grid(p->n_send)), dim3(kThreads), 0, st, p->n_send, p->send_idx,
                       static_cast<const double*>(v), static_cast<double*>(sendbuf));
  else
    hipLaunchKernelGGL(k_part_pack<float>, dim3(part_grid(p->n_send)), dim3(kThreads), 0, st, p->n_send, p->send_idx,
                       static_cast<const float*>(v), static_cast<float*>(sendbuf));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_norms(lspcg_part* p, const void* a, const void* b, double* red) {
  LSPCG_CHECK(p && a && b && red, LSPCG_ERR_ARG, "part_norms: NULL argument");
  hipStream_t st = p->ctx->stream;
  LSPCG_HIP(hipMemsetAsync(red, 0, sizeof(double) * kPartGroups * 2 * 2, st));
  const int g = part_grid(p->n_own);
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_norms<double>, dim3(g), dim3(kThreads), 0, st, p->n_own, static_cast<const double*>(a),
                       static_cast<const double*>(b), p->partials, p->ticket, red);
  else
    hipLaunchKernelGGL(k_part_norms<float>, dim3(g), dim3(kThreads), 0, st, p->n_own, static_cast<const float*>(a),
                       static_cast<const float*>(b), p->partials, p->ticket, red);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_lt(lspcg_part* p, const void* r_ext, void* t_ext) {
  LSPCG_CHECK(p && p->LT && r_ext && t_ext, LSPCG_ERR_ARG, "part_lt: NULL argument (or no L)");
  EpiOwn<double> ed{static_cast<double*>(t_ext), p->n_own};
  EpiOwn<float> ef{static_cast<float*>(t_ext), p->n_own};
  ed.r0 = ef.r0 = p->r0;
  int rc = p->dtype == LSPCG_F64 ? part_spmv<double>(p, p->LT, r_ext, ed) : part_spmv<float>(p, p->LT, r_ext, ef);
  if (rc) return rc;
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_l(lspcg_part* p, const void* t_ext, const void* r, double eps, void* z, double* red) {
  LSPCG_CHECK(p && p->L && t_ext && r && z && red, LSPCG_ERR_ARG, "part_l: NULL argument (or no L)");
  hipStream_t st = p->ctx->stream;
  LSPCG_HIP(hipMemsetAsync(red, 0, sizeof(double) * kPartGroups * 2 * 2, st));
  int rc;
  if (p->dtype == LSPCG_F64) {
    EpiZPart<double> e{static_cast<double*>(z), static_cast<const double*>(r), eps, p->n_own, p->partials, p->ticket,
                       red, 1};
    e.r0 = p->r0;
    rc = part_spmv<double>(p, p->L, t_ext, e);
  } else {
    EpiZPart<float> e{static_cast<float*>(z), static_cast<const float*>(r), float(eps), p->n_own, p->partials,
                      p->ticket, red, 1};
    e.r0 = p->r0;
    rc = part_spmv<float>(p, p->L, t_ext, e);
  }
  if (rc) return rc;
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_a(lspcg_part* p, const void* p_ext, void* q, double* red) {
  LSPCG_CHECK(p && p_ext && q && red, LSPCG_ERR_ARG, "part_a: NULL argument");
  hipStream_t st = p->ctx->stream;
  LSPCG_HIP(hipMemsetAsync(red, 0, sizeof(double) * kPartGroups * 2, st));
  int rc;
  if (p->dtype == LSPCG_F64) {
    EpiQPart<double> e{static_cast<double*>(q), static_cast<const double*>(p_ext), p->n_own, p->partials, p->ticket,
                       red, 1};
    e.r0 = p->r0;
    rc = part_spmv<double>(p, p->A, p_ext, e);
  } else {
    EpiQPart<float> e{static_cast<float*>(q), static_cast<const float*>(p_ext), p->n_own, p->partials, p->ticket,
                      red, 1};
    e.r0 = p->r0;
    rc = part_spmv<float>(p, p->A, p_ext, e);
  }
  if (rc) return rc;
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_update_p(lspcg_part* p, const void* z, void* p_ext, double beta, int first) {
  LSPCG_CHECK(p && z && p_ext, LSPCG_ERR_ARG, "part_update_p: NULL argument");
  hipStream_t st = p->ctx->stream;
  const int g = part_grid(p->n_own);
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_update_p<double>, dim3(g), dim3(kThreads), 0, st, p->n_own, static_cast<const double*>(z),
                       static_cast<double*>(p_ext), beta, first);
  else
    hipLaunchKernelGGL(k_part_update_p<float>, dim3(g), dim3(kThreads), 0, st, p->n_own, static_cast<const float*>(z),
                       static_cast<float*>(p_ext), float(beta), first);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_update_xr(lspcg_part* p, double alpha, const void* p_ext, const void* q, void* x, void* r_ext) {
  LSPCG_CHECK(p && p_ext && q && x && r_ext, LSPCG_ERR_ARG, "part_update_xr: NULL argument");
  hipStream_t st = p->ctx->stream;
  const int g = part_grid(p->n_own);
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_update_xr<double>, dim3(g), dim3(kThreads), 0, st, p->n_own, alpha,
                       static_cast<const double*>(p_ext), static_cast<const double*>(q), static_cast<double*>(x),
                       static_cast<double*>(r_ext));
  else
    hipLaunchKernelGGL(k_part_update_xr<float>, dim3(g), dim3(kThreads), 0, st, p->n_own, float(alpha),
                       static_cast<const float*>(p_ext), static_cast<const float*>(q), static_cast<float*>(x),
                       static_cast<float*>(r_ext));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_state_init(lspcg_part* p, double rtol, int64_t max_iter, double* hist) {
  LSPCG_CHECK(p && max_iter > 0, LSPCG_ERR_ARG, "part_state_init: bad argument");
  PartState h{};
  h.rtol = rtol;
  h.max_iter = max_iter;
  h.hist = hist;
  LSPCG_HIP(hipMemcpyAsync(p->S, &h, sizeof(PartState), hipMemcpyHostToDevice, p->ctx->stream));
  LSPCG_HIP(hipStreamSynchronize(p->ctx->stream));  // h is a stack copy
  return LSPCG_OK;
}

int lspcg_part_scalars(lspcg_part* p, const double* gathered, int world, int phase) {
  LSPCG_CHECK(p && world >= 1 && phase >= kPartInit && phase <= kPartR && (gathered || phase == kPartZcg),
              LSPCG_ERR_ARG, "part_scalars: bad argument");
  hipStream_t st = p->ctx->stream;
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_scalars<double>, dim3(1), dim3(64), 0, st, p->S, gathered, world, phase);
  else
    hipLaunchKernelGGL(k_part_scalars<float>, dim3(1), dim3(64), 0, st, p->S, gathered, world, phase);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_update_p_dev(lspcg_part* p, const void* z, void* p_ext) {
  LSPCG_CHECK(p && z && p_ext, LSPCG_ERR_ARG, "part_update_p_dev: NULL argument");
  hipStream_t st = p->ctx->stream;
  const int g = part_grid(p->n_own);
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_update_p_dev<double>, dim3(g), dim3(kThreads), 0, st, p->n_own, p->S,
                       static_cast<const double*>(z), static_cast<double*>(p_ext));
  else
    hipLaunchKernelGGL(k_part_update_p_dev<float>, dim3(g), dim3(kThreads), 0, st, p->n_own, p->S,
                       static_cast<const float*>(z), static_cast<float*>(p_ext));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_update_xr_dev(lspcg_part* p, const void* p_ext, const void* q, void* x, void* r_ext) {
  LSPCG_CHECK(p && p_ext && q && x && r_ext, LSPCG_ERR_ARG, "part_update_xr_dev: NULL argument");
  hipStream_t st = p->ctx->stream;
  const int g = part_grid(p->n_own);
  if (p->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_part_update_xr_dev<double>, dim3(g), dim3(kThreads), 0, st, p->n_own, p->S,
                       static_cast<const double*>(p_ext), static_cast<const double*>(q), static_cast<double*>(x),
                       static_cast<double*>(r_ext));
  else
    hipLaunchKernelGGL(k_part_update_xr_dev<float>, dim3(g), dim3(kThreads), 0, st, p->n_own, p->S,
                       static_cast<const float*>(p_ext), static_cast<const float*>(q), static_cast<float*>(x),
                       static_cast<float*>(r_ext));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_part_status(lspcg_part* p, int64_t* iter, int* done) {
  LSPCG_CHECK(p && iter && done, LSPCG_ERR_ARG, "part_status: NULL argument");
  PartState h{};
  LSPCG_HIP(hipMemcpyAsync(&h, p->S, sizeof(PartState), hipMemcpyDeviceToHost, p->ctx->stream));
  LSPCG_HIP(hipStreamSynchronize(p->ctx->stream));
  *iter = h.iter;
  *done = h.done;
  return LSPCG_OK;
}

int lspcg_part_set_rows(lspcg_part* p, int64_t r0) {
  LSPCG_CHECK(p && r0 >= 0 && r0 <= p->n_own, LSPCG_ERR_ARG, "part_set_rows: r0 outside [0, n_own]");
  p->r0 = r0;
  return LSPCG_OK;
}

int lspcg_part_progress(lspcg_part* p, int64_t* iter, int* done, double* rr, double* atol) {
  LSPCG_CHECK(p && iter && done && rr && atol, LSPCG_ERR_ARG, "part_progress: NULL argument");
  PartState h{};
  LSPCG_HIP(hipMemcpyAsync(&h, p->S, sizeof(PartState), hipMemcpyDeviceToHost, p->ctx->stream));
  LSPCG_HIP(hipStreamSynchronize(p->ctx->stream));
  *iter = h.iter;
  *done = h.done;
  *rr = h.rr;
  *atol = h.atol;
  return LSPCG_OK;
}

}  // extern "C"
