// Device-resident preconditioned CG (replaces pymathprim.linalg.PreconditionedConjugateGradient,
// call sites neural_cg/utils/validate.py:54-160; arithmetic of scipy 1.15 iterative.py:359-418,
// the reference's CPU restatement validate.py:163-341).
//
// Schedules, all with scipy's exact floating-point expressions, so every schedule
// produces the same iterate and residual history bit for bit:
//   * split ext_spai schedule (SELL views): five launches per iteration
//       KA  t = Lᵀ r_k                                         [SpMV Lᵀ]
//       KB  z = L t + ε r_k ; group partials of ρ_k = r_k·z, ‖r_k‖²   [SpMV L]
//       UP  top-of-loop test on ‖r_k‖ ; x += α_{k-1} p_{k-1} ; p_k = p_{k-1}β + z
//       KC  q = A p_k ; group partials of π_k = p_k·q              [SpMV A]
//       UR  α_k = ρ_k/π_k ; r_{k+1} = r_k - α_k q
//   * the same five phases with last-arriver grid reductions (CSR / BSR views, CG, Jacobi, IC);
//   * one-workgroup solve (k_pcg_small) for n <= LSPCG_SMALL_N.
// Every multi-launch kernel is predicated on a device `done` flag, so the host replays
// graph-captured chunks of iterations and polls once per chunk without changing the iteration
// count or the iterate; the deferred x update of the last iteration is one fix-up launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "lspcg_factor.hpp"
#include "lspcg_internal.hpp"
#include "lspcg_sell.hpp"
#include "lspcg_spmv.hpp"

namespace lspcg {

struct PcgState {
  double bb;        // ‖b‖²
  double rr;        // ‖r_k‖² (rounded to T)
  double rho;       // ρ_k = r_k·z_k (rounded to T)
  double rho_prev;  // ρ_{k-1}
  double pq;        // π_k = p_k·q_k (rounded to T)
  double alpha;     // α_k = ρ_k/π_k computed in T
  double atol;      // rtol·‖b‖
  double rtol;
  double eps;       // ε of ext_spai
  double* hist;     // ‖r_k‖ history (nullable)
  int64_t iter;     // completed iterations
  int64_t max_iter;
  int32_t done;     // 0 running, 1 converged, 2 max_iter reached, 3 non-finite residual
  int32_t pad;
  double rho_k;     // split schedule: ρ_k as UP summed it from KB's groups, read by UR (same bits)
};

template <typename T>
__device__ __forceinline__ T tsqrt(T v) { return sqrt(v); }

// Top-of-iteration test of scipy's loop: `for iteration in range(maxiter): if norm(r) < atol`.
template <typename T>
struct ProCheck {
  PcgState* S;
  __device__ __forceinline__ bool exit() const {
    if (S->done) return true;
    int code = 0;
    if (S->iter >= S->max_iter) {
      code = 2;
    } else {
      const double rn = double(tsqrt<T>(T(S->rr)));
      if (rn < S->atol) code = 1;
      else if (!(rn == rn) || rn == INFINITY) code = 3;
    }
    if (code && blockIdx.x == 0 && threadIdx.x == 0) S->done = code;
    return code != 0;
  }
};

struct ProDone {
  const PcgState* S;
  __device__ __forceinline__ bool exit() const { return S->done != 0; }
};

// KA (ext_spai): t = Lᵀ r  (scaled variant: t = (Lᵀ r)/d)
template <typename T, bool SCALED>
struct EpiT {
  static constexpr int NDOT = 0;
  T* t;
  const T* d;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD*) const {
    if constexpr (SCALED) gst(t + i, s / gld(d + i));
    else gst(t + i, s);
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

// KB: z = L t + ε r  (scaled: z = L t + (ε r)/d);  ρ = r·z and ‖r‖² in the same reduction
// (the top-of-loop test on ‖r_k‖ then runs in the p update; r_0's norm comes from the init)
template <typename T, bool SCALED>
struct EpiZ {
  static constexpr int NDOT = 2;
  T* z;
  const T* r;
  const T* d;
  T eps;
  PcgState* S;
  double* partials;
  unsigned* ticket;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T ri = gld(r + i);
    T zi;
    if constexpr (SCALED) zi = s + (eps * ri) / gld(d + i);
    else zi = s + eps * ri;
    gst(z + i, zi);
    dd_fma(dots[0], double(ri), double(zi));
    dd_fma(dots[1], double(ri), double(ri));
  }
  __device__ __forceinline__ void fin(const double* v) const {
    S->rho_prev = S->rho;
    S->rho = round_to<T>(v[0]);
    const int64_t k = S->iter;
    if (k > 0) {
      const double rr = round_to<T>(v[1]);
      S->rr = rr;
      if (S->hist) S->hist[k] = double(tsqrt<T>(T(rr)));
    }
  }
};

// KD: q = A p ; π = p·q ; α = ρ/π  (INC: this launch also completes the iteration -- ext_spai,
// whose r update carries no reduction)
template <typename T, bool INC = false>
struct EpiQ {
  static constexpr int NDOT = 1;
  T* q;
  const T* p;
  PcgState* S;
  double* partials;
  unsigned* ticket;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    gst(q + i, s);
    dd_fma(dots[0], double(gld(p + i)), double(s));
  }
  __device__ __forceinline__ void fin(const double* v) const {
    const double pq = round_to<T>(v[0]);
    S->pq = pq;
    S->alpha = double(T(S->rho) / T(pq));
    if constexpr (INC) S->iter = S->iter + 1;
  }
};

// init: r_0 = b - A x0 ; ‖r_0‖², ‖b‖² (+ z_0 = r_0/d, ρ_0 = r_0·z_0 for Jacobi)
// (scipy: r = b - matvec(x) if x.any() else b.copy(); with x0 = 0 the subtraction returns b)
template <typename T, int PRE>
struct EpiResid {
  static constexpr int NDOT = PRE == LSPCG_PRECOND_DIAGONAL ? 3 : 2;
  T* r;
  const T* b;
  const T* d;
  T* z;
  PcgState* S;
  double* partials;
  unsigned* ticket;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T bi = b[i];
    const T ri = bi - s;
    r[i] = ri;
    dd_fma(dots[0], double(ri), double(ri));
    dd_fma(dots[1], double(bi), double(bi));
    if constexpr (PRE == LSPCG_PRECOND_DIAGONAL) {
      const T zi = ri / d[i];
      z[i] = zi;
      dd_fma(dots[2], double(ri), double(zi));
    }
  }
  __device__ __forceinline__ void fin(const double* v) const {
    S->rr = round_to<T>(v[0]);
    S->bb = round_to<T>(v[1]);
    const double bn = double(tsqrt<T>(T(S->bb)));
    S->atol = fmax(0.0, S->rtol * bn);
    S->rho = PRE == LSPCG_PRECOND_DIAGONAL ? round_to<T>(v[2]) : S->rr;
    S->alpha = 0.0;
    S->iter = 0;
    S->done = (bn == 0.0) ? 1 : 0;
    if (S->hist) S->hist[0] = double(tsqrt<T>(T(S->rr)));
  }
};

// ---- elementwise kernels: 16-B vectors, 2 vectors per lane, grid <= kReduceGridMax
template <typename T>
struct VecT {
  static constexpr int W = 16 / sizeof(T);
  using type = T __attribute__((ext_vector_type(W)));
};
constexpr int kElemUnroll = 2;

template <typename T>
static int elem_vec_grid(int64_t n) {
  const int64_t nv = n / VecT<T>::W;
  const int64_t g = (nv + int64_t(kThreads) * kElemUnroll - 1) / (int64_t(kThreads) * kElemUnroll);
  return int(std::max<int64_t>(1, std::min<int64_t>(g, kReduceGridMax)));
}

// KC: x += α_{k-1} p_{k-1} (deferred, k > 0) ; p_k = p_{k-1}β + z (scipy `p *= beta; p += z`),
// p_0 = z.  `Pro` = ProCheck for CG / Jacobi (top-of-loop test), ProDone for ext_spai.
template <typename T, typename Pro>
__global__ void __launch_bounds__(kThreads) k_update_p(int64_t n, Pro pro, const PcgState* S,
                                                       const T* __restrict__ z, T* __restrict__ p,
                                                       T* __restrict__ x) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  if (pro.exit()) return;
  const bool first = S->iter == 0;
  const T beta = first ? T(0) : T(S->rho) / T(S->rho_prev);
  const T alpha = T(S->alpha);
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  for (int64_t j0 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j0 < nv; j0 += ts * kElemUnroll) {
    V zz[kElemUnroll], pp[kElemUnroll], xx[kElemUnroll];
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        zz[u] = reinterpret_cast<const V*>(z)[j];
        pp[u] = reinterpret_cast<const V*>(p)[j];
        xx[u] = reinterpret_cast<const V*>(x)[j];
      }
    }
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        if (!first) reinterpret_cast<V*>(x)[j] = xx[u] + alpha * pp[u];
        reinterpret_cast<V*>(p)[j] = first ? zz[u] : (pp[u] * beta) + zz[u];
      }
    }
  }
  for (int64_t i = nv * W + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += ts) {
    const T pi = p[i];
    if (!first) x[i] = x[i] + alpha * pi;
    p[i] = first ? z[i] : (pi * beta) + z[i];
  }
}

// KE: r -= α q ; ‖r‖² (+ Jacobi z = r/d, ρ = r·z) ; iteration count
template <typename T, int PRE>
__global__ void __launch_bounds__(kThreads) k_update_r(int64_t n, PcgState* S, const T* __restrict__ q,
                                                       T* __restrict__ r, const T* __restrict__ d, T* __restrict__ z,
                                                       double* partials, unsigned* ticket) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  constexpr int ND = PRE == LSPCG_PRECOND_DIAGONAL ? 2 : 1;
  if (S->done) return;
  const T alpha = T(S->alpha);
  DD dots[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) dots[j] = dd_zero();
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  auto elem = [&](T ri, int64_t i) {
    dd_fma(dots[0], double(ri), double(ri));
    if constexpr (PRE == LSPCG_PRECOND_DIAGONAL) {
      const T zi = ri / d[i];
      z[i] = zi;
      dd_fma(dots[1], double(ri), double(zi));
    }
  };
  for (int64_t j0 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j0 < nv; j0 += ts * kElemUnroll) {
    V rr[kElemUnroll], qq[kElemUnroll];
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        rr[u] = reinterpret_cast<const V*>(r)[j];
        qq[u] = reinterpret_cast<const V*>(q)[j];
      }
    }
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        const V rn = rr[u] - alpha * qq[u];
        reinterpret_cast<V*>(r)[j] = rn;
#pragma unroll
        for (int w = 0; w < W; ++w) elem(rn[w], j * W + w);
      }
    }
  }
  for (int64_t i = nv * W + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += ts) {
    const T ri = r[i] - alpha * q[i];
    r[i] = ri;
    elem(ri, i);
  }
  grid_reduce_dd<ND>(dots, partials, ticket, [&](const double* v) {
    const double rr2 = round_to<T>(v[0]);
    S->rr = rr2;
    if constexpr (PRE == LSPCG_PRECOND_NONE || PRE == LSPCG_PRECOND_DIAGONAL) {
      S->rho_prev = S->rho;
      S->rho = (PRE == LSPCG_PRECOND_DIAGONAL) ? round_to<T>(v[ND - 1]) : rr2;
    }
    const int64_t it = S->iter + 1;
    S->iter = it;
    if (S->hist) S->hist[it] = double(tsqrt<T>(T(rr2)));
  });
}

// ext_spai: r -= α q only (‖r‖² is reduced by the next L SpMV, the iteration count by KC)
template <typename T>
__global__ void __launch_bounds__(kThreads) k_update_r_nodot(int64_t n, const PcgState* S, const T* __restrict__ q,
                                                             T* __restrict__ r) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  if (S->done) return;
  const T alpha = T(S->alpha);
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  for (int64_t j0 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j0 < nv; j0 += ts * kElemUnroll) {
    V rr[kElemUnroll], qq[kElemUnroll];
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        rr[u] = reinterpret_cast<const V*>(r)[j];
        qq[u] = reinterpret_cast<const V*>(q)[j];
      }
    }
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) reinterpret_cast<V*>(r)[j] = rr[u] - alpha * qq[u];
    }
  }
  for (int64_t i = nv * W + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += ts) r[i] = r[i] - alpha * q[i];
}

// ---- split-reduction ext_spai schedule (SELL views; DESIGN.md "PCG schedule") --------------
// KB and KC only pre-reduce their dot partials per group of workgroups (grid_partial_groups);
// the elementwise launches that consume the scalars sum the <= 64 group totals themselves:
//   KA  t = Lᵀ r_k
//   KB  z = L t + ε r_k ; groups of ρ_k = r_k·z and ‖r_k‖²                 -> GZ
//   UP  ρ_k, ‖r_k‖ from GZ ; top-of-loop test ; x += α_{k-1} p_{k-1} ; p_k = p_{k-1}β + z
//   KC  q = A p_k ; groups of π_k = p_k·q                                  -> GQ
//   UR  α_k = ρ_k/π_k from GZ, GQ ; r_{k+1} = r_k - α_k q ; persists ρ_k, α_k, iteration k+1
// Workgroup 0 of UP / UR is the only writer of the persistent state, which only later launches
// read; every workgroup computes the same scalars (same group totals, same summation tree).
struct GroupDots {
  unsigned* ticket;
  double* partials;
  double* group_out;
  int gsz;
};

template <typename T, bool SCALED>
struct EpiZG {
  static constexpr int NDOT = 2;
  static constexpr bool GROUPS = true;
  static constexpr bool PREFETCH = !SCALED;  // r[i] loaded before the row's gathers (SELL kernel)
  T* z;
  const T* r;
  const T* d;
  T eps;
  double* partials;
  unsigned* ticket;
  double* group_out;
  int gsz;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ T prefetch(int64_t i) const { return gld(r + i); }
  __device__ __forceinline__ void row_pf(int64_t i, T s, DD* dots, T ri) const {
    const T zi = s + eps * ri;
    gst(z + i, zi);
    dd_fma(dots[0], double(ri), double(zi));
    dd_fma(dots[1], double(ri), double(ri));
  }
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T ri = gld(r + i);
    T zi;
    if constexpr (SCALED) zi = s + (eps * ri) / gld(d + i);
    else zi = s + eps * ri;
    gst(z + i, zi);
    dd_fma(dots[0], double(ri), double(zi));
    dd_fma(dots[1], double(ri), double(ri));
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

template <typename T>
struct EpiQG {
  static constexpr int NDOT = 1;
  static constexpr bool GROUPS = true;
  static constexpr bool PREFETCH = true;  // p[i] loaded before the row's gathers (SELL kernel)
  T* q;
  const T* p;
  double* partials;
  unsigned* ticket;
  double* group_out;
  int gsz;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ T prefetch(int64_t i) const { return gld(p + i); }
  __device__ __forceinline__ void row_pf(int64_t i, T s, DD* dots, T pi) const {
    gst(q + i, s);
    dd_fma(dots[0], double(pi), double(s));
  }
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    gst(q + i, s);
    dd_fma(dots[0], double(gld(p + i)), double(s));
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

// UP.  The first chunk's vector loads are issued before the group sums, so their latency overlaps
// the scalar reduction instead of following it.  x is read and written with non-temporal accesses:
// nothing else in the iteration touches it, and streaming it past the caches keeps its 8 B per row
// out of the loop's Infinity-Cache working set (kuhn101: 69.2 vs 71.0 us per iteration,
// tools/loop_ab.py, profiles/r4_loop_ab_v1.jsonl).
template <typename T>
__global__ void __launch_bounds__(kThreads) k_update_p_g(int64_t n, PcgState* S, const double* __restrict__ gz, int ngz,
                                                         const T* __restrict__ z, T* __restrict__ p,
                                                         T* __restrict__ x) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  const int64_t jt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  V zz[kElemUnroll], pp[kElemUnroll], xx[kElemUnroll];
  auto load = [&](int64_t j0) {
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        zz[u] = reinterpret_cast<const V*>(z)[j];
        pp[u] = reinterpret_cast<const V*>(p)[j];
        xx[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(x) + j);
      }
    }
  };
  // the first chunk, the group totals and every state field are all loaded before the first test:
  // one memory latency instead of a state read followed by the loads (the state fields are read
  // into registers up front -- workgroup 0's state stores below would otherwise order the later
  // ρ_{k-1} / α_{k-1} reads after them, a second scalar round trip for every wave)
  load(jt);
  const int32_t done = S->done;
  const int64_t k = S->iter;
  const int64_t max_iter = S->max_iter;
  const double atol = S->atol, rr0 = S->rr, rho_prev = S->rho, alpha_prev = S->alpha;
  double* const hist = S->hist;
  double v[2];
  group_sum_dd<2>(gz, ngz, v);
  if (done) return;
  const double rho = round_to<T>(v[0]);
  const double rr = k > 0 ? round_to<T>(v[1]) : rr0;  // ‖r_0‖² from the init launch
  int code = 0;  // scipy's top-of-loop test (ProCheck)
  if (k >= max_iter) {
    code = 2;
  } else {
    const double rn = double(tsqrt<T>(T(rr)));
    if (rn < atol) code = 1;
    else if (!(rn == rn) || rn == INFINITY) code = 3;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (k > 0) {
      S->rr = rr;
      if (hist) hist[k] = double(tsqrt<T>(T(rr)));
    }
    if (code) S->done = code;
    else S->rho_k = rho;
  }
  if (code) return;
  const bool first = k == 0;
  const T beta = first ? T(0) : T(rho) / T(rho_prev);  // ρ_{k-1}
  const T alpha = T(alpha_prev);                        // α_{k-1}
  for (int64_t j0 = jt; j0 < nv; j0 += ts * kElemUnroll) {
    if (j0 != jt) load(j0);
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        if (!first) __builtin_nontemporal_store(xx[u] + alpha * pp[u], reinterpret_cast<V*>(x) + j);
        reinterpret_cast<V*>(p)[j] = first ? zz[u] : (pp[u] * beta) + zz[u];
      }
    }
  }
  for (int64_t i = nv * W + jt; i < n; i += ts) {
    const T pi = p[i];
    if (!first) x[i] = x[i] + alpha * pi;
    p[i] = first ? z[i] : (pi * beta) + z[i];
  }
}

// UR (first chunk loaded before the group sum, as in UP).  ρ_k is read from the state, where UP's
// workgroup 0 stored the value every UP workgroup summed from KB's groups (one scalar load instead
// of a second group sum here; the same bits).
template <typename T>
__global__ void __launch_bounds__(kThreads) k_update_r_g(int64_t n, PcgState* S, const double* __restrict__ gq,
                                                         int ngq, const T* __restrict__ q, T* __restrict__ r) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  const int64_t jt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  V rr[kElemUnroll], qq[kElemUnroll];
  auto load = [&](int64_t j0) {
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        rr[u] = reinterpret_cast<const V*>(r)[j];
        qq[u] = reinterpret_cast<const V*>(q)[j];
      }
    }
  };
  load(jt);  // first chunk, group totals and state line together (as in UP)
  const int32_t done = S->done;
  const int64_t k = S->iter;
  const double rho_prev = S->rho;
  const double rho = S->rho_k;
  double vq[1];
  group_sum_dd<1>(gq, ngq, vq);
  if (done) return;
  const double pq = round_to<T>(vq[0]);
  const T alpha = T(rho) / T(pq);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->rho_prev = rho_prev;
    S->rho = rho;
    S->pq = pq;
    S->alpha = double(alpha);
    S->iter = k + 1;
  }
  for (int64_t j0 = jt; j0 < nv; j0 += ts * kElemUnroll) {
    if (j0 != jt) load(j0);
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) reinterpret_cast<V*>(r)[j] = rr[u] - alpha * qq[u];
    }
  }
  for (int64_t i = nv * W + jt; i < n; i += ts) r[i] = r[i] - alpha * q[i];
}

// UR of the split CG / Jacobi schedule (no preconditioner or the diagonal one): as k_update_r_g --
// α_k = ρ_k/π_k from KC's groups, r_{k+1} = r_k - α_k q -- plus, for the next iteration's UP, the
// groups of ρ_{k+1} = r·z (z = r / d for Jacobi; r·r without a preconditioner) and ‖r_{k+1}‖², the
// dots the ext_spai schedule takes from KB.
template <typename T, int PRE>
__global__ void __launch_bounds__(kThreads) k_update_r_gd(int64_t n, PcgState* S, const double* __restrict__ gq,
                                                          int ngq, const T* __restrict__ q, T* __restrict__ r,
                                                          const T* __restrict__ d, T* __restrict__ z,
                                                          double* partials, unsigned* ticket, int gsz,
                                                          double* __restrict__ gz) {
  using V = typename VecT<T>::type;
  constexpr int W = VecT<T>::W;
  const int64_t nv = n / W;
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  const int64_t jt = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  V rr[kElemUnroll], qq[kElemUnroll];
  auto load = [&](int64_t j0) {
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        rr[u] = reinterpret_cast<const V*>(r)[j];
        qq[u] = reinterpret_cast<const V*>(q)[j];
      }
    }
  };
  load(jt);  // first chunk, group totals and state line together (as in UP)
  const int32_t done = S->done;
  const int64_t k = S->iter;
  const double rho_prev = S->rho;
  const double rho = S->rho_k;
  double vq[1];
  group_sum_dd<1>(gq, ngq, vq);
  if (done) return;  // uniform: UP exits too, nobody reads the groups
  const double pq = round_to<T>(vq[0]);
  const T alpha = T(rho) / T(pq);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->rho_prev = rho_prev;
    S->rho = rho;
    S->pq = pq;
    S->alpha = double(alpha);
    S->iter = k + 1;
  }
  DD dots[2] = {dd_zero(), dd_zero()};  // ρ_{k+1}, ‖r_{k+1}‖²
  auto elem = [&](T ri, int64_t i) {
    dd_fma(dots[1], double(ri), double(ri));
    if constexpr (PRE == LSPCG_PRECOND_DIAGONAL) {
      const T zi = ri / d[i];
      z[i] = zi;
      dd_fma(dots[0], double(ri), double(zi));
    } else {
      dd_fma(dots[0], double(ri), double(ri));
    }
  };
  for (int64_t j0 = jt; j0 < nv; j0 += ts * kElemUnroll) {
    if (j0 != jt) load(j0);
#pragma unroll
    for (int u = 0; u < kElemUnroll; ++u) {
      const int64_t j = j0 + u * ts;
      if (j < nv) {
        const V rn = rr[u] - alpha * qq[u];
        reinterpret_cast<V*>(r)[j] = rn;
#pragma unroll
        for (int c = 0; c < W; ++c) elem(rn[c], j * W + c);
      }
    }
  }
  for (int64_t i = nv * W + jt; i < n; i += ts) {
    const T ri = r[i] - alpha * q[i];
    r[i] = ri;
    elem(ri, i);
  }
  grid_partial_groups<2>(dots, partials, ticket, gsz, gz);
}

// the split CG / Jacobi schedule's first UP reads ρ_0 from the groups: group 0 <- (ρ_0, ‖r_0‖²) of
// the init launch's state, the other groups <- 0 (exact in the dd sums)
__global__ void k_seed_groups(const PcgState* S, double* __restrict__ gz, int ng) {
  for (int i = threadIdx.x; i < 4 * ng; i += blockDim.x) {
    double v = 0.0;
    if (i == 0) v = S->rho;
    if (i == 2) v = S->rr;
    gz[i] = v;
  }
}

// ---- small systems: the whole solve in ONE workgroup --------------------------------------
// Below a few thousand unknowns an iteration of the multi-kernel schedules is 5 dependent
// launches of almost no work (~16 us per iteration at n = 900).  k_pcg_small runs
// scipy's loop (iterative.py:359-418) in one 512-thread workgroup, the phases separated by
// workgroup barriers instead of kernel boundaries.  Thread `tid` owns rows tid + 512 m (m < R):
// their x, r, z, p, q live in registers; the three gathered vectors (r for Lᵀ, t for L, p for A)
// are mirrored in LDS, so a row sum's gathers are LDS reads and its global loads (the row's
// column indices and values, L2-resident after the first iteration) are independent of the
// iteration and issued 8 at a time.  Expressions are those of the split schedule: row sums in
// CSR index order (scipy's csr_matvec), T arithmetic, compensated dots rounded to T, the same
// top-of-loop test and history; x's last update is left to k_x_fixup (x and p are stored at the
// end).  The loop is bounded by max_iter, so every launch ends.
struct CsrView {
  const int32_t* rp;
  const int32_t* ci;
  const void* v;
  int f32;  // values stored as fp32 (compact view of an fp32-exact fp64 matrix, or T = float)
  // the solver's SELL-64 copy of the same view (lspcg_sell.hpp) when gp != nullptr: lane-major
  // 4-entry groups, so a wave's row loads are contiguous 16-B accesses (the CSR row-per-lane
  // loads touch ~12 cache lines per instruction and bound the one-CU solve on L1/L2 requests)
  const int32_t* gp;
  const void* scol;
  const void* sv;
  int sf32;
  int cmode;             // SELL column storage: 0 int32, 1 16-bit offsets
};

constexpr int kSmallThreads = 512;  // 2 waves per SIMD: the compensated reductions are VALU work
constexpr int kSmallThreadsBig = 1024;  // n > 1024: 4 waves per SIMD keep rows per thread <= 3
constexpr int64_t kSmallLds = 61440;  // dynamic LDS: 3 gathered vectors
constexpr int64_t kSmallNDefault = 3072;  // LSPCG_SMALL_N default
constexpr int kSmallQB = 2;  // SELL groups (4 entries each) loaded per wait (4 measured slower: 13.0 vs 9.8 us per iteration)

// row i; [b, e): its CSR entry range, or (SELL) its slice's group range; gx(c) reads the
// gathered vector (LDS in the one-workgroup solve)
template <typename T, int QB, class Gx>
__device__ __forceinline__ T sell_row(const CsrView& M, int32_t b, int32_t e, int32_t i, Gx gx) {
  T acc = T(0);
  if (M.gp) {
    const int32_t lane = i & 63, base = i & ~63;
    for (int32_t q0 = b; q0 < e; q0 += QB) {
      T v[4 * QB];
      int32_t c[4 * QB];
      bool ok[4 * QB];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const size_t off = 256 * size_t(min(q0 + u, e - 1)) + 4 * lane;
        if (M.sf32) {
          const f32x4 a = *(const __attribute__((address_space(1))) f32x4*)(static_cast<const float*>(M.sv) + off);
          v[4 * u + 0] = T(a.x); v[4 * u + 1] = T(a.y); v[4 * u + 2] = T(a.z); v[4 * u + 3] = T(a.w);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * u + j] = gld(static_cast<const T*>(M.sv) + off + j);
        }
        int o[4];
        if (M.cmode == 1) {
          const i16x4 cc = *(const __attribute__((address_space(1))) i16x4*)(static_cast<const int16_t*>(M.scol) + off);
          o[0] = cc.x; o[1] = cc.y; o[2] = cc.z; o[3] = cc.w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ok[4 * u + j] = o[j] != kSellPad16 && q0 + u < e;
            c[4 * u + j] = ok[4 * u + j] ? base + o[j] : i;  // masked slots gather the row's own entry
          }
        } else {
          const i32x4 cc = *(const __attribute__((address_space(1))) i32x4*)(static_cast<const int32_t*>(M.scol) + off);
          o[0] = cc.x; o[1] = cc.y; o[2] = cc.z; o[3] = cc.w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ok[4 * u + j] = o[j] >= 0 && q0 + u < e;
            c[4 * u + j] = ok[4 * u + j] ? o[j] : i;
          }
        }
      }
      T xv[4 * QB];
#pragma unroll
      for (int u = 0; u < 4 * QB; ++u) xv[u] = gx(c[u]);
#pragma unroll
      for (int u = 0; u < 4 * QB; ++u)
        if (ok[u]) acc = acc + v[u] * xv[u];
    }
    return acc;
  }
  for (int32_t k0 = b; k0 < e; k0 += 8) {
    int32_t c[8];
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int32_t k = min(k0 + u, e - 1);
      c[u] = gld(M.ci + k);
      v[u] = M.f32 ? T(gld(static_cast<const float*>(M.v) + k)) : gld(static_cast<const T*>(M.v) + k);
    }
    T xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xv[u] = gx(c[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < e) acc = acc + v[u] * xv[u];
  }
  return acc;
}

// row i (global index) of M with the gathered vector mirrored in LDS from global row `off` on
template <typename T>
__device__ __forceinline__ T small_row(const CsrView& M, int32_t b, int32_t e, int32_t i, const T* xs, int32_t off) {
  return sell_row<T, kSmallQB>(M, b, e, i, [xs, off](int32_t c) { return xs[c - off]; });
}

// fixed-order workgroup sum of N compensated dots, rounded to T, returned to every thread: wave
// butterflies, one barrier, then every wave sums the 8 wave totals with an 8-lane butterfly and
// takes lane 0's (one LDS round trip instead of a serial sum in thread 0 and a broadcast).  `lds`
// is written again only after later barriers (each reduction site has its own buffer).
template <typename T, int N, int TH>
__device__ __forceinline__ void small_dots(DD (&v)[N], DD* lds, double (&out)[N]) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  wave_reduce_dd<N>(v);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) lds[wid * N + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < N; ++j) {
    DD a = lane < TH / 64 ? lds[lane * N + j] : dd_zero();
#pragma unroll
    for (int m = 1; m < TH / 64; m <<= 1) a = dd_add(a, dd_shfl_xor(a, m));
    out[j] = round_to<T>(dd_value(DD{__shfl(a.s, 0, 64), __shfl(a.c, 0, 64)}));
  }
}

// boff / bn (batched solves, lspcg_batch_solve): workgroup k solves system k of a block-diagonal
// window -- rows [boff[k], boff[k] + bn[k]) of the views and vectors, state S[k]; nullptr: the one
// system of n rows.
template <typename T, int PRE, int R, int TH>
__global__ void __launch_bounds__(TH) k_pcg_small(int32_t n, PcgState* S, CsrView A, CsrView L, CsrView LT,
                                                  const T* __restrict__ d, T* x, T* r, T* p,
                                                  const int32_t* __restrict__ boff, const int32_t* __restrict__ bn) {
  constexpr bool SPAI = PRE == LSPCG_PRECOND_EXT_SPAI || PRE == LSPCG_PRECOND_EXT_SPAI_SCALED;
  constexpr bool SCALED = PRE == LSPCG_PRECOND_EXT_SPAI_SCALED;
  int32_t off = 0;
  if (boff) {
    off = boff[blockIdx.x];
    n = bn[blockIdx.x];
    S += blockIdx.x;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char small_lds[];
  T* rs = reinterpret_cast<T*>(small_lds);
  T* ts = rs + n;
  T* ps = ts + n;
  __shared__ DD lds_z[TH / 64 * 2];
  __shared__ DD lds_q[TH / 64];
  if (S->done) return;  // ‖b‖ = 0 (init)
  const int tid = threadIdx.x;
  const T eps = T(S->eps);
  const double atol = S->atol;
  const int64_t max_iter = S->max_iter;
  double* hist = S->hist;
  const double rr0 = S->rr;
  double rho_prev = S->rho, rho = S->rho, pq = S->pq;
  T alpha = T(S->alpha);
  int64_t k = S->iter;
  int code = 0;
  bool own[R];
  int32_t row[R], ab[R], ae[R], lb[R], le[R], tb[R], te[R];
  T xr[R], rr_[R], pr[R], dr[R];
#pragma unroll
  for (int m = 0; m < R; ++m) {
    row[m] = tid + TH * m;
    own[m] = row[m] < n;
    const int32_t i = off + (own[m] ? row[m] : 0);  // global row
    auto range = [&](const CsrView& M, int32_t& b, int32_t& e) {  // CSR entries or SELL groups
      const int32_t* rp = M.gp ? M.gp : M.rp;
      const int32_t j = M.gp ? (i >> 6) : i;
      b = rp[j];
      e = own[m] ? rp[j + 1] : b;
    };
    range(A, ab[m], ae[m]);
    if constexpr (SPAI) {
      range(L, lb[m], le[m]);
      range(LT, tb[m], te[m]);
    }
    xr[m] = own[m] ? x[i] : T(0);
    rr_[m] = own[m] ? r[i] : T(0);
    pr[m] = T(0);
    if constexpr (SCALED || PRE == LSPCG_PRECOND_DIAGONAL) dr[m] = own[m] ? d[i] : T(1);
    if (own[m]) rs[row[m]] = rr_[m];
  }
  __syncthreads();
  for (;; ++k) {
    // z = M⁻¹ r ; ρ_k = r·z ; ‖r_k‖²
    if constexpr (SPAI) {
#pragma unroll
      for (int m = 0; m < R; ++m) {
        if (!own[m]) continue;
        const T s = small_row<T>(LT, tb[m], te[m], off + row[m], rs, off);
        if constexpr (SCALED) ts[row[m]] = s / dr[m];
        else ts[row[m]] = s;
      }
      __syncthreads();
    }
    DD dz[2] = {dd_zero(), dd_zero()};
    T zr[R];
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const T ri = rr_[m];
      T zi;
      if constexpr (SCALED) zi = small_row<T>(L, lb[m], le[m], off + row[m], ts, off) + (eps * ri) / dr[m];
      else if constexpr (SPAI) zi = small_row<T>(L, lb[m], le[m], off + row[m], ts, off) + eps * ri;
      else if constexpr (PRE == LSPCG_PRECOND_DIAGONAL) zi = ri / dr[m];
      else zi = ri;
      zr[m] = zi;
      if (own[m]) {
        dd_fma(dz[0], double(ri), double(zi));
        dd_fma(dz[1], double(ri), double(ri));
      }
    }
    double v2[2];
    small_dots<T, 2, TH>(dz, lds_z, v2);
    const double rr = k > 0 ? v2[1] : rr0;
    if (k >= max_iter) {
      code = 2;
    } else {
      const double rn = double(tsqrt<T>(T(rr)));
      if (rn < atol) code = 1;
      else if (!(rn == rn) || rn == INFINITY) code = 3;
    }
    if (tid == 0 && k > 0) {
      S->rr = rr;
      if (hist) hist[k] = double(tsqrt<T>(T(rr)));
    }
    if (code) break;
    rho_prev = rho;
    rho = v2[0];
    // x += α_{k-1} p_{k-1} ; p_k = p_{k-1}β + z
    const bool first = k == 0;
    const T beta = first ? T(0) : T(rho) / T(rho_prev);
#pragma unroll
    for (int m = 0; m < R; ++m) {
      if (!first) xr[m] = xr[m] + alpha * pr[m];
      pr[m] = first ? zr[m] : (pr[m] * beta) + zr[m];
      if (own[m]) ps[row[m]] = pr[m];
    }
    __syncthreads();
    // q = A p ; π = p·q ; α = ρ/π ; r -= α q
    DD dq[1] = {dd_zero()};
    T qr[R];
#pragma unroll
    for (int m = 0; m < R; ++m) {
      qr[m] = own[m] ? small_row<T>(A, ab[m], ae[m], off + row[m], ps, off) : T(0);
      if (own[m]) dd_fma(dq[0], double(pr[m]), double(qr[m]));
    }
    double v1[1];
    small_dots<T, 1, TH>(dq, lds_q, v1);
    pq = v1[0];
    alpha = T(rho) / T(pq);
#pragma unroll
    for (int m = 0; m < R; ++m) {
      rr_[m] = rr_[m] - alpha * qr[m];
      if (own[m]) rs[row[m]] = rr_[m];
    }
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < R; ++m) {
    if (!own[m]) continue;
    x[off + row[m]] = xr[m];
    p[off + row[m]] = pr[m];
  }
  if (tid == 0) {
    S->rho_prev = rho_prev;
    S->rho = rho;
    S->pq = pq;
    S->alpha = double(alpha);
    S->iter = k;
    S->done = code;
  }
}

// IC: ρ = r·z after the two triangular solves
template <typename T>
__global__ void __launch_bounds__(kThreads) k_dot_rho(int64_t n, PcgState* S, const T* __restrict__ r,
                                                      const T* __restrict__ z, double* partials, unsigned* ticket) {
  if (S->done) return;
  DD dots[1] = {dd_zero()};
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    dd_fma(dots[0], double(r[i]), double(z[i]));
  grid_reduce_dd<1>(dots, partials, ticket, [&](const double* v) {
    S->rho_prev = S->rho;
    S->rho = round_to<T>(v[0]);
  });
}

// ---- OpenBLAS-order dots (lspcg_solver_set_dot_order(s, LSPCG_DOT_OPENBLAS, threads)) --------
// Parity mode: the dots and norms of the loop are recomputed in the summation order of the
// reference's own recorded runs -- numpy's cblas_ddot = OpenBLAS 0.3.29, SkylakeX kernel, split
// over `threads` OpenBLAS threads for n > 10000 (oracle/openblas_ddot.c restates the algorithm and
// cites it): per chunk, 32 FMA accumulators (element i into i % 32) over the 32-aligned prefix,
// folded 8 -> 4 lanes, one 16-element step on 4 x 4 lanes, a fixed lane tree, then a sequential
// FMA tail; chunks summed in order.  One workgroup; each wave owns one (dot, chunk) item at a
// time, lanes 0..31 its accumulators.  The launch follows the reducing launch whose scalars it
// replaces (same predicate on `done`), so the loop's order of state updates is unchanged.
constexpr int kObMaxThreads = 16;
constexpr int kObBlock = 512;  // 8 waves: <= 256 VGPRs for the two register buffers
constexpr int64_t kObSplitN = 131072;  // from this n the parity dots run one workgroup per (dot, chunk)

// chunk c of OpenBLAS's blas_level1_thread split of [0, n) (width = ceil(rest / threads left))
__device__ __forceinline__ void ob_chunk(int64_t n, int nch, int c, int64_t* start, int64_t* width) {
  int64_t m = n, s = 0, w = 0;
  for (int t = 0; t <= c; ++t) {
    w = (m + (nch - t) - 1) / (nch - t);
    m -= w;
    if (m < 0) w += m;
    if (t < c) s += w;
  }
  *start = s;
  *width = w > 0 ? w : 0;
}

// dot_compute(w, x, y) of one chunk (ob_chains, then ob_finish); the result is returned to every
// lane of the wave.  Each accumulator's FMA chain is sequential, so the loads set the time: groups
// of kObU 32-element steps are double-buffered in registers (group g + 1's loads in flight while group g's
// FMAs run; prefetch addresses are clamped instead of branched, so the compiler's in-order vmcnt
// waits never drain the other buffer), and the remainder and tail are loaded at once.  BASELINE
// config 1 (n = 10,240): 8.7 us per launch against 15-16 with flat loads and one 8-step batch
// (~18 GB/s: one wave's loads in flight); a third buffer measured the same, and staging tiles
// through LDS with every wave loading (one barrier per 16-step tile) measured slower (~19 us).
constexpr int kObU = 16;   // steps per register buffer, single-workgroup kernel (8 waves: <= 256 VGPRs)
constexpr int kObU1 = 32;  // the split kernel's one-wave workgroups hold twice as many steps in flight

template <int U>
__device__ __forceinline__ void ob_load(const double* __restrict__ x, const double* __restrict__ y, int64_t i,
                                        double (&xv)[U], double (&yv)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    xv[u] = x[i + 32 * u];
    yv[u] = y[i + 32 * u];
  }
}

template <int U>
__device__ __forceinline__ double ob_fma(const double (&xv)[U], const double (&yv)[U], double acc) {
#pragma unroll
  for (int u = 0; u < U; ++u) acc = __builtin_fma(xv[u], yv[u], acc);
  return acc;
}

// the 32 accumulators over the 32-aligned prefix (lanes 0..31; one wave reads everything)
template <int U = kObU>
__device__ __forceinline__ double ob_chains(const double* __restrict__ x, const double* __restrict__ y, int64_t w) {
  const int lane = threadIdx.x & 63;
  const int64_t n32 = (w & -int64_t(16)) & ~int64_t(31);
  double acc = 0.0;
  if (lane < 32) {
    constexpr int64_t GW = 32 * U;  // elements per group
    const int64_t G = n32 / GW;
    double ax[U], ay[U], bx[U], by[U];
    int64_t g = 0;
    if (G > 0) ob_load<U>(x, y, lane, ax, ay);
    for (; g + 1 < G; g += 2) {
      ob_load<U>(x, y, (g + 1) * GW + lane, bx, by);
      acc = ob_fma<U>(ax, ay, acc);
      ob_load<U>(x, y, (g + 2 < G ? g + 2 : g + 1) * GW + lane, ax, ay);
      acc = ob_fma<U>(bx, by, acc);
    }
    if (g < G) acc = ob_fma<U>(ax, ay, acc);
    // the remaining < U steps, loaded at once and added in order
    const int64_t base = G * GW;
    const int rem = int((n32 - base) >> 5);
    if (rem > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + (u < rem ? 32 * u : 0) + lane;
        bx[u] = x[i];
        by[u] = y[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < rem) acc = __builtin_fma(bx[u], by[u], acc);
    }
  }
  return acc;
}

// fold, 16-element step, lane tree and sequential tail of one chunk from its accumulators
__device__ __forceinline__ double ob_finish(const double* __restrict__ x, const double* __restrict__ y, int64_t w,
                                            double acc) {
  const int lane = threadIdx.x & 63;
  const int64_t n1 = w & -int64_t(16);
  const int64_t n32 = n1 & ~int64_t(31);
  // fold the 512-bit accumulators: lane 8v + j (j < 4) <- acc[8v + j] + acc[8v + 4 + j]
  double a = acc + __shfl_down(acc, 4, 64);
  if (n1 > n32 && lane < 32 && (lane & 7) < 4) {
    const int64_t e = n32 + 4 * (lane >> 3) + (lane & 3);
    a = __builtin_fma(x[e], y[e], a);
  }
  const int j = lane & 3;
  const double s = ((__shfl(a, j, 64) + __shfl(a, 8 + j, 64)) + __shfl(a, 16 + j, 64)) + __shfl(a, 24 + j, 64);
  double dot = (__shfl(s, 0, 64) + __shfl(s, 2, 64)) + (__shfl(s, 1, 64) + __shfl(s, 3, 64));
  // sequential tail of < 16 elements, loaded at once
  const int nt = int(w - n1);
  double tx = 0.0, ty = 0.0;
  if (lane < nt) {
    tx = x[n1 + lane];
    ty = y[n1 + lane];
  }
  for (int t = 0; t < nt; ++t) dot = __builtin_fma(__shfl(ty, t, 64), __shfl(tx, t, 64), dot);
  return dot;
}

template <int U = kObU>
__device__ __forceinline__ double ob_chunk_dot(const double* __restrict__ x, const double* __restrict__ y, int64_t w) {
  return ob_finish(x, y, w, ob_chains<U>(x, y, w));
}

enum ObWhich { kObInit = 0, kObZ = 1, kObQ = 2, kObR = 3, kObRho = 4, kObRR = 5 };

// up to 3 dots (xs[j] · ys[j]); thread 0 then writes the scalars of phase WHICH:
//   kObInit  rr = r·r, bb = b·b, atol, rho = (DIAG ? r·z : rr), done (‖b‖ = 0), hist[0]
//   kObZ     rho = r·z ; rr = r·r and hist[k] for k > 0           (after KB's EpiZ)
//   kObQ     pq = p·q ; alpha = rho / pq                           (after KC's EpiQ)
//   kObR     rr = r·r ; rho = (DIAG ? r·z : rr) ; hist[k]           (after CG / Jacobi k_update_r)
//   kObRho   rho = r·z                                             (after IC's k_dot_rho)
//   kObRR    rr = r·r ; hist[k]                                    (after IC's k_update_r)
// thread 0's scalar update of phase WHICH from the dot values v[0..nd)
template <int WHICH, bool DIAG>
__device__ __forceinline__ void ob_epilogue(PcgState* S, const double (&v)[3]) {
  const int64_t k = S->iter;
  if constexpr (WHICH == kObInit) {
    S->rr = v[0];
    S->bb = v[1];
    const double bn = sqrt(v[1]);
    S->atol = fmax(0.0, S->rtol * bn);
    S->rho = DIAG ? v[2] : v[0];
    S->done = (bn == 0.0) ? 1 : 0;
    if (S->hist) S->hist[0] = sqrt(v[0]);
  } else if constexpr (WHICH == kObZ) {
    S->rho = v[0];
    if (k > 0) {
      S->rr = v[1];
      if (S->hist) S->hist[k] = sqrt(v[1]);
    }
  } else if constexpr (WHICH == kObQ) {
    S->pq = v[0];
    S->alpha = S->rho / v[0];
  } else if constexpr (WHICH == kObR) {
    S->rr = v[0];
    S->rho = DIAG ? v[1] : v[0];
    if (S->hist) S->hist[k] = sqrt(v[0]);
  } else if constexpr (WHICH == kObRho) {
    S->rho = v[0];
  } else {
    S->rr = v[0];
    if (S->hist) S->hist[k] = sqrt(v[0]);
  }
}

// the chunk totals of dot j summed in chunk order (numpy's threads joined in order)
__device__ __forceinline__ void ob_join(const double* part, int nd, int ch, double (&v)[3]) {
  for (int j = 0; j < 3; ++j) v[j] = 0.0;
  for (int j = 0; j < nd; ++j) {
    double d = 0.0;
    for (int c = 0; c < ch; ++c) d = d + part[j * kObMaxThreads + c];
    v[j] = ch > 1 ? d : part[j * kObMaxThreads];
  }
}

template <int WHICH, bool DIAG>
__global__ void __launch_bounds__(kObBlock) k_dot_openblas(int64_t n, int nch, int nd, PcgState* S, const double* x0,
                                                           const double* y0, const double* x1, const double* y1,
                                                           const double* x2, const double* y2) {
  __shared__ double part[3 * kObMaxThreads];
  if (WHICH != kObInit && S->done) return;
  const int ch = (n > 10000 && nch > 1) ? nch : 1;
  const int nw = blockDim.x >> 6;
  for (int item = threadIdx.x >> 6; item < nd * ch; item += nw) {
    const int j = item / ch, c = item % ch;
    int64_t s = 0, w = n;
    if (ch > 1) ob_chunk(n, ch, c, &s, &w);
    // selects, not an array of pointers: the loads stay global_load (a flat load's lgkmcnt forces
    // waits on ALL outstanding loads, which would serialise the two register buffers)
    const double* xj = j == 0 ? x0 : j == 1 ? x1 : x2;
    const double* yj = j == 0 ? y0 : j == 1 ? y1 : y2;
    const double v = ob_chunk_dot(xj + s, yj + s, w);
    if ((threadIdx.x & 63) == 0) part[j * kObMaxThreads + c] = v;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double v[3];
  ob_join(part, nd, ch, v);
  ob_epilogue<WHICH, DIAG>(S, v);
}

// Large n (>= kObSplitN): one single-wave workgroup per (dot, chunk) item -- every chunk of every
// dot on its own CU, with twice the steps in flight per register buffer (kObU1) -- writing its
// chunk total to a scratch slot; k_dot_openblas_fin then joins them in order and updates the
// scalars (one more launch; the same bits).  (Feeding the chains from an LDS ring filled by 7
// producer waves measured slower: kuhn101 parity solve 591 vs 272 ms at 1 thread, 91 vs 50 ms at 8
// -- the LDS hand-off per 64-step tile costs more than the loads it hides)
template <int WHICH>
__global__ void __launch_bounds__(64) k_dot_openblas_item(int64_t n, int nch, const PcgState* S, double* part,
                                                          const double* x0, const double* y0, const double* x1,
                                                          const double* y1, const double* x2, const double* y2) {
  if (WHICH != kObInit && S->done) return;
  const int ch = (n > 10000 && nch > 1) ? nch : 1;
  const int j = int(blockIdx.x) / ch, c = int(blockIdx.x) % ch;
  int64_t s = 0, w = n;
  if (ch > 1) ob_chunk(n, ch, c, &s, &w);
  const double* xj = j == 0 ? x0 : j == 1 ? x1 : x2;
  const double* yj = j == 0 ? y0 : j == 1 ? y1 : y2;
  const double v = ob_chunk_dot<kObU1>(xj + s, yj + s, w);
  if (threadIdx.x == 0) part[j * kObMaxThreads + c] = v;
}

template <int WHICH, bool DIAG>
__global__ void k_dot_openblas_fin(int64_t n, int nch, int nd, PcgState* S, const double* part) {
  if (threadIdx.x != 0 || (WHICH != kObInit && S->done)) return;
  const int ch = (n > 10000 && nch > 1) ? nch : 1;
  double v[3];
  ob_join(part, nd, ch, v);
  ob_epilogue<WHICH, DIAG>(S, v);
}

// after the loop: the deferred x += α_{k-1} p_{k-1} of the last completed iteration
template <typename T>
__global__ void __launch_bounds__(kThreads) k_x_fixup(int64_t n, const PcgState* S, const T* __restrict__ p,
                                                      T* __restrict__ x) {
  if (S->iter < 1 || S->bb == 0.0) return;
  const T alpha = T(S->alpha);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    x[i] = x[i] + alpha * p[i];
}

// ---- storage optimisation helpers (see DESIGN.md "PCG storage")
__global__ void k_f32_inexact(int64_t n, const double* __restrict__ v, int* __restrict__ flag) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const double a = v[i];
    if (!(double(float(a)) == a)) atomicOr(flag, 1);  // also true for NaN
  }
}
__global__ void k_to_f32(int64_t n, const double* __restrict__ v, float* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = float(v[i]);
}
__global__ void k_i32_neq(int64_t n, const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                          int* __restrict__ flag) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    if (a[i] != b[i]) atomicOr(flag, 2);
}

static int elem_grid(int64_t n) {  // 2 elements per lane, >= 2 pairs per lane, <= 1024 partials
  const int64_t g = (n + kThreads * 4 - 1) / (kThreads * 4);
  return int(std::max<int64_t>(1, std::min<int64_t>(g, 1024)));
}

}  // namespace lspcg

using namespace lspcg;

struct lspcg_solver {
  lspcg_ctx* ctx = nullptr;
  const lspcg_mat* A = nullptr;       // the system the loop runs on: A_user, or Ap when reordered
  const lspcg_mat* A_user = nullptr;  // the caller's A
  const lspcg_mat* L = nullptr;       // the caller's L (ext_spai)
  lspcg_mat* LT = nullptr;  // owned (the permuted Lᵀ when reordered)
  // bandwidth-reducing row placement (lspcg_reorder.hip): A, L, Lᵀ permuted with each row's
  // entries in their original order, vectors gathered in / scattered out around the loop
  Reorder ro;
  lspcg_mat* Ap = nullptr;   // owned P A Pᵀ
  lspcg_mat* Lp = nullptr;   // owned P L Pᵀ
  lspcg_mat* LTo = nullptr;  // owned Lᵀ in the original numbering (reordered ext_spai; kept for reuse)
  int reorder_mode = -1;     // LSPCG_REORDER: -1 auto, 0 off, 1 always
  bool reorder_ok = false;   // single solves in the compensated order only (not batches, IC, parity)
  int precond = LSPCG_PRECOND_NONE;
  int dtype = LSPCG_F64;
  int64_t n = 0;
  double eps = 0.0;
  hipStream_t stream = nullptr;  // solver-owned (capturable) stream
  void *x = nullptr, *b = nullptr, *r = nullptr, *z = nullptr, *t = nullptr, *p = nullptr, *q = nullptr,
       *d = nullptr;
  bool split = false;   // current ext_spai schedule uses the split reductions (set_spai decides)
  bool allow_split = true;  // LSPCG_SPLIT_REDUCE=0 keeps the last-arriver reductions
  int split_mode = -1;  // -1 auto (by grid size), 1 groups, 2 no groups (LSPCG_SPLIT_REDUCE)
  double* groups = nullptr;  // [GZ: <= 4096 x 2 dots x DD | GQ: <= 4096 x DD]
  int gsz_l = 1, ng_l = 1, gsz_a = 1, ng_a = 1;  // group size / count of the KB and KC launches
  bool split_cg = false;  // CG / Jacobi on the split reductions (UP, KC, UR with the dots of ρ, ‖r‖²)
  int gsz_r = 1, ng_r = 1;  // ... group size / count of that UR launch
  KernelTimer* tk = nullptr;  // lspcg_solver_time_kernels: start / end stamps armed for each launch
  int tk_i = 0;
  PcgState* S = nullptr;
  PcgState* hS = nullptr;  // pinned host mirrors [2] (poll slots)
  double* partials = nullptr;
  unsigned* ticket = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_t0 = nullptr, ev_t1 = nullptr, ev_poll = nullptr, ev_poll2 = nullptr;
  std::map<int, hipGraphExec_t> graphs;
  std::map<int, hipGraph_t> graph_defs;
  // iteration views of A, L, Lᵀ: compact fp32 values when lossless, one shared index
  // structure when the patterns coincide (non-owning copies of the handles + owned buffers)
  lspcg_mat Av, Lv, LTv;
  void* own_A = nullptr;
  void* own_L = nullptr;
  void* own_LT = nullptr;
  int64_t own_L_n = -1, own_LT_n = -1;  // entries of the fp32 copies above (refilled in place)
  int* flag = nullptr;
  // IC(0): factor, its explicit transpose and their level sets
  lspcg_mat* icL = nullptr;
  lspcg_mat* icU = nullptr;
  Levels levL, levU;
  // SELL-64 copies of the scalar iteration views A (0), L (1), Lᵀ (2) (lspcg_sell.hpp); sp[w]
  // is null where the CSR kernel is used (block size 3, irregular rows, LSPCG_NO_SELL=1)
  bool use_sell = true;
  SellPattern spat[3];
  const SellPattern* sp[3] = {nullptr, nullptr, nullptr};
  void* sv[3] = {nullptr, nullptr, nullptr};
  int svd[3] = {0, 0, 0};  // storage of sv[w]: LSPCG_F32 / LSPCG_F64
  int64_t svn[3] = {0, 0, 0};  // entries sv[w] was allocated for (an in-place refill must fit them)
  double* dhist = nullptr;  // device residual history (lspcg_solver_solve with res_hist), grown on demand
  double* hhist = nullptr;  // its pinned host mirror (the history's copy is enqueued, not a blocking copy)
  int64_t dhist_cap = 0;
  unsigned* hflags = nullptr;  // pinned: the IC triangular solves' timeout flags, copied behind the solve
  int64_t small_n = kSmallNDefault;  // largest n solved by k_pcg_small (LSPCG_SMALL_N; 0 disables it; also bounded by
                           // 3 rows per thread at 1024 threads and the LDS of 3 vectors: 2560 in fp64)
  bool small_sell = true;  // k_pcg_small reads the SELL copies (LSPCG_SMALL_SELL=0: the CSR views)
  bool split_ok = false;   // set_spai found SELL views for the split schedule
  bool dia_ok = true;      // SELL-DIA views allowed (a batch of one-workgroup solves turns them off)
  int dot_order = LSPCG_DOT_COMPENSATED;  // lspcg_solver_set_dot_order
  int dot_threads = 1;
  double* ob_part = nullptr;  // [3 dots x kObMaxThreads chunks] parity-mode chunk totals (k_dot_openblas_item)
};

// parity mode: every reducing launch is followed by k_dot_openblas, which rewrites its scalars
template <int WHICH, bool DIAG = false>
static void enqueue_ob(lspcg_solver* s, hipStream_t st, int nd, const void* x0, const void* y0,
                       const void* x1 = nullptr, const void* y1 = nullptr, const void* x2 = nullptr,
                       const void* y2 = nullptr) {
  if (s->dot_order != LSPCG_DOT_OPENBLAS) return;
  const int ch = (s->n > 10000 && s->dot_threads > 1) ? s->dot_threads : 1;
  const auto* X0 = static_cast<const double*>(x0);
  const auto* Y0 = static_cast<const double*>(y0);
  const auto* X1 = static_cast<const double*>(x1);
  const auto* Y1 = static_cast<const double*>(y1);
  const auto* X2 = static_cast<const double*>(x2);
  const auto* Y2 = static_cast<const double*>(y2);
  if (s->n >= kObSplitN) {  // large n: one CU per (dot, chunk), then the ordered join
    hipLaunchKernelGGL(k_dot_openblas_item<WHICH>, dim3(nd * ch), dim3(64), 0, st, s->n, s->dot_threads, s->S,
                       s->ob_part, X0, Y0, X1, Y1, X2, Y2);
    hipLaunchKernelGGL((k_dot_openblas_fin<WHICH, DIAG>), dim3(1), dim3(64), 0, st, s->n, s->dot_threads, nd, s->S,
                       static_cast<const double*>(s->ob_part));
    return;
  }
  const int waves = std::min(kObBlock / 64, std::max(1, nd * ch));
  hipLaunchKernelGGL((k_dot_openblas<WHICH, DIAG>), dim3(1), dim3(64 * waves), 0, st, s->n, s->dot_threads, nd, s->S,
                     X0, Y0, X1, Y1, X2, Y2);
}

// (Re)build the SELL copy of iteration view w (0 = A, 1 = L, 2 = Lᵀ); L and Lᵀ reuse A's
// pattern when make_view found the same index arrays.
static int build_sell_bsr3(lspcg_solver* s, int w, const lspcg_mat* view);

static int build_sell(lspcg_solver* s, int w, const lspcg_mat* view) {
  hipStream_t st = s->ctx->stream;
  if (s->sv[w] || s->spat[w].gp) LSPCG_HIP(hipStreamSynchronize(s->stream));  // a solve may use them
  // L / Lᵀ on A's pattern again (a new L for the same system): refill the value array in place, so
  // its address -- and with it every captured iteration graph -- stays valid (get_graph)
  // (the pattern may have been rebuilt at the same host address -- set_dot_order's switch back to the
  // unpermuted A -- so the array's entry count must match the pattern's, not just the pointers)
  if (w > 0 && s->use_sell && s->sv[w] && s->sp[w] && s->sp[w] == s->sp[0] &&
      view->rowptr == s->Av.rowptr && view->colind == s->Av.colind && view->storage_dtype() == s->svd[w] &&
      s->svn[w] == s->sp[w]->slots()) {
    const SellPattern* P = s->sp[w];
    const int vd = view->storage_dtype();
    return P->bs == 3 ? bsell_fill_values(*P, view->vals, vd, vd, st, &s->sv[w])
                      : sell_fill_values(*P, view->colind, view->vals, vd, vd, st, &s->sv[w]);
  }
  (void)hipFree(s->sv[w]);
  s->sv[w] = nullptr;
  s->spat[w].release();
  s->sp[w] = nullptr;
  if (!s->use_sell || view->n == 0 || view->nnzb == 0) return LSPCG_OK;
  if (view->block_size == 3) return build_sell_bsr3(s, w, view);
  if (view->block_size != 1) return LSPCG_OK;
  const SellPattern* P = nullptr;
  if (w > 0 && s->sp[0] && view->rowptr == s->Av.rowptr && view->colind == s->Av.colind) {
    P = s->sp[0];
  } else {
    // SELL-DIA except for systems the one-workgroup solve takes (its per-thread rows load 4-entry
    // groups with one 16-B load; slot-by-slot loads measured 16.0 vs 9.8 us per iteration at n = 900)
    const bool dia = s->dia_ok && view->n > std::min<int64_t>(s->small_n, int64_t(kSmallThreadsBig) * 3);
    const int rc = sell_build_pattern(view->n, view->nnzb, view->rowptr, view->colind, sell_max_pad(),
                                      kSellCol16 | (dia ? kSellColDia | kSellColJag | kSellColXs : 0) |
                                          (dia && sellc_allowed(view->n) ? kSellColCode : 0),
                                      st, &s->spat[w]);
    if (rc == LSPCG_ERR_UNSUPPORTED) return LSPCG_OK;  // padding too large: CSR kernel
    if (rc) return rc;
    P = &s->spat[w];
  }
  const int vd = view->storage_dtype();
  if (int rc = sell_fill_values(*P, view->colind, view->vals, vd, vd, st, &s->sv[w])) return rc;
  s->svd[w] = vd;
  s->svn[w] = P->slots();
  s->sp[w] = P;
  return LSPCG_OK;
}

// BSR 3x3 views: the BSELL-64 block layout (lspcg_sell.hpp), pattern shared with A's when the
// index arrays are A's, values in the view's storage dtype (fp32 when lossless)
static int build_sell_bsr3(lspcg_solver* s, int w, const lspcg_mat* view) {
  hipStream_t st = s->ctx->stream;
  const bool shared = w > 0 && s->sp[0] && view->rowptr == s->Av.rowptr && view->colind == s->Av.colind;
  const SellPattern* P = nullptr;
  if (shared) {
    P = s->sp[0];
  } else {
    const int rc = bsell_build_pattern(view->nb, view->nnzb, view->rowptr, view->colind, sell_max_pad(), true,
                                       s->dia_ok && bsdia_allowed(), st, &s->spat[w]);
    if (rc == LSPCG_ERR_UNSUPPORTED) return LSPCG_OK;  // padding too large: the staged block kernel
    if (rc) return rc;
    P = &s->spat[w];
  }
  const int vd = view->storage_dtype();
  if (int rc = bsell_fill_values(*P, view->vals, vd, vd, st, &s->sv[w])) return rc;
  s->svd[w] = vd;
  s->svn[w] = P->slots();
  s->sp[w] = P;
  return LSPCG_OK;
}

// SpMV of iteration view w with the fused prologue / gather / epilogue, SELL when available.
template <typename T, class Gx, class Pro, class Epi>
static int launch_it_gx(lspcg_solver* s, int w, Gx gx, Pro pro, Epi epi, hipStream_t st) {
  if (const SellPattern* P = s->sp[w]) {
    if constexpr (sizeof(T) == 8) {
      if (s->svd[w] == LSPCG_F32) {
        launch_spmv_sell_cfg<T, float>(*P, s->sv[w], gx, pro, epi, st);
        return LSPCG_OK;
      }
    }
    launch_spmv_sell_cfg<T, T>(*P, s->sv[w], gx, pro, epi, st);
    return LSPCG_OK;
  }
  const lspcg_mat* V = w == 0 ? &s->Av : (w == 1 ? &s->Lv : &s->LTv);
  return launch_spmv_gx<T>(V, gx, pro, epi, st);
}

template <typename T, class Pro, class Epi>
static int launch_it(lspcg_solver* s, int w, const T* x, Pro pro, Epi epi, hipStream_t st) {
  return launch_it_gx<T>(s, w, GatherVec<T>{x}, pro, epi, st);
}

static int flag_run(lspcg_solver* s, hipStream_t st, int* out) {
  int h = 0;
  LSPCG_HIP(hipMemcpyAsync(&h, s->flag, sizeof(int), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  *out = h;
  return LSPCG_OK;
}

// view <- M; compact fp64 values to fp32 when exact; share `base`'s index arrays when equal.
// Both checks run before ONE host read of the flag (bit 0: some value not fp32-exact, bit 1:
// index arrays differ).  `known` (optional) supplies that flag instead -- Lᵀ from the
// symmetric-pattern transpose has L's pattern and a permutation of L's values.  Returns the
// flag in *flag_out (optional).
static int make_view(lspcg_solver* s, const lspcg_mat* M, lspcg_mat* view, const lspcg_mat* base, void** own,
                     const int* known = nullptr, int* flag_out = nullptr, int64_t* own_n = nullptr) {
  hipStream_t st = s->ctx->stream;
  const int64_t ne = M->nnzb * M->block_size * M->block_size;
  if (*own) {
    LSPCG_HIP(hipStreamSynchronize(s->stream));
    if (!own_n || *own_n != ne) {  // an fp32 copy of the same length is refilled in place below
      (void)hipFree(*own);
      *own = nullptr;
    }
  }
  *view = *M;
  const bool try_compact = M->dtype == LSPCG_F64 && M->storage_dtype() == LSPCG_F64 && ne > 0;
  const bool try_share = base && base != M && base->nb == M->nb && base->nnzb == M->nnzb &&
                         base->block_size == M->block_size;
  int f = 3;
  if (known) {
    f = *known;
  } else if (try_compact || try_share) {
    LSPCG_HIP(hipMemsetAsync(s->flag, 0, sizeof(int), st));
    if (try_compact)
      hipLaunchKernelGGL(k_f32_inexact, dim3(elem_grid(ne)), dim3(kThreads), 0, st, ne,
                         static_cast<const double*>(M->vals), s->flag);
    if (try_share) {
      hipLaunchKernelGGL(k_i32_neq, dim3(elem_grid(M->nb + 1)), dim3(kThreads), 0, st, M->nb + 1, M->rowptr,
                         base->rowptr, s->flag);
      if (M->nnzb)
        hipLaunchKernelGGL(k_i32_neq, dim3(elem_grid(M->nnzb)), dim3(kThreads), 0, st, M->nnzb, M->colind,
                           base->colind, s->flag);
    }
    if (int rc = flag_run(s, st, &f)) return rc;
    if (!try_compact) f |= 1;
    if (!try_share) f |= 2;
  }
  if (flag_out) *flag_out = f;
  if (*own && !(try_compact && !(f & 1))) {  // the new matrix is not stored compactly
    (void)hipFree(*own);
    *own = nullptr;
  }
  if (try_compact && !(f & 1)) {
    float* v = static_cast<float*>(*own);
    if (!v) {
      LSPCG_HIP(hipMalloc(&v, sizeof(float) * (ne + kEntryPad)));
      *own = v;
      if (own_n) *own_n = ne;
      LSPCG_HIP(hipMemsetAsync(v + ne, 0, sizeof(float) * kEntryPad, st));
    }
    hipLaunchKernelGGL(k_to_f32, dim3(elem_grid(ne)), dim3(kThreads), 0, st, ne, static_cast<const double*>(M->vals), v);
    view->vals = v;
    view->val_dtype = LSPCG_F32;
  }
  if (try_share && !(f & 2)) {
    view->rowptr = base->rowptr;
    view->colind = base->colind;
  }
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

// lspcg_solver_time_kernels only: record the next timing event behind the launch just enqueued
// lspcg_solver_time_kernels: the next launch is stamped with its own start / end events
static void arm(lspcg_solver* s) {
  if (s->tk) kernel_timer() = &s->tk[s->tk_i++];
}

template <typename T, bool SC>
static int enqueue_iteration_split(lspcg_solver* s, hipStream_t st) {
  const int64_t n = s->n;
  PcgState* S = s->S;
  T* x = static_cast<T*>(s->x);
  T* r = static_cast<T*>(s->r);
  T* z = static_cast<T*>(s->z);
  T* t = static_cast<T*>(s->t);
  T* p = static_cast<T*>(s->p);
  T* q = static_cast<T*>(s->q);
  const T* d = static_cast<const T*>(s->d);
  double* gz = s->groups;
  double* gq = s->groups + 4096 * 2 * 2;
  const int eg = elem_vec_grid<T>(n);
  arm(s);
  int rc = launch_it<T>(s, 2, static_cast<const T*>(r), ProDone{S}, EpiT<T, SC>{t, d}, st);
  if (rc) return rc;
  arm(s);
  rc = launch_it<T>(s, 1, static_cast<const T*>(t), ProDone{S},
                    EpiZG<T, SC>{z, r, d, T(s->eps), s->partials, s->ticket, gz, s->gsz_l}, st);
  if (rc) return rc;
  arm(s);
  LSPCG_LAUNCH_SPMV(k_update_p_g<T>, dim3(eg), dim3(kThreads), 0, st, n, S, static_cast<const double*>(gz), s->ng_l,
                    static_cast<const T*>(z), p, x);
  arm(s);
  rc = launch_it<T>(s, 0, static_cast<const T*>(p), ProDone{S}, EpiQG<T>{q, p, s->partials, s->ticket, gq, s->gsz_a},
                    st);
  if (rc) return rc;
  arm(s);
  LSPCG_LAUNCH_SPMV(k_update_r_g<T>, dim3(eg), dim3(kThreads), 0, st, n, S, static_cast<const double*>(gq), s->ng_a,
                    static_cast<const T*>(q), r);
  kernel_timer() = nullptr;
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

template <typename T>
static int enqueue_iteration(lspcg_solver* s, hipStream_t st) {
  if (s->split)
    return s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED ? enqueue_iteration_split<T, true>(s, st)
                                                       : enqueue_iteration_split<T, false>(s, st);
  const int64_t n = s->n;
  T* x = static_cast<T*>(s->x);
  T* r = static_cast<T*>(s->r);
  T* z = static_cast<T*>(s->z);
  T* t = static_cast<T*>(s->t);
  T* p = static_cast<T*>(s->p);
  T* q = static_cast<T*>(s->q);
  const T* d = static_cast<const T*>(s->d);
  PcgState* S = s->S;
  const int eg = elem_vec_grid<T>(n);
  int rc = LSPCG_OK;
  if (s->split_cg) {  // UP (ρ_k, ‖r_k‖² from UR's groups) -> KC (π groups) -> UR (+ next dots' groups)
    double* gz = s->groups;
    double* gq = s->groups + 4096 * 2 * 2;
    const bool jac = s->precond == LSPCG_PRECOND_DIAGONAL;
    hipLaunchKernelGGL(k_update_p_g<T>, dim3(eg), dim3(kThreads), 0, st, n, S, static_cast<const double*>(gz), s->ng_r,
                       static_cast<const T*>(jac ? z : r), p, x);
    rc = launch_it<T>(s, 0, static_cast<const T*>(p), ProDone{S}, EpiQG<T>{q, p, s->partials, s->ticket, gq, s->gsz_a},
                      st);
    if (rc) return rc;
    if (jac)
      hipLaunchKernelGGL((k_update_r_gd<T, LSPCG_PRECOND_DIAGONAL>), dim3(eg), dim3(kThreads), 0, st, n, S,
                         static_cast<const double*>(gq), s->ng_a, static_cast<const T*>(q), r, d, z, s->partials,
                         s->ticket, s->gsz_r, gz);
    else
      hipLaunchKernelGGL((k_update_r_gd<T, LSPCG_PRECOND_NONE>), dim3(eg), dim3(kThreads), 0, st, n, S,
                         static_cast<const double*>(gq), s->ng_a, static_cast<const T*>(q), r, d, z, s->partials,
                         s->ticket, s->gsz_r, gz);
    LSPCG_HIP(hipGetLastError());
    return LSPCG_OK;
  }
  switch (s->precond) {
    case LSPCG_PRECOND_EXT_SPAI:
    case LSPCG_PRECOND_EXT_SPAI_SCALED: {
      const bool sc = s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED;
      rc = sc ? launch_it<T>(s, 2, static_cast<const T*>(r), ProDone{S}, EpiT<T, true>{t, d}, st)
              : launch_it<T>(s, 2, static_cast<const T*>(r), ProDone{S}, EpiT<T, false>{t, d}, st);
      if (rc) return rc;
      rc = sc ? launch_it<T>(s, 1, static_cast<const T*>(t), ProDone{S},
                                   EpiZ<T, true>{z, r, d, T(s->eps), S, s->partials, s->ticket}, st)
              : launch_it<T>(s, 1, static_cast<const T*>(t), ProDone{S},
                                   EpiZ<T, false>{z, r, d, T(s->eps), S, s->partials, s->ticket}, st);
      if (rc) return rc;
      enqueue_ob<kObZ>(s, st, 2, r, z, r, r);
      // top-of-loop test on ‖r_k‖ (reduced by KB) before the first update of iteration k
      hipLaunchKernelGGL((k_update_p<T, ProCheck<T>>), dim3(eg), dim3(kThreads), 0, st, n, ProCheck<T>{S}, S,
                         static_cast<const T*>(z), p, x);
      break;
    }
    case LSPCG_PRECOND_NONE:
    case LSPCG_PRECOND_DIAGONAL:
      hipLaunchKernelGGL((k_update_p<T, ProCheck<T>>), dim3(eg), dim3(kThreads), 0, st, n, ProCheck<T>{S}, S,
                         static_cast<const T*>(s->precond == LSPCG_PRECOND_NONE ? r : z), p, x);
      break;
    case LSPCG_PRECOND_IC: {
      // z = L⁻ᵀ L⁻¹ r (t holds L⁻¹ r), ρ = r·z; then the top-of-loop test in the p update
      const int32_t* done = &S->done;
      if ((rc = enqueue_trsv(s->icL, s->levL, true, r, t, done, st))) return rc;
      if ((rc = enqueue_trsv(s->icU, s->levU, false, t, z, done, st))) return rc;
      hipLaunchKernelGGL(k_dot_rho<T>, dim3(eg), dim3(kThreads), 0, st, n, S, static_cast<const T*>(r),
                         static_cast<const T*>(z), s->partials, s->ticket);
      enqueue_ob<kObRho>(s, st, 1, r, z);
      hipLaunchKernelGGL((k_update_p<T, ProCheck<T>>), dim3(eg), dim3(kThreads), 0, st, n, ProCheck<T>{S}, S,
                         static_cast<const T*>(z), p, x);
      break;
    }
    default:
      set_error("unknown preconditioner");
      return LSPCG_ERR_ARG;
  }
  const bool spai = s->precond == LSPCG_PRECOND_EXT_SPAI || s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED;
  rc = spai ? launch_it<T>(s, 0, static_cast<const T*>(p), ProDone{S}, EpiQ<T, true>{q, p, S, s->partials, s->ticket},
                           st)
            : launch_it<T>(s, 0, static_cast<const T*>(p), ProDone{S}, EpiQ<T>{q, p, S, s->partials, s->ticket}, st);
  if (rc) return rc;
  enqueue_ob<kObQ>(s, st, 1, p, q);
  switch (s->precond) {
    case LSPCG_PRECOND_EXT_SPAI:
    case LSPCG_PRECOND_EXT_SPAI_SCALED:
      hipLaunchKernelGGL(k_update_r_nodot<T>, dim3(eg), dim3(kThreads), 0, st, n, S, static_cast<const T*>(q), r);
      break;
    case LSPCG_PRECOND_NONE:
      hipLaunchKernelGGL((k_update_r<T, LSPCG_PRECOND_NONE>), dim3(eg), dim3(kThreads), 0, st, n, S, q, r, d, z,
                         s->partials, s->ticket);
      enqueue_ob<kObR>(s, st, 1, r, r);
      break;
    case LSPCG_PRECOND_DIAGONAL:
      hipLaunchKernelGGL((k_update_r<T, LSPCG_PRECOND_DIAGONAL>), dim3(eg), dim3(kThreads), 0, st, n, S, q, r, d, z,
                         s->partials, s->ticket);
      enqueue_ob<kObR, true>(s, st, 2, r, r, r, z);
      break;
    default:  // IC
      hipLaunchKernelGGL((k_update_r<T, LSPCG_PRECOND_EXT_SPAI>), dim3(eg), dim3(kThreads), 0, st, n, S, q, r, d, z,
                         s->partials, s->ticket);
      enqueue_ob<kObRR>(s, st, 1, r, r);
  }
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

template <typename T>
static int enqueue_init(lspcg_solver* s, hipStream_t st) {
  T* r = static_cast<T*>(s->r);
  const T* b = static_cast<const T*>(s->b);
  const T* d = static_cast<const T*>(s->d);
  T* z = static_cast<T*>(s->z);
  const T* x = static_cast<const T*>(s->x);
  const int rc = s->precond == LSPCG_PRECOND_DIAGONAL
                     ? launch_it<T>(s, 0, x, ProNone{},
                                          EpiResid<T, LSPCG_PRECOND_DIAGONAL>{r, b, d, z, s->S, s->partials, s->ticket},
                                          st)
                     : launch_it<T>(s, 0, x, ProNone{},
                                          EpiResid<T, LSPCG_PRECOND_NONE>{r, b, d, z, s->S, s->partials, s->ticket},
                                          st);
  if (rc) return rc;
  if (s->split_cg) hipLaunchKernelGGL(k_seed_groups, dim3(1), dim3(256), 0, st, s->S, s->groups, s->ng_r);
  if (s->precond == LSPCG_PRECOND_DIAGONAL) enqueue_ob<kObInit, true>(s, st, 3, r, r, b, b, r, z);
  else enqueue_ob<kObInit>(s, st, 2, r, r, b, b);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

template <typename T>
static int enqueue_fixup(lspcg_solver* s, hipStream_t st) {
  hipLaunchKernelGGL(k_x_fixup<T>, dim3(elem_grid(s->n)), dim3(kThreads), 0, st, s->n, s->S,
                     static_cast<const T*>(s->p), static_cast<T*>(s->x));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

static bool small_path(const lspcg_solver* s) {
  if (s->dot_order != LSPCG_DOT_COMPENSATED) return false;  // parity mode: the multi-kernel schedule
  if (s->n <= 0 || s->n > s->small_n || s->precond == LSPCG_PRECOND_IC || s->Av.block_size != 1) return false;
  if (s->n > int64_t(kSmallThreadsBig) * 3 || 3 * s->n * (s->dtype == LSPCG_F32 ? 4 : 8) > kSmallLds) return false;
  if (s->precond == LSPCG_PRECOND_EXT_SPAI || s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED)
    return s->Lv.block_size == 1 && s->LTv.block_size == 1;
  return true;
}

static CsrView csr_view(const lspcg_solver* s, int w, const lspcg_mat& M) {
  CsrView v{M.rowptr, M.colind, M.vals, M.storage_dtype() == LSPCG_F32 ? 1 : 0, nullptr, nullptr, nullptr, 0, 0};
  if (const SellPattern* P = s->sp[w]) {
    // (SELL-DIA views are never built for systems this kernel solves: build_sell / lspcg_batch_create)
    if (s->small_sell && s->sv[w] && P->bs == 1 && P->groups > 0 && (P->col_bits == 16 || P->col_bits == 32)) {
      v.gp = P->gp;
      v.scol = P->col;
      v.sv = s->sv[w];
      v.sf32 = s->svd[w] == LSPCG_F32 ? 1 : 0;
      v.cmode = P->col_bits == 16 ? 1 : 0;
    }
  }
  return v;
}

template <typename T>
static int launch_small(lspcg_solver* s, hipStream_t st) {
  const bool spai = s->precond == LSPCG_PRECOND_EXT_SPAI || s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED;
  const CsrView A = csr_view(s, 0, s->Av);
  const CsrView L = spai ? csr_view(s, 1, s->Lv) : CsrView{};
  const CsrView LT = spai ? csr_view(s, 2, s->LTv) : CsrView{};
  auto* x = static_cast<T*>(s->x);
  auto* r = static_cast<T*>(s->r);
  auto* p = static_cast<T*>(s->p);
  const T* d = static_cast<const T*>(s->d);
  const int32_t n = int32_t(s->n);
  const dim3 g(1);
  const size_t lds = 3 * sizeof(T) * size_t(n);
  auto go = [&](auto rows, auto threads) {
    constexpr int R = decltype(rows)::value;
    constexpr int TH = decltype(threads)::value;
    const dim3 b(TH);
    switch (s->precond) {
      case LSPCG_PRECOND_NONE:
        hipLaunchKernelGGL((k_pcg_small<T, LSPCG_PRECOND_NONE, R, TH>), g, b, lds, st, n, s->S, A, L, LT, d, x, r, p,
                           nullptr, nullptr);
        break;
      case LSPCG_PRECOND_DIAGONAL:
        hipLaunchKernelGGL((k_pcg_small<T, LSPCG_PRECOND_DIAGONAL, R, TH>), g, b, lds, st, n, s->S, A, L, LT, d, x, r,
                           p, nullptr, nullptr);
        break;
      case LSPCG_PRECOND_EXT_SPAI:
        hipLaunchKernelGGL((k_pcg_small<T, LSPCG_PRECOND_EXT_SPAI, R, TH>), g, b, lds, st, n, s->S, A, L, LT, d, x, r,
                           p, nullptr, nullptr);
        break;
      default:
        hipLaunchKernelGGL((k_pcg_small<T, LSPCG_PRECOND_EXT_SPAI_SCALED, R, TH>), g, b, lds, st, n, s->S, A, L, LT, d,
                           x, r, p, nullptr, nullptr);
    }
  };
  using I = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using T512 = std::integral_constant<int, kSmallThreads>;
  using T1024 = std::integral_constant<int, kSmallThreadsBig>;
  // n <= 1024: 512 threads, <= 2 rows each (the measured best there); above: 1024 threads, 2-3 rows
  // (512 threads x 5 rows measured 20.5-28.2 vs 16.3-21.7 us per iteration)
  if (n <= kSmallThreads) go(I{}, T512{});
  else if (n <= 2 * kSmallThreads) go(I2{}, T512{});
  else if (n <= 2 * kSmallThreadsBig) go(I2{}, T1024{});
  else go(I3{}, T1024{});
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}


static int get_graph(lspcg_solver* s, int chunk, hipGraphExec_t* out) {
  auto it = s->graphs.find(chunk);
  if (it != s->graphs.end()) {
    *out = it->second;
    return LSPCG_OK;
  }
  hipGraph_t g = nullptr;
  LSPCG_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  int rc = LSPCG_OK;
  for (int i = 0; i < chunk && rc == LSPCG_OK; ++i)
    rc = s->dtype == LSPCG_F64 ? enqueue_iteration<double>(s, s->stream) : enqueue_iteration<float>(s, s->stream);
  hipError_t e = hipStreamEndCapture(s->stream, &g);
  if (rc) return rc;
  LSPCG_HIP(e);
  hipGraphExec_t ex = nullptr;
  LSPCG_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  s->graphs[chunk] = ex;
  s->graph_defs[chunk] = g;
  *out = ex;
  return LSPCG_OK;
}

static size_t esize(int dtype) { return dtype == LSPCG_F32 ? 4 : 8; }

extern "C" {

static int solver_create(lspcg_ctx* ctx, const lspcg_mat* A, int precond, bool dia_ok, bool reorder_ok,
                         lspcg_solver** out);

int lspcg_solver_create(lspcg_ctx* ctx, const lspcg_mat* A, int precond, lspcg_solver** out) {
  return solver_create(ctx, A, precond, true, true, out);
}

// diag(A) into s->d in the loop's numbering.  lspcg_mat_diagonal binary-searches sorted rows, so
// a permuted solver takes the caller's (sorted) A's diagonal and permutes it (s->z is scratch here:
// no solve is in flight while the preconditioner is installed).
static int solver_diagonal(lspcg_solver* s) {
  if (!s->ro.perm) return lspcg_mat_diagonal(s->A, s->d);  // issues on ctx stream
  if (int rc = lspcg_mat_diagonal(s->A_user, s->z)) return rc;
  const int bs = s->A->block_size;
  return vec_permute(s->dtype, s->n / bs, bs, s->ro.perm, s->z, s->d, false, s->ctx->stream);
}

// reducing grid of iteration view w's SpMV (the SELL / SELL-DIA copy, else the staged CSR kernel)
static int64_t view_reduce_grid(const lspcg_solver* s, int w) {
  if (s->sp[w]) return sell_grid(*s->sp[w], true);
  const lspcg_mat& V = w == 0 ? s->Av : (w == 1 ? s->Lv : s->LTv);
  const int64_t cap = std::min<int64_t>(kReduceGridMax, kElemBlocksMax);
  const int64_t g = V.block_size == 3 ? spmv_grid_t<256, 3>(V.nb) : spmv_grid_t<256, 1>(V.nb);
  return std::min<int64_t>(g, cap);
}

// group size / count of a reducing launch of `grid` workgroups (see lspcg_solver_set_spai)
static void split_groups(int mode, int64_t grid, int* gsz, int* ng) {
  const bool nogroups = mode == 2 || (mode < 0 && grid <= kNoGroupGrid);
  *gsz = nogroups ? 1 : int((grid + kMaxGroups - 1) / kMaxGroups);
  *ng = int((grid + *gsz - 1) / *gsz);
}

// CG / Jacobi on the split reductions: compensated dot order, fp64 / fp32 alike, the multi-kernel
// schedule (the one-workgroup solve has its own loop)
static void setup_split_cg(lspcg_solver* s) {
  s->split_cg = false;
  if (!(s->precond == LSPCG_PRECOND_NONE || s->precond == LSPCG_PRECOND_DIAGONAL)) return;
  if (!s->allow_split || s->dot_order != LSPCG_DOT_COMPENSATED || s->n == 0) return;
  split_groups(s->split_mode, view_reduce_grid(s, 0), &s->gsz_a, &s->ng_a);
  const int64_t eg = s->dtype == LSPCG_F64 ? elem_vec_grid<double>(s->n) : elem_vec_grid<float>(s->n);
  split_groups(s->split_mode, eg, &s->gsz_r, &s->ng_r);
  s->split_cg = s->gsz_a <= kMaxGroups && s->gsz_r <= kMaxGroups && s->ng_a <= 4096 && s->ng_r <= 4096;
}

// The A side of the solver: (optionally) the permuted system, its iteration view and SELL copy,
// the diagonal of the Jacobi preconditioner.
static int setup_A(lspcg_solver* s) {
  s->A = s->A_user;
  if (s->Ap) {
    lspcg_mat_destroy(s->Ap);
    s->Ap = nullptr;
  }
  s->ro.release();
  bool applied = false;
  if (s->reorder_ok && s->n > s->small_n) {
    if (int rc = rcm_reorder(s->A_user, s->reorder_mode, &s->ro, &applied)) return rc;
    if (applied) {
      if (int rc = mat_permute(s->A_user, s->ro, &s->Ap)) return rc;
      s->A = s->Ap;
    }
  }
  if (int rc = make_view(s, s->A, &s->Av, nullptr, &s->own_A)) return rc;
  if (int rc = build_sell(s, 0, &s->Av)) return rc;
  setup_split_cg(s);
  if (s->precond == LSPCG_PRECOND_DIAGONAL) {
    if (int rc = solver_diagonal(s)) return rc;
    LSPCG_HIP(hipStreamSynchronize(s->ctx->stream));
  }
  return LSPCG_OK;
}

static int solver_create(lspcg_ctx* ctx, const lspcg_mat* A, int precond, bool dia_ok, bool reorder_ok,
                         lspcg_solver** out) {
  LSPCG_CHECK(ctx && A && out, LSPCG_ERR_ARG, "solver_create: NULL argument");
  LSPCG_CHECK(precond >= LSPCG_PRECOND_NONE && precond <= LSPCG_PRECOND_IC, LSPCG_ERR_ARG,
              "solver_create: unknown preconditioner " + std::to_string(precond));
  LSPCG_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<lspcg_solver> s(new lspcg_solver());
  s->ctx = ctx;
  s->A = A;
  s->A_user = A;
  s->dia_ok = dia_ok;
  s->reorder_ok = reorder_ok && precond != LSPCG_PRECOND_IC;
  s->precond = precond;
  s->dtype = A->dtype;
  s->n = A->n;
  const size_t vb = esize(s->dtype) * std::max<int64_t>(s->n, 1);
  LSPCG_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
  // q (KC -> UR) and t (KA -> KB; the IC solve's intermediate) are never live together: one
  // buffer, 8 B per row less in the loop's working set (kuhn101: 78 vs 84 us per iteration with
  // two buffers, profiles/r3_tq_probe_v7.txt -- the loop sits at the Infinity Cache's size)
  for (void** v : {&s->x, &s->b, &s->r, &s->z, &s->t, &s->p, &s->q, &s->d}) {
    if (v == &s->q) {
      s->q = s->t;
      continue;
    }
    LSPCG_HIP(hipMalloc(v, vb));
    LSPCG_HIP(hipMemsetAsync(*v, 0, vb, s->stream));
  }
  LSPCG_HIP(hipMalloc(&s->S, sizeof(PcgState)));
  LSPCG_HIP(hipHostMalloc(&s->hS, 2 * sizeof(PcgState), hipHostMallocDefault));
  // partial slots: largest grid of any reducing launch (SpMV grid of A / L, element grid) x 2 dots
  // (n/255 bounds the grid of a CSR (256 rows/WG) and a BSR3 (85 block rows/WG) launch,
  // so L / Lᵀ in either layout fit too)
  const int64_t g = std::max<int64_t>((A->n + 254) / 255 + 1, 4096);
  LSPCG_HIP(hipMalloc(&s->partials, sizeof(double) * 2 * 2 * (g + 1)));
  LSPCG_HIP(hipMalloc(&s->ticket, sizeof(unsigned) * kTicketWords));
  LSPCG_HIP(hipMemsetAsync(s->ticket, 0, sizeof(unsigned) * kTicketWords, s->stream));
  LSPCG_HIP(hipMalloc(&s->groups, sizeof(double) * 4096 * 2 * 3));
  LSPCG_HIP(hipMemsetAsync(s->groups, 0, sizeof(double) * 4096 * 2 * 3, s->stream));
  LSPCG_HIP(hipMemsetAsync(s->S, 0, sizeof(PcgState), s->stream));
  for (hipEvent_t* e : {&s->ev_in, &s->ev_out, &s->ev_poll, &s->ev_poll2}) LSPCG_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  LSPCG_HIP(hipEventCreate(&s->ev_t0));
  LSPCG_HIP(hipEventCreate(&s->ev_t1));
  LSPCG_HIP(hipMalloc(&s->flag, sizeof(int)));
  LSPCG_HIP(hipMalloc(&s->ob_part, sizeof(double) * 3 * kObMaxThreads));
  if (const char* e = std::getenv("LSPCG_NO_SELL")) s->use_sell = e[0] == '0';
  if (const char* e = std::getenv("LSPCG_SMALL_N")) s->small_n = std::max<int64_t>(0, std::atoll(e));
  if (const char* e = std::getenv("LSPCG_SMALL_SELL")) s->small_sell = e[0] != '0';
  if (const char* e = std::getenv("LSPCG_SPLIT_REDUCE")) {
    s->allow_split = e[0] != '0';
    s->split_mode = std::atoi(e);
  }
  if (const char* e = std::getenv("LSPCG_REORDER")) s->reorder_mode = e[0] == 'a' ? -1 : std::atoi(e) ? 1 : 0;
  if (int rc = setup_A(s.get())) return rc;
  LSPCG_HIP(hipStreamSynchronize(s->stream));
  *out = s.release();
  return LSPCG_OK;
}

// Everything a captured iteration graph holds by value besides the solver's own fixed buffers: the
// views' arrays (SELL copies or CSR views), their value types, the reduction geometry and ε.  A
// new L whose views land at the same addresses keeps the graphs (build_sell / make_view refill in
// place), so a sample-by-sample loop does not re-capture every chunk size per sample.
struct GraphKey {
  std::vector<int64_t> v;  // pointers, kinds and sizes, in a fixed order
  double eps = 0.0;
  bool operator==(const GraphKey& o) const { return v == o.v && eps == o.eps; }
};
static GraphKey graph_key(const lspcg_solver* s) {
  GraphKey k;
  auto put = [&](auto x) {
    if constexpr (std::is_pointer<decltype(x)>::value) k.v.push_back(int64_t(reinterpret_cast<intptr_t>(x)));
    else k.v.push_back(int64_t(x));
  };
  for (int w = 0; w < 3; ++w) {
    const lspcg_mat& V = w == 0 ? s->Av : (w == 1 ? s->Lv : s->LTv);
    put(s->sp[w]);
    if (const SellPattern* P = s->sp[w]) {  // its contents too: a rebuilt pattern may reuse the host address
      put(P->gp);
      put(P->col);
      put(P->dict);
      put(P->rgp);
      put(P->col2);
      put(P->rowptr);
      put(P->col_bits);
      put(P->bs);
      put(P->n);
      put(P->ns);
      put(P->groups);
    }
    put(s->sv[w]);
    put(V.rowptr);
    put(V.colind);
    put(V.vals);
    put(s->svd[w]);
    put(V.val_dtype);
  }
  put(s->split);
  put(s->split_cg);
  put(s->gsz_l);
  put(s->ng_l);
  put(s->gsz_a);
  put(s->ng_a);
  put(s->dot_order);
  k.eps = s->eps;
  return k;
}

int lspcg_solver_set_spai(lspcg_solver* s, const lspcg_mat* L, double epsilon, double* t_prec_ms) {
  LSPCG_CHECK(s && L, LSPCG_ERR_ARG, "set_spai: NULL");
  LSPCG_CHECK(s->precond == LSPCG_PRECOND_EXT_SPAI || s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED, LSPCG_ERR_ARG,
              "set_spai: solver was not created with an ext_spai preconditioner");
  LSPCG_CHECK(L->n == s->n, LSPCG_ERR_ARG, "set_spai: L has a different size than A");
  LSPCG_CHECK(L->dtype == s->dtype, LSPCG_ERR_ARG, "set_spai: L dtype differs from A dtype");
  hipStream_t cst = s->ctx->stream;
  const GraphKey key_before = graph_key(s);
  LSPCG_HIP(hipStreamSynchronize(s->stream));  // Lᵀ below may be referenced by a running solve
  LSPCG_HIP(hipEventRecord(s->ev_t0, cst));
  // Lᵀ (and, reordered, P L Pᵀ / P Lᵀ Pᵀ) of the previous factor are overwritten in place when the
  // new L has its shape: no free / allocate per sample, and the iteration views keep their addresses
  // (so the captured graphs survive, graph_key below)
  auto renew = [](lspcg_mat** slot, lspcg_mat* keep, int rc) {
    if (keep && keep != *slot) lspcg_mat_destroy(keep);
    return rc;
  };
  bool lt_same = false;
  lspcg_mat** raw_slot = s->ro.perm ? &s->LTo : &s->LT;  // Lᵀ in the ORIGINAL numbering: rows in scipy's order
  lspcg_mat* keep = *raw_slot;
  *raw_slot = nullptr;
  int rc = renew(raw_slot, keep, mat_transpose(L, raw_slot, &lt_same, keep));
  if (rc) return rc;
  const lspcg_mat* Lu = L;
  if (s->ro.perm) {  // reordered solver: P L Pᵀ and P Lᵀ Pᵀ, every row's entries in their original order
    LSPCG_CHECK(L->block_size == s->A->block_size, LSPCG_ERR_ARG, "set_spai: L and A block sizes differ");
    keep = s->Lp;
    s->Lp = nullptr;
    if ((rc = renew(&s->Lp, keep, mat_permute(L, s->ro, &s->Lp, keep)))) return rc;
    keep = s->LT;
    s->LT = nullptr;
    if ((rc = renew(&s->LT, keep, mat_permute(s->LTo, s->ro, &s->LT, keep)))) return rc;
    Lu = s->Lp;
  }
  if (s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED) {
    LSPCG_HIP(hipStreamSynchronize(s->stream));  // s->z is the permuted path's scratch
    rc = solver_diagonal(s);
    if (rc) return rc;
  }
  int lflag = 3;
  if ((rc = make_view(s, Lu, &s->Lv, &s->Av, &s->own_L, nullptr, &lflag, &s->own_L_n))) return rc;
  if ((rc = make_view(s, s->LT, &s->LTv, &s->Av, &s->own_LT, lt_same ? &lflag : nullptr, nullptr, &s->own_LT_n)))
    return rc;
  if ((rc = build_sell(s, 1, &s->Lv))) return rc;
  if ((rc = build_sell(s, 2, &s->LTv))) return rc;
  // the split schedule runs on any iteration views (SELL copies or the staged CSR kernel, whose
  // epilogues finish their dots the same way; round 5 -- before, it needed SELL views of A, L, Lᵀ)
  s->split_ok = s->allow_split;
  s->split = s->split_ok && s->dot_order == LSPCG_DOT_COMPENSATED;
  if (s->split_ok) {
    // <= 64 groups per reducing launch; no groups at all (the consumers sum every workgroup's
    // partial) for grids of <= kNoGroupGrid workgroups -- mid-size systems, where the group ticket's
    // round trip costs more than the consumers' extra loads (Poisson 256^2: 20.6 vs 22.0 us per
    // iteration; at 1 M rows, 1536 workgroups, the groups win: 91.4 vs 94.3).
    // LSPCG_SPLIT_REDUCE=1 / 2 force groups / no groups.
    split_groups(s->split_mode, view_reduce_grid(s, 1), &s->gsz_l, &s->ng_l);
    split_groups(s->split_mode, view_reduce_grid(s, 0), &s->gsz_a, &s->ng_a);
    LSPCG_CHECK(s->gsz_l <= kMaxGroups && s->gsz_a <= kMaxGroups, LSPCG_ERR_UNSUPPORTED,
                "set_spai: reducing grid too large for one-wave group sums");
  }
  LSPCG_HIP(hipEventRecord(s->ev_t1, cst));
  LSPCG_HIP(hipEventSynchronize(s->ev_t1));
  float ms = 0.f;
  LSPCG_HIP(hipEventElapsedTime(&ms, s->ev_t0, s->ev_t1));
  if (t_prec_ms) *t_prec_ms = ms;
  s->L = L;
  s->eps = epsilon;
  // graphs capture the views' addresses and ε: drop them unless the new L kept every one of them
  if (!(graph_key(s) == key_before)) {
    for (auto& kv : s->graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto& kv : s->graph_defs) (void)hipGraphDestroy(kv.second);
    s->graphs.clear();
    s->graph_defs.clear();
  }
  return LSPCG_OK;
}

// IC preconditioner: factor (given, or IC(0) of A computed on the device), its explicit transpose
// and both level orders
static int install_ic(lspcg_solver* s, const lspcg_mat* given, double* t_prec_ms) {
  LSPCG_CHECK(s, LSPCG_ERR_ARG, "set_ic: NULL");
  LSPCG_CHECK(s->precond == LSPCG_PRECOND_IC, LSPCG_ERR_ARG, "set_ic: solver was not created with LSPCG_PRECOND_IC");
  LSPCG_HIP(hipSetDevice(s->ctx->device));
  LSPCG_HIP(hipStreamSynchronize(s->stream));
  if (given) {
    LSPCG_CHECK(given->n == s->n && given->block_size == 1 && given->dtype == s->dtype &&
                    given->storage_dtype() == given->dtype,
                LSPCG_ERR_ARG, "set_ic_factor: L must be a scalar CSR of the solver's size and dtype");
    // lower triangular with the diagonal stored last in every row, and a nonzero diagonal (host
    // check; scipy's spsolve_triangular, the reference's apply, raises LinAlgError "A is singular:
    // zero entry on diagonal" there -- validate.py:344-419)
    std::vector<int32_t> rp(size_t(s->n) + 1), ci(size_t(std::max<int64_t>(given->nnzb, 1)));
    std::vector<double> vd(given->dtype == LSPCG_F64 ? ci.size() : 0);
    std::vector<float> vf(given->dtype == LSPCG_F32 ? ci.size() : 0);
    void* vals = given->dtype == LSPCG_F64 ? static_cast<void*>(vd.data()) : static_cast<void*>(vf.data());
    if (int rc = lspcg_mat_copy_out(given, rp.data(), ci.data(), vals)) return rc;
    for (int64_t i = 0; i < s->n; ++i) {
      bool ok = rp[i + 1] > rp[i] && ci[rp[i + 1] - 1] == i;
      for (int32_t p = rp[i]; ok && p < rp[i + 1] - 1; ++p) ok = ci[p] < ci[p + 1];
      LSPCG_CHECK(ok, LSPCG_ERR_FORMAT,
                  "set_ic_factor: row " + std::to_string(i) + " is not lower triangular with its diagonal last");
      const int32_t dp = rp[i + 1] - 1;
      const double dv = given->dtype == LSPCG_F64 ? vd[dp] : double(vf[dp]);
      LSPCG_CHECK(dv != 0.0, LSPCG_ERR_SINGULAR,
                  "set_ic_factor: A is singular: zero entry on diagonal (row " + std::to_string(i) + ")");
    }
  }
  hipStream_t cst = s->ctx->stream;
  LSPCG_HIP(hipEventRecord(s->ev_t0, cst));
  for (lspcg_mat** m : {&s->icL, &s->icU}) {
    if (*m) lspcg_mat_destroy(*m);
    *m = nullptr;
  }
  s->levL.release();
  s->levU.release();
  int rc = given ? lspcg_mat_create_csr(s->ctx, given->n, given->nnzb, given->rowptr, given->colind, given->vals,
                                        given->dtype, &s->icL)
                 : ic0_factor(s->A, &s->icL);
  if (!rc) rc = lspcg_mat_transpose(s->icL, &s->icU);
  if (!rc) rc = build_levels(s->ctx, s->n, s->icL->rowptr, s->icL->colind, true, &s->levL);
  if (!rc) rc = build_levels(s->ctx, s->n, s->icU->rowptr, s->icU->colind, false, &s->levU);
  if (!rc) rc = trsv_prepare(s->icL, true, &s->levL);
  if (!rc) rc = trsv_prepare(s->icU, false, &s->levU);
  if (rc) return rc;
  LSPCG_HIP(hipEventRecord(s->ev_t1, cst));
  LSPCG_HIP(hipEventSynchronize(s->ev_t1));
  float ms = 0.f;
  LSPCG_HIP(hipEventElapsedTime(&ms, s->ev_t0, s->ev_t1));
  if (t_prec_ms) *t_prec_ms = ms;
  for (auto& kv : s->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : s->graph_defs) (void)hipGraphDestroy(kv.second);
  s->graphs.clear();
  s->graph_defs.clear();
  return LSPCG_OK;
}

int lspcg_solver_set_ic(lspcg_solver* s, double* t_prec_ms) { return install_ic(s, nullptr, t_prec_ms); }

int lspcg_solver_set_ic_factor(lspcg_solver* s, const lspcg_mat* L, double* t_prec_ms) {
  LSPCG_CHECK(L, LSPCG_ERR_ARG, "set_ic_factor: NULL factor");
  return install_ic(s, L, t_prec_ms);
}

int lspcg_solver_solve(lspcg_solver* s, const void* b, void* x, double rtol, int64_t max_iter, int64_t* iters,
                       double* res_hist, double* t_solve_ms) {
  LSPCG_CHECK(s && b && x && iters, LSPCG_ERR_ARG, "solve: NULL argument");
  LSPCG_CHECK(!(s->precond == LSPCG_PRECOND_EXT_SPAI || s->precond == LSPCG_PRECOND_EXT_SPAI_SCALED) || s->LT,
              LSPCG_ERR_ARG, "solve: ext_spai not set");
  LSPCG_CHECK(s->precond != LSPCG_PRECOND_IC || s->icL, LSPCG_ERR_ARG, "solve: IC factor not set (lspcg_solver_set_ic)");
  LSPCG_HIP(hipSetDevice(s->ctx->device));
  const int64_t n = s->n;
  if (max_iter <= 0) max_iter = n;
  hipStream_t st = s->stream;
  const size_t vb = esize(s->dtype) * n;
  double* dhist = nullptr;  // the solver's persistent history buffer, grown on demand
  if (res_hist) {
    if (s->dhist_cap < max_iter + 2) {
      LSPCG_HIP(hipStreamSynchronize(st));
      (void)hipFree(s->dhist);
      (void)hipHostFree(s->hhist);
      s->dhist = nullptr;
      s->hhist = nullptr;
      s->dhist_cap = 0;
      LSPCG_HIP(hipMalloc(&s->dhist, sizeof(double) * (max_iter + 2)));
      LSPCG_HIP(hipHostMalloc(&s->hhist, sizeof(double) * (max_iter + 2), hipHostMallocDefault));
      s->dhist_cap = max_iter + 2;
    }
    dhist = s->dhist;
  }

  // every enqueue below runs under the process-wide submission lock, released around each host
  // wait (lspcg_internal.hpp: concurrent solves from several host threads)
  std::unique_lock<std::mutex> sub(submit_mutex());
  auto wait = [&sub](hipEvent_t e) {
    sub.unlock();
    const hipError_t r = hipEventSynchronize(e);
    sub.lock();
    return r;
  };
  LSPCG_HIP(hipEventRecord(s->ev_in, s->ctx->stream));
  LSPCG_HIP(hipStreamWaitEvent(st, s->ev_in, 0));
  LSPCG_HIP(hipEventRecord(s->ev_t0, st));
  if (n && s->ro.perm) {  // into the permuted numbering
    const int bs = s->A->block_size;
    if (int r2 = vec_permute(s->dtype, n / bs, bs, s->ro.perm, b, s->b, false, st)) return r2;
    if (int r2 = vec_permute(s->dtype, n / bs, bs, s->ro.perm, x, s->x, false, st)) return r2;
  } else if (n) {
    LSPCG_HIP(hipMemcpyAsync(s->b, b, vb, hipMemcpyDeviceToDevice, st));
    LSPCG_HIP(hipMemcpyAsync(s->x, x, vb, hipMemcpyDeviceToDevice, st));
  }
  PcgState init{};
  init.rtol = rtol;
  init.eps = s->eps;
  init.hist = dhist;
  init.max_iter = max_iter;
  *s->hS = init;
  LSPCG_HIP(hipMemcpyAsync(s->S, s->hS, sizeof(PcgState), hipMemcpyHostToDevice, st));
  int rc = s->dtype == LSPCG_F64 ? enqueue_init<double>(s, st) : enqueue_init<float>(s, st);
  if (rc) return rc;

  // Poll loop, one chunk ahead: the state copied after chunk k is read while chunk k+1 runs, so
  // the GPU does not idle through the host round trip.  Chunk sizes follow the observed residual
  // decay minus the iterations already in flight, so that at most a few early-exit launches trail
  // the converged iteration (every launch is predicated on the device `done` flag).
  // graphs hold <= ~4096 nodes (IC: one launch per level of each triangular solve)
  const int kpi = s->precond == LSPCG_PRECOND_IC ? 2 * kTrsvLaunches + 4 : 5;
  const int max_chunk = std::max(1, std::min(32, 4096 / kpi));
  PcgState* const hs[2] = {s->hS, s->hS + 1};
  const hipEvent_t evp[2] = {s->ev_poll, s->ev_poll2};
  int64_t queued[2] = {0, 0};  // iterations launched after each outstanding poll
  int head = 0, npend = 0;     // oldest outstanding poll slot, number outstanding (<= 2)
  auto post = [&]() -> int {   // a state copy + event after everything enqueued so far
    const int k = (head + npend) & 1;
    LSPCG_HIP(hipMemcpyAsync(hs[k], s->S, sizeof(PcgState), hipMemcpyDeviceToHost, st));
    LSPCG_HIP(hipEventRecord(evp[k], st));
    queued[k] = 0;
    ++npend;
    return LSPCG_OK;
  };
  int64_t launched = 0, nlaunch = 0;  // iterations / graphs enqueued (LSPCG_SOLVE_PROFILE)
  auto launch = [&](int c) -> int {
    hipGraphExec_t ex = nullptr;
    int r = get_graph(s, c, &ex);
    if (r) return r;
    LSPCG_HIP(hipGraphLaunch(ex, st));
    launched += c;
    ++nlaunch;
    for (int j = 0; j < npend; ++j) queued[(head + j) & 1] += c;
    return post();
  };
  PcgState cur{};
  const bool small = small_path(s);
  if (small) {  // one launch runs the whole loop (k_pcg_small)
    rc = s->dtype == LSPCG_F64 ? launch_small<double>(s, st) : launch_small<float>(s, st);
    if (!rc) rc = post();
    if (rc) return rc;
    LSPCG_HIP(wait(evp[head]));
    cur = *hs[head];
  } else {
    rc = post();
    if (!rc) rc = launch(std::min(4, max_chunk));
    if (rc) return rc;
  }
  int64_t last_it = 0;
  double last_rr = -1.0;
  int chunk = std::min(4, max_chunk);
  for (; !small;) {
    LSPCG_HIP(wait(evp[head]));
    cur = *hs[head];
    const int64_t inflight = queued[head];
    head ^= 1;
    --npend;
    if (cur.done) break;  // ProCheck sets done (convergence, max_iter or a non-finite residual)
    int64_t rem = -1;     // predicted iterations still needed after this state
    if (last_rr > 0 && cur.iter > last_it && cur.rr > 0 && cur.rr < last_rr) {
      const double rate = std::log(cur.rr / last_rr) / double(cur.iter - last_it);  // < 0
      const double need = std::log((cur.atol * cur.atol) / cur.rr) / rate;
      rem = need > 0 ? int64_t(std::ceil(need)) : 1;
      rem = std::max<int64_t>(1, std::min<int64_t>(rem, max_iter - cur.iter));
    }
    if (cur.iter > last_it || last_rr < 0) {
      last_it = cur.iter;
      last_rr = cur.rr;
    }
    if (rem >= 0) {
      const int64_t more = rem - inflight;
      if (more <= 0) {
        if (npend == 0) rc = launch(1);  // predicted to converge in flight; nothing in flight
        if (rc) return rc;
        continue;
      }
      int c = 1;
      while (c * 2 <= more && c < max_chunk) c *= 2;
      chunk = c;
    } else {
      chunk = std::min(max_chunk, chunk * 2);
    }
    rc = launch(std::min(chunk, max_chunk));
    if (rc) return rc;
  }
  const PcgState fin = cur;  // later (early-exit) launches leave the state unchanged
  rc = s->dtype == LSPCG_F64 ? enqueue_fixup<double>(s, st) : enqueue_fixup<float>(s, st);
  if (rc) return rc;
  const void* src = (fin.bb == 0.0) ? s->b : s->x;  // scipy returns b when ‖b‖ = 0
  if (n && s->ro.perm) {  // back to the caller's numbering
    if (int r2 = vec_permute(s->dtype, n / s->A->block_size, s->A->block_size, s->ro.perm, src, x, true, st)) return r2;
  } else if (n) {
    LSPCG_HIP(hipMemcpyAsync(x, src, vb, hipMemcpyDeviceToDevice, st));
  }
  LSPCG_HIP(hipEventRecord(s->ev_t1, st));
  // the tail's device-to-host copies (IC timeout flags, the residual history) are enqueued behind the
  // solve into pinned mirrors, so the last host wait is the only one and the submission lock is not
  // held through it (a blocking copy under the lock serialised concurrent solves' tails)
  const bool ic = s->precond == LSPCG_PRECOND_IC;
  if (ic) {
    if (!s->hflags) LSPCG_HIP(hipHostMalloc(&s->hflags, 2 * sizeof(unsigned), hipHostMallocDefault));
    s->hflags[0] = s->hflags[1] = 0;
    if (s->levL.head)
      LSPCG_HIP(hipMemcpyAsync(&s->hflags[0], s->levL.head + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    if (s->levU.head)
      LSPCG_HIP(hipMemcpyAsync(&s->hflags[1], s->levU.head + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  }
  const int64_t it = (fin.done == 3) ? max_iter : fin.iter;
  // history entries 0..fin.iter were written; a non-finite residual stops early while iters reports
  // max_iter (pymathprim's count), so the rest of 0..iters is NaN-filled
  const int64_t hcnt = std::min<int64_t>(fin.iter, max_iter) + 1;
  if (res_hist) LSPCG_HIP(hipMemcpyAsync(s->hhist, dhist, sizeof(double) * hcnt, hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipEventRecord(s->ev_out, st));
  LSPCG_HIP(hipStreamWaitEvent(s->ctx->stream, s->ev_out, 0));
  sub.unlock();
  LSPCG_HIP(hipEventSynchronize(s->ev_out));
  if (ic && (s->hflags[0] || s->hflags[1])) {  // a timed-out sync-free hand-off fails the solve loudly
    sub.lock();
    if (int r2 = trsv_check_timeout(s->levL, st)) return r2;  // resets the flag, sets the message
    if (int r2 = trsv_check_timeout(s->levU, st)) return r2;
  }
  float ms = 0.f;
  LSPCG_HIP(hipEventElapsedTime(&ms, s->ev_t0, s->ev_t1));
  if (t_solve_ms) *t_solve_ms = ms;
  static const bool prof = [] {
    const char* e = std::getenv("LSPCG_SOLVE_PROFILE");
    return e && e[0] == '1';
  }();
  if (prof)
    std::fprintf(stderr, "[lspcg solve] n=%lld iters=%lld launched=%lld in %lld graphs, %.3f ms\n",
                 static_cast<long long>(n), static_cast<long long>(it), static_cast<long long>(launched),
                 static_cast<long long>(nlaunch), double(ms));
  *iters = it;
  if (res_hist) {
    std::memcpy(res_hist, s->hhist, sizeof(double) * hcnt);
    for (int64_t k = hcnt; k <= it; ++k) res_hist[k] = NAN;
  }
  return (fin.done == 1) ? LSPCG_OK : LSPCG_NOT_CONVERGED;
}

int lspcg_solver_set_dot_order(lspcg_solver* s, int order, int threads) {
  LSPCG_CHECK(s, LSPCG_ERR_ARG, "set_dot_order: NULL");
  LSPCG_CHECK(order == LSPCG_DOT_COMPENSATED || order == LSPCG_DOT_OPENBLAS, LSPCG_ERR_ARG,
              "set_dot_order: unknown order " + std::to_string(order));
  LSPCG_CHECK(order == LSPCG_DOT_COMPENSATED || (threads >= 1 && threads <= kObMaxThreads), LSPCG_ERR_ARG,
              "set_dot_order: threads must be in [1, 16]");
  LSPCG_CHECK(order == LSPCG_DOT_COMPENSATED || s->dtype == LSPCG_F64, LSPCG_ERR_UNSUPPORTED,
              "set_dot_order: the OpenBLAS order is the fp64 ddot's (the reference solves in fp64)");
  LSPCG_HIP(hipStreamSynchronize(s->stream));
  s->dot_order = order;
  s->dot_threads = order == LSPCG_DOT_OPENBLAS ? threads : 1;
  if (order == LSPCG_DOT_OPENBLAS && s->reorder_ok) {
    // numpy's ddot order runs over the ORIGINAL numbering: back to the unpermuted system for good
    s->reorder_ok = false;
    if (s->ro.perm) {
      if (int rc = setup_A(s)) return rc;
      if (s->L) {
        if (int rc = lspcg_solver_set_spai(s, s->L, s->eps, nullptr)) return rc;
      }
    }
  }
  s->split = s->split_ok && order == LSPCG_DOT_COMPENSATED;
  setup_split_cg(s);
  for (auto& kv : s->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : s->graph_defs) (void)hipGraphDestroy(kv.second);
  s->graphs.clear();
  s->graph_defs.clear();
  return LSPCG_OK;
}

int lspcg_solver_time_kernels(lspcg_solver* s, const void* b, int64_t iters, double* kernel_ms, int* nk) {
  LSPCG_CHECK(s && b && kernel_ms && nk && iters > 0, LSPCG_ERR_ARG, "time_kernels: bad argument");
  *nk = 0;
  LSPCG_CHECK(s->split, LSPCG_ERR_UNSUPPORTED, "time_kernels: only the split ext_spai schedule (LSPCG_SPLIT_REDUCE != 0)");
  LSPCG_HIP(hipSetDevice(s->ctx->device));
  const int64_t n = s->n;
  hipStream_t st = s->stream;
  const size_t vb = esize(s->dtype) * n;
  LSPCG_HIP(hipEventRecord(s->ev_in, s->ctx->stream));
  LSPCG_HIP(hipStreamWaitEvent(st, s->ev_in, 0));
  if (s->ro.perm) {
    if (int r2 = vec_permute(s->dtype, n / s->A->block_size, s->A->block_size, s->ro.perm, b, s->b, false, st)) return r2;
  } else {
    LSPCG_HIP(hipMemcpyAsync(s->b, b, vb, hipMemcpyDeviceToDevice, st));
  }
  LSPCG_HIP(hipMemsetAsync(s->x, 0, vb, st));
  PcgState init{};
  init.rtol = 0.0;  // atol 0: no convergence stop, `iters` full iterations
  init.eps = s->eps;
  init.max_iter = iters + 1;
  *s->hS = init;
  LSPCG_HIP(hipMemcpyAsync(s->S, s->hS, sizeof(PcgState), hipMemcpyHostToDevice, st));
  int rc = s->dtype == LSPCG_F64 ? enqueue_init<double>(s, st) : enqueue_init<float>(s, st);
  if (rc) return rc;
  // each launch timed by its own start / end stamps (KernelTimer: the kernel durations rocprofv3's
  // trace reports, without the in-stream boundaries event pairs between launches would add)
  constexpr int K = 5;
  KernelTimer kt[K];
  for (auto& t : kt) {
    LSPCG_HIP(hipEventCreate(&t.start));
    LSPCG_HIP(hipEventCreate(&t.stop));
  }
  double acc[K] = {0, 0, 0, 0, 0};
  for (int64_t it = 0; it < iters && rc == LSPCG_OK; ++it) {
    s->tk = kt;
    s->tk_i = 0;
    rc = s->dtype == LSPCG_F64 ? enqueue_iteration<double>(s, st) : enqueue_iteration<float>(s, st);
    s->tk = nullptr;
    kernel_timer() = nullptr;
    if (rc) break;
    LSPCG_HIP(hipEventSynchronize(kt[K - 1].stop));
    for (int k = 0; k < K; ++k) {
      float ms = 0.f;
      LSPCG_HIP(hipEventElapsedTime(&ms, kt[k].start, kt[k].stop));
      acc[k] += ms;
    }
  }
  for (auto& t : kt) {
    (void)hipEventDestroy(t.start);
    (void)hipEventDestroy(t.stop);
  }
  if (rc) return rc;
  for (int k = 0; k < K; ++k) kernel_ms[k] = acc[k] / double(iters);
  *nk = K;
  LSPCG_HIP(hipEventRecord(s->ev_out, st));
  LSPCG_HIP(hipStreamWaitEvent(s->ctx->stream, s->ev_out, 0));
  return LSPCG_OK;
}

int lspcg_solver_views(const lspcg_solver* s, int* col_kind, int* value_bytes) {
  LSPCG_CHECK(s && col_kind && value_bytes, LSPCG_ERR_ARG, "solver_views: NULL argument");
  for (int w = 0; w < 3; ++w) {
    const SellPattern* P = s->sp[w];
    col_kind[w] = P ? P->col_bits : 0;
    value_bytes[w] = !P ? 0 : s->svd[w] == LSPCG_F32 ? 4 : 8;
  }
  return LSPCG_OK;
}

int lspcg_solver_reorder_info(const lspcg_solver* s, int* applied, double* mean_offset_before,
                              double* mean_offset_after) {
  LSPCG_CHECK(s && applied, LSPCG_ERR_ARG, "reorder_info: NULL argument");
  *applied = s->ro.perm ? 1 : 0;
  if (mean_offset_before) *mean_offset_before = s->ro.off_before;
  if (mean_offset_after) *mean_offset_after = s->ro.off_after;
  return LSPCG_OK;
}

int lspcg_solver_destroy(lspcg_solver* s) {
  if (!s) return LSPCG_OK;
  (void)hipSetDevice(s->ctx->device);
  (void)hipStreamSynchronize(s->stream);
  for (auto& kv : s->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : s->graph_defs) (void)hipGraphDestroy(kv.second);
  for (void* v : {s->x, s->b, s->r, s->z, s->t, s->p, s->d}) (void)hipFree(v);
  if (s->q != s->t) (void)hipFree(s->q);
  (void)hipFree(s->S);
  (void)hipHostFree(s->hS);
  (void)hipFree(s->partials);
  (void)hipFree(s->ticket);
  (void)hipFree(s->groups);
  for (hipEvent_t e : {s->ev_in, s->ev_out, s->ev_poll, s->ev_poll2, s->ev_t0, s->ev_t1}) (void)hipEventDestroy(e);
  if (s->LT) lspcg_mat_destroy(s->LT);
  if (s->Lp) lspcg_mat_destroy(s->Lp);
  if (s->LTo) lspcg_mat_destroy(s->LTo);
  if (s->Ap) lspcg_mat_destroy(s->Ap);
  s->ro.release();
  if (s->icL) lspcg_mat_destroy(s->icL);
  if (s->icU) lspcg_mat_destroy(s->icU);
  s->levL.release();
  s->levU.release();
  for (void* p : {s->own_A, s->own_L, s->own_LT}) (void)hipFree(p);
  for (int w = 0; w < 3; ++w) {
    (void)hipFree(s->sv[w]);
    s->spat[w].release();
  }
  (void)hipFree(s->flag);
  (void)hipFree(s->ob_part);
  (void)hipFree(s->dhist);
  (void)hipHostFree(s->hhist);
  (void)hipHostFree(s->hflags);
  (void)hipStreamDestroy(s->stream);
  delete s;
  return LSPCG_OK;
}

}  // extern "C"

// ==== batched lockstep ext_spai PCG (lspcg_batch_*) ===========================
// A window of independent systems is laid out block-diagonally, every system's rows padded to
// whole SpMV row tiles (256 block rows), and ONE launch per phase covers all of them: the split
// schedule's five launches (KA, KB, UP, KC, UR) with
//   * one row tile per workgroup (launch_spmv_sell_cfg one_tile_per_wg), so a workgroup's dot
//     partial is its tile's and its prologue tests the tile's own system (done systems' tiles
//     leave at once);
//   * per-system last-arriver dot reductions (batch_sys_reduce): the last tile of a system to
//     finish KB / KC sums the system's tile partials and updates its PcgState (scipy's scalars,
//     the top-of-loop test, the iteration count), as the last-arriver schedule does for one system;
//   * elementwise launches (UP, UR) of one 256-row tile per workgroup that read their system's
//     finished scalars.
// Padding rows are empty: they stay 0 in every vector and add exact zeros to the dots.
namespace lspcg {

struct BatchMap {
  const int32_t* etile_sys;  // [n / 256] system of each 256-row elementwise tile
  const int32_t* tile0;      // [nsys + 1] first SpMV row tile (256 block rows) of each system
  const int32_t* tk0;        // [nsys] first ticket line of each system: [top | group 0 | group 1 | ...]
  int bs;                    // block size: SpMV tile b covers elementwise tiles bs*b .. bs*b + bs - 1
};

struct ProTile {
  const PcgState* S;
  BatchMap m;
  __device__ __forceinline__ bool exit() const { return S[m.etile_sys[int64_t(blockIdx.x) * m.bs]].done != 0; }
};

// Per-system last-arriver reduction of a batched launch's N dots: each workgroup (= one row tile)
// publishes its tile total (sc1 stores, drained, then relaxed agent-scope adds -- MI355X_MICROARCH.md
// "Valid forms", table row 1, as grid_reduce_dd); the adds go to a two-level ticket (groups of
// kTicketGroup tiles, then the system's top line: <= 32 serialised arrivals per line instead of a
// system's few hundred -- the fan-in price), and the system's last arriving tile sums the system's
// tile totals in tile order (fixed tree: the result does not depend on which tile came last);
// thread 0 then runs fin(sys, values).  The elementwise launches read finished per-system scalars.
template <int N, class Fin>
__device__ __forceinline__ void batch_sys_reduce(DD (&v)[N], double* partials, unsigned* tickets, const BatchMap& m,
                                                 Fin fin) {
  __shared__ DD lds[16 * N];
  __shared__ int s_last;
  block_reduce_dd<N>(v, lds);
  const int64_t tile = blockIdx.x;
  const int sys = m.etile_sys[tile * m.bs];
  const int t0 = m.tile0[sys], nt = m.tile0[sys + 1] - t0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      st_agent_f64(&partials[(size_t(tile) * N + j) * 2 + 0], v[j].s);
      st_agent_f64(&partials[(size_t(tile) * N + j) * 2 + 1], v[j].c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* top = tickets + size_t(kTicketStride) * m.tk0[sys];
    const unsigned g = unsigned(tile - t0) / kTicketGroup;
    const unsigned gsize = min(unsigned(kTicketGroup), unsigned(nt) - g * kTicketGroup);
    const unsigned ng = (unsigned(nt) + kTicketGroup - 1) / kTicketGroup;
    unsigned* gt = top + size_t(kTicketStride) * (1 + g);
    int last = 0;
    if (__hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
      if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  DD acc[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = dd_zero();
  for (int b = threadIdx.x; b < nt; b += blockDim.x) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const size_t k = (size_t(t0 + b) * N + j) * 2;
      acc[j] = dd_add(acc[j], DD{ld_agent_f64(&partials[k]), ld_agent_f64(&partials[k + 1])});
    }
  }
  __syncthreads();
  block_reduce_dd<N>(acc, lds);
  if (threadIdx.x == 0) {
    double out[N];
#pragma unroll
    for (int j = 0; j < N; ++j) out[j] = dd_value(acc[j]);
    fin(sys, out);
  }
}

// init: r_0 = b - A x0 ; ‖r_0‖², ‖b‖² -> the system's initial state (EpiResid::fin)
template <typename T>
struct EpiResidB {
  static constexpr int NDOT = 2;
  static constexpr bool CUSTOM_FINISH = true;
  T* r;
  const T* b;
  PcgState* S;
  double* partials;
  unsigned* tickets;
  BatchMap m;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T bi = gld(b + i);
    const T ri = bi - s;
    gst(r + i, ri);
    dd_fma(dots[0], double(ri), double(ri));
    dd_fma(dots[1], double(bi), double(bi));
  }
  __device__ __forceinline__ void finish(DD (&d)[2]) const {
    PcgState* Sb = S;
    batch_sys_reduce<2>(d, partials, tickets, m, [Sb](int sys, const double* v) {
      PcgState* St = Sb + sys;
      St->rr = round_to<T>(v[0]);
      St->bb = round_to<T>(v[1]);
      const double bn = double(tsqrt<T>(T(St->bb)));
      St->atol = fmax(0.0, St->rtol * bn);
      St->rho = St->rr;
      St->alpha = 0.0;
      St->iter = 0;
      St->done = (bn == 0.0) ? 1 : 0;
      if (St->hist) St->hist[0] = double(tsqrt<T>(T(St->rr)));
    });
  }
};

// KB: z = L t + ε r ; ρ_k = r·z, ‖r_k‖² -> the system's last arriver keeps ρ_k (EpiZ::fin) and runs
// scipy's top-of-loop test on ‖r_k‖ (ProCheck / k_update_p_g): every tile of the system has
// already passed this launch's prologue, so setting `done` here is seen first by UP
template <typename T>
struct EpiZB {
  static constexpr int NDOT = 2;
  static constexpr bool CUSTOM_FINISH = true;
  T* z;
  const T* r;
  T eps;
  PcgState* S;
  double* partials;
  unsigned* tickets;
  BatchMap m;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T ri = gld(r + i);
    const T zi = s + eps * ri;
    gst(z + i, zi);
    dd_fma(dots[0], double(ri), double(zi));
    dd_fma(dots[1], double(ri), double(ri));
  }
  __device__ __forceinline__ void finish(DD (&d)[2]) const {
    PcgState* Sb = S;
    batch_sys_reduce<2>(d, partials, tickets, m, [Sb](int sys, const double* v) {
      PcgState* St = Sb + sys;
      St->rho_prev = St->rho;
      St->rho = round_to<T>(v[0]);
      const int64_t k = St->iter;
      double rr = St->rr;  // ‖r_0‖² from the init
      if (k > 0) {
        rr = round_to<T>(v[1]);
        St->rr = rr;
        if (St->hist) St->hist[k] = double(tsqrt<T>(T(rr)));
      }
      int code = 0;
      if (k >= St->max_iter) {
        code = 2;
      } else {
        const double rn = double(tsqrt<T>(T(rr)));
        if (rn < St->atol) code = 1;
        else if (!(rn == rn) || rn == INFINITY) code = 3;
      }
      if (code) St->done = code;
    });
  }
};

// KC: q = A p ; π_k = p·q -> α_k = ρ_k/π_k, iteration k+1 (EpiQ<INC>::fin)
template <typename T>
struct EpiQB {
  static constexpr int NDOT = 1;
  static constexpr bool CUSTOM_FINISH = true;
  T* q;
  const T* p;
  PcgState* S;
  double* partials;
  unsigned* tickets;
  BatchMap m;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    gst(q + i, s);
    dd_fma(dots[0], double(gld(p + i)), double(s));
  }
  __device__ __forceinline__ void finish(DD (&d)[1]) const {
    PcgState* Sb = S;
    batch_sys_reduce<1>(d, partials, tickets, m, [Sb](int sys, const double* v) {
      PcgState* St = Sb + sys;
      const double pq = round_to<T>(v[0]);
      St->pq = pq;
      St->alpha = double(T(St->rho) / T(pq));
      St->iter = St->iter + 1;
    });
  }
};

// UP: x += α_{k-1} p_{k-1} (k > 0) ; p_k = p_{k-1}β + z with β = ρ_k/ρ_{k-1} (k_update_p_g's
// expressions), one 256-row tile of one system per workgroup
template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_update_p(BatchMap m, const PcgState* S, const T* __restrict__ z,
                                                             T* __restrict__ p, T* __restrict__ x) {
  const int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  const T zi = z[i], pi = p[i], xi = x[i];
  const PcgState* St = S + m.etile_sys[blockIdx.x];
  if (St->done) return;
  const bool first = St->iter == 0;
  const T beta = first ? T(0) : T(St->rho) / T(St->rho_prev);
  const T alpha = T(St->alpha);
  if (!first) x[i] = xi + alpha * pi;
  p[i] = first ? zi : (pi * beta) + zi;
}

// UR: r_{k+1} = r_k - α_k q
template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_update_r(BatchMap m, const PcgState* S, const T* __restrict__ q,
                                                             T* __restrict__ r) {
  const int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  const T ri = r[i], qi = q[i];
  const PcgState* St = S + m.etile_sys[blockIdx.x];
  if (St->done) return;
  r[i] = ri - T(St->alpha) * qi;
}

// ---- consumer-sum mode (windows whose systems have <= 128 tiles each): KB / KC only store
// per-tile partials (grid_partial_groups, gsz = 1: no tickets) and every UP / UR workgroup sums its
// system's tile partials itself (group_sum_dd, one wave for <= 256) ------------------------------
// init: r_0 = b - A x0 ; per-tile partials of ‖r_0‖², ‖b‖²
template <typename T>
struct EpiResidTile {
  static constexpr int NDOT = 2;
  static constexpr bool GROUPS = true;
  T* r;
  const T* b;
  double* partials;
  unsigned* ticket;
  double* group_out;
  int gsz;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t i, T s, DD* dots) const {
    const T bi = gld(b + i);
    const T ri = bi - s;
    gst(r + i, ri);
    dd_fma(dots[0], double(ri), double(ri));
    dd_fma(dots[1], double(bi), double(bi));
  }
  __device__ __forceinline__ void fin(const double*) const {}
};

// one workgroup per system: the init state from the system's tile partials (EpiResid::fin)
template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_init(PcgState* S, const int32_t* __restrict__ tile0,
                                                         const double* __restrict__ gi) {
  const int sys = blockIdx.x;
  const int t0 = tile0[sys], t1 = tile0[sys + 1];
  double v[2];
  group_sum_dd<2>(gi + size_t(t0) * 4, t1 - t0, v);
  if (threadIdx.x) return;
  PcgState* St = S + sys;
  St->rr = round_to<T>(v[0]);
  St->bb = round_to<T>(v[1]);
  const double bn = double(tsqrt<T>(T(St->bb)));
  St->atol = fmax(0.0, St->rtol * bn);
  St->rho = St->rr;
  St->alpha = 0.0;
  St->iter = 0;
  St->done = (bn == 0.0) ? 1 : 0;
  if (St->hist) St->hist[0] = double(tsqrt<T>(T(St->rr)));
}

// consumer-sum mode: UP of the split schedule (k_update_p_g) for the tile's system, summing the
// system's tile partials itself
template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_update_p_sums(BatchMap m, PcgState* S, const double* __restrict__ gz,
                                                             const T* __restrict__ z, T* __restrict__ p,
                                                             T* __restrict__ x) {
  const int sys = m.etile_sys[blockIdx.x];
  PcgState* St = S + sys;
  // `done` is loaded once and tested only after the group sums: group_sum_dd may hold workgroup
  // barriers, and this system's first workgroup can write `done` during this launch
  const int32_t done = St->done;
  const int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  const T zi = z[i], pi = p[i], xi = x[i];
  const int t0 = m.tile0[sys], t1 = m.tile0[sys + 1];
  const int64_t k = St->iter;
  double v[2];
  group_sum_dd<2>(gz + size_t(t0) * 4, t1 - t0, v);
  if (done) return;
  const double rho = round_to<T>(v[0]);
  const double rr = k > 0 ? round_to<T>(v[1]) : St->rr;
  int code = 0;
  if (k >= St->max_iter) {
    code = 2;
  } else {
    const double rn = double(tsqrt<T>(T(rr)));
    if (rn < St->atol) code = 1;
    else if (!(rn == rn) || rn == INFINITY) code = 3;
  }
  if (int64_t(blockIdx.x) == int64_t(t0) * m.bs && threadIdx.x == 0) {
    if (k > 0) {
      St->rr = rr;
      if (St->hist) St->hist[k] = double(tsqrt<T>(T(rr)));
    }
    if (code) St->done = code;
  }
  if (code) return;
  const bool first = k == 0;
  const T beta = first ? T(0) : T(rho) / T(St->rho);
  const T alpha = T(St->alpha);
  if (!first) x[i] = xi + alpha * pi;
  p[i] = first ? zi : (pi * beta) + zi;
}

// consumer-sum mode: UR of the split schedule (k_update_r_g) for the tile's system
template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_update_r_sums(BatchMap m, PcgState* S, const double* __restrict__ gz,
                                                             const double* __restrict__ gq, const T* __restrict__ q,
                                                             T* __restrict__ r) {
  const int sys = m.etile_sys[blockIdx.x];
  PcgState* St = S + sys;
  if (St->done) return;
  const int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  const T ri = r[i], qi = q[i];
  const int t0 = m.tile0[sys], t1 = m.tile0[sys + 1];
  double vz[2], vq[1];
  group_sum_dd<2>(gz + size_t(t0) * 4, t1 - t0, vz);
  group_sum_dd<1>(gq + size_t(t0) * 2, t1 - t0, vq);
  const double rho = round_to<T>(vz[0]);
  const double pq = round_to<T>(vq[0]);
  const T alpha = T(rho) / T(pq);
  if (int64_t(blockIdx.x) == int64_t(t0) * m.bs && threadIdx.x == 0) {
    St->rho_prev = St->rho;
    St->rho = rho;
    St->pq = pq;
    St->alpha = double(alpha);
    St->iter = St->iter + 1;
  }
  r[i] = ri - alpha * qi;
}


template <typename T>
__global__ void __launch_bounds__(kThreads) k_batch_x_fixup(BatchMap m, const PcgState* S, const T* __restrict__ p,
                                                            T* __restrict__ x) {
  const PcgState* St = S + m.etile_sys[blockIdx.x];
  if (St->iter < 1 || St->bb == 0.0) return;
  const int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x;
  x[i] = x[i] + T(St->alpha) * p[i];
}

// block-diagonal assembly: rows [0, cnt) of one system at its row offset (rows >= nb empty)
__global__ void k_cat_rowptr(int64_t cnt, int64_t nb, const int32_t* __restrict__ rp, int32_t e0,
                             int32_t* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < cnt; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = rp[i < nb ? i : nb] + e0;
}
__global__ void k_cat_colind(int64_t nnz, const int32_t* __restrict__ c, int32_t off, int32_t* __restrict__ out) {
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < nnz; k += int64_t(gridDim.x) * blockDim.x)
    out[k] = c[k] + off;
}

}  // namespace lspcg

struct lspcg_batch {
  lspcg_ctx* ctx = nullptr;
  int nsys = 0;
  int bs = 1;
  int dtype = LSPCG_F64;
  lspcg_mat* Acat = nullptr;
  lspcg_mat* Lcat = nullptr;
  lspcg_solver* s = nullptr;  // solver of the block-diagonal system: views, vectors, stream
  std::vector<int64_t> off, n;  // scalar row offset and size of every system
  int64_t ntot = 0;             // padded scalar rows
  int32_t* etile_sys = nullptr;
  int32_t* tile0 = nullptr;
  int32_t* tk0 = nullptr;
  double* partials = nullptr;  // per-tile dot partials (<= 2 dots, DD each)
  unsigned* tickets = nullptr;  // per system: top line + one line per kTicketGroup tiles (batch_sys_reduce)
  bool sums = false;            // consumer-sum reductions (every system <= 128 tiles; LSPCG_BATCH_REDUCE)
  bool small = false;           // every system fits the one-workgroup solve: one launch, one workgroup per system
  int64_t max_n = 0;
  int32_t* boff = nullptr;      // [nsys] scalar row offset / size of each system (small mode)
  int32_t* bn = nullptr;
  double* gsum = nullptr;       // consumer-sum partials: init (2 dots) | KB (2 dots) | KC (1 dot), per tile
  int64_t ntiles = 0;
  PcgState* S = nullptr;
  PcgState* hS = nullptr;  // pinned: 2 poll slots x nsys
  double* dhist = nullptr;
  int64_t dhist_cap = 0;
  std::map<int, hipGraphExec_t> graphs;
  std::map<int, hipGraph_t> graph_defs;
};

namespace lspcg {

static BatchMap batch_map(const lspcg_batch* bt) { return BatchMap{bt->etile_sys, bt->tile0, bt->tk0, bt->bs}; }

// SpMV of iteration view w over the block-diagonal system, one row tile per workgroup
template <typename T, class Pro, class Epi>
static int launch_it_tiles(lspcg_solver* s, int w, const T* x, Pro pro, Epi epi, hipStream_t st) {
  const SellPattern* P = s->sp[w];
  if (!P) return LSPCG_ERR_UNSUPPORTED;
  if constexpr (sizeof(T) == 8) {
    if (s->svd[w] == LSPCG_F32) {
      launch_spmv_sell_cfg<T, float>(*P, s->sv[w], GatherVec<T>{x}, pro, epi, st, true);
      return LSPCG_OK;
    }
  }
  launch_spmv_sell_cfg<T, T>(*P, s->sv[w], GatherVec<T>{x}, pro, epi, st, true);
  return LSPCG_OK;
}

template <typename T>
static int enqueue_batch_init(lspcg_batch* bt, hipStream_t st) {
  lspcg_solver* s = bt->s;
  if (bt->sums) {
    int rc = launch_it_tiles<T>(s, 0, static_cast<const T*>(s->x), ProNone{},
                                EpiResidTile<T>{static_cast<T*>(s->r), static_cast<const T*>(s->b), nullptr, nullptr,
                                                bt->gsum, 1},
                                st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_batch_init<T>, dim3(bt->nsys), dim3(kThreads), 0, st, bt->S,
                       static_cast<const int32_t*>(bt->tile0), static_cast<const double*>(bt->gsum));
    LSPCG_HIP(hipGetLastError());
    return LSPCG_OK;
  }
  return launch_it_tiles<T>(s, 0, static_cast<const T*>(s->x), ProNone{},
                            EpiResidB<T>{static_cast<T*>(s->r), static_cast<const T*>(s->b), bt->S, bt->partials,
                                         bt->tickets, batch_map(bt)},
                            st);
}

template <typename T>
static int enqueue_batch_iteration(lspcg_batch* bt, hipStream_t st) {
  lspcg_solver* s = bt->s;
  T* x = static_cast<T*>(s->x);
  T* r = static_cast<T*>(s->r);
  T* z = static_cast<T*>(s->z);
  T* t = static_cast<T*>(s->t);
  T* p = static_cast<T*>(s->p);
  T* q = static_cast<T*>(s->q);
  const BatchMap m = batch_map(bt);
  const ProTile pro{bt->S, m};
  const dim3 eg(unsigned(bt->ntot / kThreads));
  int rc = launch_it_tiles<T>(s, 2, static_cast<const T*>(r), pro, EpiT<T, false>{t, nullptr}, st);
  if (rc) return rc;
  if (bt->sums) {
    double* gz = bt->gsum + 4 * bt->ntiles;
    double* gq = bt->gsum + 8 * bt->ntiles;
    rc = launch_it_tiles<T>(s, 1, static_cast<const T*>(t), pro,
                            EpiZG<T, false>{z, r, nullptr, T(s->eps), nullptr, nullptr, gz, 1}, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_batch_update_p_sums<T>, eg, dim3(kThreads), 0, st, m, bt->S, static_cast<const double*>(gz),
                       static_cast<const T*>(z), p, x);
    rc = launch_it_tiles<T>(s, 0, static_cast<const T*>(p), pro, EpiQG<T>{q, p, nullptr, nullptr, gq, 1}, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_batch_update_r_sums<T>, eg, dim3(kThreads), 0, st, m, bt->S, static_cast<const double*>(gz),
                       static_cast<const double*>(gq), static_cast<const T*>(q), r);
    LSPCG_HIP(hipGetLastError());
    return LSPCG_OK;
  }
  rc = launch_it_tiles<T>(s, 1, static_cast<const T*>(t), pro,
                          EpiZB<T>{z, r, T(s->eps), bt->S, bt->partials, bt->tickets, m}, st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_batch_update_p<T>, eg, dim3(kThreads), 0, st, m, static_cast<const PcgState*>(bt->S),
                     static_cast<const T*>(z), p, x);
  rc = launch_it_tiles<T>(s, 0, static_cast<const T*>(p), pro, EpiQB<T>{q, p, bt->S, bt->partials, bt->tickets, m},
                          st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_batch_update_r<T>, eg, dim3(kThreads), 0, st, m, static_cast<const PcgState*>(bt->S),
                     static_cast<const T*>(q), r);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

// every system of the window in its own workgroup (k_pcg_small in batch mode): the whole loop in
// one launch; rows per thread / threads from the window's largest system (launch_small's rule)
template <typename T>
static int launch_batch_small(lspcg_batch* bt, hipStream_t st) {
  lspcg_solver* s = bt->s;
  const CsrView A = csr_view(s, 0, s->Av), L = csr_view(s, 1, s->Lv), LT = csr_view(s, 2, s->LTv);
  auto* x = static_cast<T*>(s->x);
  auto* r = static_cast<T*>(s->r);
  auto* p = static_cast<T*>(s->p);
  const T* d = static_cast<const T*>(s->d);
  const int64_t n = bt->max_n;
  const dim3 g(unsigned(bt->nsys));
  const size_t lds = 3 * sizeof(T) * size_t(n);
  auto go = [&](auto rows, auto threads) {
    constexpr int R = decltype(rows)::value;
    constexpr int TH = decltype(threads)::value;
    hipLaunchKernelGGL((k_pcg_small<T, LSPCG_PRECOND_EXT_SPAI, R, TH>), g, dim3(TH), lds, st, int32_t(n), bt->S, A, L,
                       LT, d, x, r, p, static_cast<const int32_t*>(bt->boff), static_cast<const int32_t*>(bt->bn));
  };
  using T512 = std::integral_constant<int, kSmallThreads>;
  using T1024 = std::integral_constant<int, kSmallThreadsBig>;
  if (n <= kSmallThreads) go(std::integral_constant<int, 1>{}, T512{});
  else if (n <= 2 * kSmallThreads) go(std::integral_constant<int, 2>{}, T512{});
  else if (n <= 2 * kSmallThreadsBig) go(std::integral_constant<int, 2>{}, T1024{});
  else go(std::integral_constant<int, 3>{}, T1024{});
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

static int get_batch_graph(lspcg_batch* bt, int chunk, hipGraphExec_t* out) {
  auto it = bt->graphs.find(chunk);
  if (it != bt->graphs.end()) {
    *out = it->second;
    return LSPCG_OK;
  }
  hipStream_t st = bt->s->stream;
  hipGraph_t g = nullptr;
  LSPCG_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  int rc = LSPCG_OK;
  for (int i = 0; i < chunk && rc == LSPCG_OK; ++i)
    rc = bt->dtype == LSPCG_F64 ? enqueue_batch_iteration<double>(bt, st) : enqueue_batch_iteration<float>(bt, st);
  hipError_t e = hipStreamEndCapture(st, &g);
  if (rc) return rc;
  LSPCG_HIP(e);
  hipGraphExec_t ex = nullptr;
  LSPCG_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  bt->graphs[chunk] = ex;
  bt->graph_defs[chunk] = g;
  *out = ex;
  return LSPCG_OK;
}

// block-diagonal copy of M[0..nsys) with system k's block rows starting at brow[k] (padded)
static int cat_matrices(lspcg_ctx* ctx, int nsys, const lspcg_mat* const* M, const std::vector<int64_t>& brow,
                        lspcg_mat** out) {
  const int bs = M[0]->block_size;
  int64_t nnz = 0;
  for (int k = 0; k < nsys; ++k) nnz += M[k]->nnzb;
  LSPCG_CHECK(nnz < (int64_t(1) << 31), LSPCG_ERR_ARG, "batch: more than 2^31 stored blocks in the window");
  lspcg_mat* C = nullptr;
  if (int rc = mat_alloc(ctx, brow[nsys], nnz, bs, M[0]->dtype, &C)) return rc;
  hipStream_t st = ctx->stream;
  const size_t vb = (M[0]->dtype == LSPCG_F32 ? 4 : 8) * size_t(bs) * bs;
  int64_t e0 = 0;
  for (int k = 0; k < nsys; ++k) {
    const int64_t cnt = brow[k + 1] - brow[k] + (k == nsys - 1 ? 1 : 0);
    hipLaunchKernelGGL(k_cat_rowptr, dim3(unsigned(std::min<int64_t>((cnt + 255) / 256, 1024))), dim3(256), 0, st, cnt,
                       M[k]->nb, static_cast<const int32_t*>(M[k]->rowptr), int32_t(e0), C->rowptr + brow[k]);
    if (M[k]->nnzb) {
      hipLaunchKernelGGL(k_cat_colind, dim3(unsigned(std::min<int64_t>((M[k]->nnzb + 255) / 256, 1024))), dim3(256), 0,
                         st, M[k]->nnzb, static_cast<const int32_t*>(M[k]->colind), int32_t(brow[k]), C->colind + e0);
      LSPCG_HIP(hipMemcpyAsync(static_cast<char*>(C->vals) + vb * e0, M[k]->vals, vb * M[k]->nnzb,
                               hipMemcpyDeviceToDevice, st));
    }
    e0 += M[k]->nnzb;
  }
  LSPCG_HIP(hipGetLastError());
  LSPCG_HIP(hipStreamSynchronize(st));
  *out = C;
  return LSPCG_OK;
}

}  // namespace lspcg

extern "C" {

int lspcg_batch_destroy(lspcg_batch* bt) {
  if (!bt) return LSPCG_OK;
  (void)hipSetDevice(bt->ctx->device);
  if (bt->s) (void)hipStreamSynchronize(bt->s->stream);
  for (auto& kv : bt->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : bt->graph_defs) (void)hipGraphDestroy(kv.second);
  if (bt->s) lspcg_solver_destroy(bt->s);
  if (bt->Acat) lspcg_mat_destroy(bt->Acat);
  if (bt->Lcat) lspcg_mat_destroy(bt->Lcat);
  for (void* v : {(void*)bt->boff, (void*)bt->bn, (void*)bt->etile_sys, (void*)bt->tile0, (void*)bt->tk0, (void*)bt->gsum, (void*)bt->partials, (void*)bt->tickets, (void*)bt->S,
                  (void*)bt->dhist})
    (void)hipFree(v);
  (void)hipHostFree(bt->hS);
  delete bt;
  return LSPCG_OK;
}

int lspcg_batch_create(lspcg_ctx* ctx, int nsys, const lspcg_mat* const* A, const lspcg_mat* const* L,
                       double epsilon, lspcg_batch** out) {
  LSPCG_CHECK(ctx && A && L && out && nsys >= 1, LSPCG_ERR_ARG, "batch_create: NULL argument or nsys < 1");
  for (int k = 0; k < nsys; ++k) {
    LSPCG_CHECK(A[k] && L[k], LSPCG_ERR_ARG, "batch_create: NULL matrix " + std::to_string(k));
    LSPCG_CHECK(A[k]->dtype == A[0]->dtype && L[k]->dtype == A[0]->dtype, LSPCG_ERR_ARG,
                "batch_create: every A and L must have one dtype");
    LSPCG_CHECK(A[k]->block_size == A[0]->block_size && L[k]->block_size == A[0]->block_size, LSPCG_ERR_ARG,
                "batch_create: every A and L must have one block size");
    LSPCG_CHECK(L[k]->n == A[k]->n && A[k]->n >= 1, LSPCG_ERR_ARG,
                "batch_create: system " + std::to_string(k) + ": L and A differ in size or are empty");
  }
  LSPCG_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<lspcg_batch, int (*)(lspcg_batch*)> bt(new lspcg_batch(), lspcg_batch_destroy);
  bt->ctx = ctx;
  bt->nsys = nsys;
  bt->bs = A[0]->block_size;
  bt->dtype = A[0]->dtype;
  // block-row offsets, each system padded to whole SpMV row tiles (kSellWG block rows)
  std::vector<int64_t> brow(nsys + 1, 0);
  for (int k = 0; k < nsys; ++k) brow[k + 1] = brow[k] + (A[k]->nb + kSellWG - 1) / kSellWG * kSellWG;
  LSPCG_CHECK(brow[nsys] * bt->bs < (int64_t(1) << 31), LSPCG_ERR_ARG, "batch_create: window exceeds 2^31 rows");
  for (int k = 0; k < nsys; ++k) {
    bt->off.push_back(brow[k] * bt->bs);
    bt->n.push_back(A[k]->n);
  }
  bt->ntot = brow[nsys] * bt->bs;
  if (int rc = cat_matrices(ctx, nsys, A, brow, &bt->Acat)) return rc;
  if (int rc = cat_matrices(ctx, nsys, L, brow, &bt->Lcat)) return rc;
  // one workgroup per system when every system fits the one-workgroup solve (scalar views; its
  // row and LDS bounds, small_path); LSPCG_BATCH_SMALL=0 keeps the lockstep phases.  Decided before
  // the views are built: that mode reads 4-entry-group SELL copies, not SELL-DIA
  for (int k = 0; k < nsys; ++k) bt->max_n = std::max<int64_t>(bt->max_n, bt->n[k]);
  {
    const char* e = std::getenv("LSPCG_BATCH_SMALL");
    const char* en = std::getenv("LSPCG_SMALL_N");
    const int64_t small_n = en ? std::max<int64_t>(0, std::atoll(en)) : kSmallNDefault;
    const int64_t row_cap = int64_t(kSmallThreadsBig) * 3;
    bt->small = !(e && e[0] == '0') && bt->bs == 1 && bt->max_n <= std::min<int64_t>(row_cap, small_n) &&
                3 * bt->max_n * int64_t(esize(bt->dtype)) <= kSmallLds;
  }
  if (int rc = solver_create(ctx, bt->Acat, LSPCG_PRECOND_EXT_SPAI, !bt->small, false, &bt->s)) return rc;
  if (int rc = lspcg_solver_set_spai(bt->s, bt->Lcat, epsilon, nullptr)) return rc;
  LSPCG_CHECK(bt->s->sp[0] && bt->s->sp[1] && bt->s->sp[2], LSPCG_ERR_UNSUPPORTED,
              "batch_create: no SELL view of the block-diagonal system (irregular rows): solve one by one");
  // tile maps
  const int64_t ntiles = brow[nsys] / kSellWG;
  std::vector<int32_t> esys(size_t(bt->ntot / kThreads)), t0(nsys + 1);
  for (int k = 0; k < nsys; ++k) {
    t0[k] = int32_t(brow[k] / kSellWG);
    for (int64_t e = bt->off[k] / kThreads; e < (bt->off[k] + (brow[k + 1] - brow[k]) * bt->bs) / kThreads; ++e)
      esys[size_t(e)] = k;
  }
  t0[nsys] = int32_t(ntiles);
  std::vector<int32_t> tk(nsys);
  int64_t lines = 0;
  for (int k = 0; k < nsys; ++k) {
    tk[k] = int32_t(lines);
    lines += 1 + (t0[k + 1] - t0[k] + kTicketGroup - 1) / kTicketGroup;
  }
  LSPCG_HIP(hipMalloc(&bt->tk0, sizeof(int32_t) * nsys));
  LSPCG_HIP(hipMemcpy(bt->tk0, tk.data(), sizeof(int32_t) * nsys, hipMemcpyHostToDevice));
  LSPCG_HIP(hipMalloc(&bt->etile_sys, sizeof(int32_t) * esys.size()));
  LSPCG_HIP(hipMalloc(&bt->tile0, sizeof(int32_t) * t0.size()));
  LSPCG_HIP(hipMemcpy(bt->etile_sys, esys.data(), sizeof(int32_t) * esys.size(), hipMemcpyHostToDevice));
  LSPCG_HIP(hipMemcpy(bt->tile0, t0.data(), sizeof(int32_t) * t0.size(), hipMemcpyHostToDevice));
  LSPCG_HIP(hipMalloc(&bt->partials, sizeof(double) * 4 * ntiles));
  // reductions: consumer sums when every system has <= 128 tiles (C5 heat, <= 117 tiles: 25.6 vs
  // 26.8 us per lockstep iteration), else per-system last arrivers (8 x Poisson 256^2, 256 tiles:
  // 47.1 vs 49.9); LSPCG_BATCH_REDUCE=0 / 1 forces either
  int max_nt = 0;
  for (int k = 0; k < nsys; ++k) max_nt = std::max(max_nt, t0[k + 1] - t0[k]);
  bt->sums = max_nt <= 128;
  if (const char* e = std::getenv("LSPCG_BATCH_REDUCE")) bt->sums = e[0] == '1';
  bt->ntiles = ntiles;
  LSPCG_HIP(hipMalloc(&bt->gsum, sizeof(double) * 10 * ntiles));
  if (bt->small) {
    std::vector<int32_t> ho(nsys), hn(nsys);
    for (int k = 0; k < nsys; ++k) {
      ho[k] = int32_t(bt->off[k]);
      hn[k] = int32_t(bt->n[k]);
    }
    LSPCG_HIP(hipMalloc(&bt->boff, sizeof(int32_t) * nsys));
    LSPCG_HIP(hipMalloc(&bt->bn, sizeof(int32_t) * nsys));
    LSPCG_HIP(hipMemcpy(bt->boff, ho.data(), sizeof(int32_t) * nsys, hipMemcpyHostToDevice));
    LSPCG_HIP(hipMemcpy(bt->bn, hn.data(), sizeof(int32_t) * nsys, hipMemcpyHostToDevice));
  }
  LSPCG_HIP(hipMalloc(&bt->tickets, sizeof(unsigned) * kTicketStride * lines));
  LSPCG_HIP(hipMemset(bt->tickets, 0, sizeof(unsigned) * kTicketStride * lines));
  LSPCG_HIP(hipMalloc(&bt->S, sizeof(PcgState) * nsys));
  LSPCG_HIP(hipHostMalloc(&bt->hS, 2 * sizeof(PcgState) * nsys, hipHostMallocDefault));
  *out = bt.release();
  return LSPCG_OK;
}

int lspcg_batch_solve(lspcg_batch* bt, const void* const* b, void* const* x, double rtol, int64_t max_iter,
                      int64_t* iters, int32_t* status, double* const* res_hist, double* t_solve_ms) {
  LSPCG_CHECK(bt && b && x && iters && status, LSPCG_ERR_ARG, "batch_solve: NULL argument");
  const int ns = bt->nsys;
  for (int k = 0; k < ns; ++k) LSPCG_CHECK(b[k] && x[k], LSPCG_ERR_ARG, "batch_solve: NULL vector " + std::to_string(k));
  lspcg_solver* s = bt->s;
  LSPCG_HIP(hipSetDevice(bt->ctx->device));
  hipStream_t st = s->stream;
  const size_t es = esize(bt->dtype);
  std::vector<int64_t> mi(ns), hoff(ns + 1, 0);
  for (int k = 0; k < ns; ++k) {
    mi[k] = max_iter > 0 ? max_iter : bt->n[k];
    hoff[k + 1] = hoff[k] + ((res_hist && res_hist[k]) ? mi[k] + 2 : 0);
  }
  if (hoff[ns] > bt->dhist_cap) {
    LSPCG_HIP(hipStreamSynchronize(st));
    (void)hipFree(bt->dhist);
    bt->dhist = nullptr;
    bt->dhist_cap = 0;
    LSPCG_HIP(hipMalloc(&bt->dhist, sizeof(double) * hoff[ns]));
    bt->dhist_cap = hoff[ns];
  }
  std::unique_lock<std::mutex> sub(submit_mutex());  // as in lspcg_solver_solve
  auto wait = [&sub](hipEvent_t e) {
    sub.unlock();
    const hipError_t r = hipEventSynchronize(e);
    sub.lock();
    return r;
  };
  LSPCG_HIP(hipEventRecord(s->ev_in, bt->ctx->stream));
  LSPCG_HIP(hipStreamWaitEvent(st, s->ev_in, 0));
  LSPCG_HIP(hipEventRecord(s->ev_t0, st));
  char* cb = static_cast<char*>(s->b);
  char* cx = static_cast<char*>(s->x);
  for (int k = 0; k < ns; ++k) {  // padding rows stay 0 (zeroed at creation, never written)
    LSPCG_HIP(hipMemcpyAsync(cb + es * bt->off[k], b[k], es * bt->n[k], hipMemcpyDeviceToDevice, st));
    LSPCG_HIP(hipMemcpyAsync(cx + es * bt->off[k], x[k], es * bt->n[k], hipMemcpyDeviceToDevice, st));
  }
  for (int k = 0; k < ns; ++k) {
    PcgState init{};
    init.rtol = rtol;
    init.eps = s->eps;
    init.hist = (res_hist && res_hist[k]) ? bt->dhist + hoff[k] : nullptr;
    init.max_iter = mi[k];
    bt->hS[k] = init;
  }
  LSPCG_HIP(hipMemcpyAsync(bt->S, bt->hS, sizeof(PcgState) * ns, hipMemcpyHostToDevice, st));
  int rc = bt->dtype == LSPCG_F64 ? enqueue_batch_init<double>(bt, st) : enqueue_batch_init<float>(bt, st);
  if (rc) return rc;

  // the poll loop of lspcg_solver_solve over every system's state: run while any system runs;
  // chunks sized from the slowest system's predicted remaining iterations (small mode: one launch)
  constexpr int max_chunk = 32;
  PcgState* const hs[2] = {bt->hS, bt->hS + ns};
  const hipEvent_t evp[2] = {s->ev_poll, s->ev_poll2};
  int64_t queued[2] = {0, 0};
  int head = 0, npend = 0;
  auto post = [&]() -> int {
    const int k = (head + npend) & 1;
    LSPCG_HIP(hipMemcpyAsync(hs[k], bt->S, sizeof(PcgState) * ns, hipMemcpyDeviceToHost, st));
    LSPCG_HIP(hipEventRecord(evp[k], st));
    queued[k] = 0;
    ++npend;
    return LSPCG_OK;
  };
  auto launch = [&](int c) -> int {
    hipGraphExec_t ex = nullptr;
    int r = get_batch_graph(bt, c, &ex);
    if (r) return r;
    LSPCG_HIP(hipGraphLaunch(ex, st));
    for (int j = 0; j < npend; ++j) queued[(head + j) & 1] += c;
    return post();
  };
  std::vector<PcgState> cur(ns);
  if (bt->small) {
    rc = bt->dtype == LSPCG_F64 ? launch_batch_small<double>(bt, st) : launch_batch_small<float>(bt, st);
    if (!rc) rc = post();
    if (rc) return rc;
    LSPCG_HIP(wait(evp[head]));
    std::copy(hs[head], hs[head] + ns, cur.begin());
  }
  if (!bt->small) {
    rc = post();
    if (!rc) rc = launch(4);
    if (rc) return rc;
  }
  std::vector<int64_t> last_it(ns, 0);
  std::vector<double> last_rr(ns, -1.0);
  int chunk = 4;
  for (; !bt->small;) {
    LSPCG_HIP(wait(evp[head]));
    std::copy(hs[head], hs[head] + ns, cur.begin());
    const int64_t inflight = queued[head];
    head ^= 1;
    --npend;
    int64_t rem = 0;  // largest predicted remaining count over the running systems
    bool unknown = false, running = false;
    for (int k = 0; k < ns; ++k) {
      const PcgState& c = cur[k];
      if (c.done) continue;
      running = true;
      int64_t rk = -1;
      if (last_rr[k] > 0 && c.iter > last_it[k] && c.rr > 0 && c.rr < last_rr[k]) {
        const double rate = std::log(c.rr / last_rr[k]) / double(c.iter - last_it[k]);
        const double need = std::log((c.atol * c.atol) / c.rr) / rate;
        rk = need > 0 ? int64_t(std::ceil(need)) : 1;
        rk = std::max<int64_t>(1, std::min<int64_t>(rk, mi[k] - c.iter));
      }
      if (c.iter > last_it[k] || last_rr[k] < 0) {
        last_it[k] = c.iter;
        last_rr[k] = c.rr;
      }
      if (rk < 0) unknown = true;
      else rem = std::max(rem, rk);
    }
    if (!running) break;
    if (unknown) rem = -1;
    if (rem >= 0) {
      const int64_t more = rem - inflight;
      if (more <= 0) {
        if (npend == 0) rc = launch(1);
        if (rc) return rc;
        continue;
      }
      int c = 1;
      while (c * 2 <= more && c < max_chunk) c *= 2;
      chunk = c;
    } else {
      chunk = std::min(max_chunk, chunk * 2);
    }
    rc = launch(chunk);
    if (rc) return rc;
  }
  const BatchMap m = batch_map(bt);
  if (bt->dtype == LSPCG_F64)
    hipLaunchKernelGGL(k_batch_x_fixup<double>, dim3(unsigned(bt->ntot / kThreads)), dim3(kThreads), 0, st, m, bt->S,
                       static_cast<const double*>(s->p), static_cast<double*>(s->x));
  else
    hipLaunchKernelGGL(k_batch_x_fixup<float>, dim3(unsigned(bt->ntot / kThreads)), dim3(kThreads), 0, st, m, bt->S,
                       static_cast<const float*>(s->p), static_cast<float*>(s->x));
  LSPCG_HIP(hipGetLastError());
  for (int k = 0; k < ns; ++k) {
    const char* src = (cur[k].bb == 0.0) ? cb : cx;  // scipy returns b when ‖b‖ = 0
    LSPCG_HIP(hipMemcpyAsync(x[k], src + es * bt->off[k], es * bt->n[k], hipMemcpyDeviceToDevice, st));
  }
  LSPCG_HIP(hipEventRecord(s->ev_t1, st));
  LSPCG_HIP(hipEventRecord(s->ev_out, st));
  LSPCG_HIP(hipStreamWaitEvent(bt->ctx->stream, s->ev_out, 0));
  LSPCG_HIP(wait(s->ev_t1));
  float ms = 0.f;
  LSPCG_HIP(hipEventElapsedTime(&ms, s->ev_t0, s->ev_t1));
  if (t_solve_ms) *t_solve_ms = ms;
  bool all = true;
  for (int k = 0; k < ns; ++k) {
    const PcgState& f = cur[k];
    const int64_t it = (f.done == 3) ? mi[k] : f.iter;
    iters[k] = it;
    status[k] = f.done == 1 ? LSPCG_OK : LSPCG_NOT_CONVERGED;
    all = all && f.done == 1;
    if (res_hist && res_hist[k]) {
      const int64_t cnt = std::min<int64_t>(f.iter, mi[k]) + 1;
      LSPCG_HIP(hipMemcpy(res_hist[k], bt->dhist + hoff[k], sizeof(double) * cnt, hipMemcpyDeviceToHost));
      for (int64_t j = cnt; j <= it; ++j) res_hist[k][j] = NAN;
    }
  }
  return all ? LSPCG_OK : LSPCG_NOT_CONVERGED;
}

}  // extern "C"
