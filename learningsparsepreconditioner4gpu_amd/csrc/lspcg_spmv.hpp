// Staged CSR / BSR(3x3) SpMV for gfx950 with fused prologue / epilogue.
//
// Layout (DESIGN.md "SpMV"): one 256-thread workgroup owns RB = 256/bs consecutive
// block rows (256 scalar rows for CSR, 85x3 for BSR3).  Its entries
// [rowptr[b0], rowptr[b1]) are contiguous in HBM, so the workgroup streams them in
// chunks of <= kSpmvCap scalar entries: every lane loads value + column index with
// unit stride (coalesced), gathers x[col], multiplies and writes the product to LDS.
// After a barrier each thread owns ONE scalar row and adds that row's products in
// index order -- the exact summation order of scipy's csr_matvec, so the result is
// bit-identical to it (no FMA contraction: -ffp-contract=off).  Chunks are processed
// in order and the running sums stay in registers, so rows that straddle a chunk
// boundary keep the sequential order.  The epilogue consumes the row sum in
// registers (fused AXPY / scaling / dot products), so no separate vector pass is
// needed for them.
#pragma once

#include <algorithm>
#include <type_traits>

#include "lspcg_internal.hpp"

namespace lspcg {

template <typename T, typename VT, int BS>
struct SpmvArgs {
  int64_t nb;             // block rows
  const int32_t* rowptr;  // [nb+1]
  const int32_t* colind;  // [nnzb]
  const VT* vals;         // [nnzb*BS*BS] storage type (VT = float for compact fp64 matrices)
};

// Gather functors: x_j as seen by the SpMV.  prepare() runs once per workgroup after the
// prologue (it may read solver state); operator() is evaluated for every gathered column.
template <typename T>
struct GatherVec {
  const T* x;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ T operator()(int64_t j) const { return gld(x + j); }
};

inline int64_t spmv_grid(int64_t nb, int bs) {  // grid of the production configuration (<= n/255 + 1)
  const int rb = 256 / bs;
  return (nb + rb - 1) / rb;
}

// Prologue functors: return true when the whole workgroup must exit (uniform).
struct ProNone {
  __device__ __forceinline__ bool exit() const { return false; }
};

// Epilogue with no dot product: y[r] = s.
template <typename T>
struct EpiStore {
  static constexpr int NDOT = 0;
  T* y;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t r, T s, DD*) const { gst(y + r, s); }
  __device__ __forceinline__ void fin(const double*) const {}
  double* partials = nullptr;
  unsigned* ticket = nullptr;
};

// Epilogue of the reordered standalone SpMV (lspcg_spmv on P A Pᵀ): row r of the permuted system is
// row perm[r / BS] (block row) of the caller's, so the result goes straight to its place:
// y[BS perm[r / BS] + r % BS] = s (no scatter pass).
template <typename T, int BS>
struct EpiStorePerm {
  static constexpr int NDOT = 0;
  T* y;
  const int32_t* perm;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ void row(int64_t r, T s, DD*) const {
    const int64_t I = r / BS;
    gst(y + int64_t(BS) * perm[I] + (r - I * BS), s);
  }
  __device__ __forceinline__ void fin(const double*) const {}
  double* partials = nullptr;
  unsigned* ticket = nullptr;
};

// Entries are loaded in groups of 4 consecutive scalar entries (16-B column-index loads,
// 2x16-B fp64 value loads) with NO per-element predicate: group indices are clamped to the
// chunk, and the index/value arrays carry kEntryPad padding entries (column 0, value 0),
// so every load is in bounds and the compiler issues all of them before the first wait.
using i32x4 = int __attribute__((ext_vector_type(4)));
using f64x2 = double __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));

template <typename T>
struct Vec4;
template <>
struct Vec4<double> {
  template <bool NT>
  __device__ static __forceinline__ void load(const double* p, double (&v)[4]) {
    const f64x2* q = reinterpret_cast<const f64x2*>(p);
    const f64x2 a = NT ? __builtin_nontemporal_load(q) : q[0];
    const f64x2 b = NT ? __builtin_nontemporal_load(q + 1) : q[1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ static __forceinline__ void store(double* p, const double (&v)[4]) {
    reinterpret_cast<double2*>(p)[0] = make_double2(v[0], v[1]);
    reinterpret_cast<double2*>(p)[1] = make_double2(v[2], v[3]);
  }
};
template <>
struct Vec4<float> {
  template <bool NT>
  __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p);
    const f32x4 a = NT ? __builtin_nontemporal_load(q) : q[0];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  __device__ static __forceinline__ void store(float* p, const float (&v)[4]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  }
};

// Epilogues with GROUPS = true finish their dots with grid_partial_groups (the consumers sum the
// group totals), the others with the last-arriver grid_reduce_dd + fin().
template <class E, class = void>
struct epi_groups : std::false_type {};
template <class E>
struct epi_groups<E, std::void_t<decltype(E::GROUPS)>> : std::bool_constant<E::GROUPS> {};

// Epilogues with CUSTOM_FINISH = true reduce their dots themselves (epi.finish(d); batched solves)
template <class E, class = void>
struct epi_custom : std::false_type {};
template <class E>
struct epi_custom<E, std::void_t<decltype(E::CUSTOM_FINISH)>> : std::bool_constant<E::CUSTOM_FINISH> {};

template <class Epi>
__device__ __forceinline__ void finish_epi_dots(DD (&d)[Epi::NDOT > 0 ? Epi::NDOT : 1], Epi& epi) {
  if constexpr (Epi::NDOT > 0) {
    if constexpr (epi_custom<Epi>::value)
      epi.finish(d);
    else if constexpr (epi_groups<Epi>::value)
      grid_partial_groups<Epi::NDOT>(d, epi.partials, epi.ticket, epi.gsz, epi.group_out);
    else
      grid_reduce_dd<Epi::NDOT>(d, epi.partials, epi.ticket, [&](const double* vals) { epi.fin(vals); });
  }
}

// THREADS = workgroup size (one scalar row per thread), GPT = groups of 4 entries each
// thread stages per chunk (chunk = THREADS*GPT*4 entries), NT = non-temporal matrix loads.
// LANEC: lane-consecutive staging (lane t <-> entry c0 + t + u*THREADS, 4/8-B loads): one
// gather instruction then covers ~64/15 consecutive rows, i.e. few distinct cache lines.
// XCD: persistent grid (multiple of 8) whose workgroups b, b+8, ... (one XCD under the observed
// round-robin dispatch) walk one contiguous eighth of the row tiles, so each XCD's 4 MiB L2
// only holds the gather window of its own slice.  Placement is a speed hint only.
template <typename T, typename VT, int BS, int THREADS, int GPT, bool NT, class Pro, class Gx, class Epi,
          bool LANEC = false, bool XCD = false>
__global__ void __launch_bounds__(THREADS) k_spmv(SpmvArgs<T, VT, BS> a, Pro pro, Gx gx, Epi epi) {
  constexpr int BB = BS * BS;
  constexpr int CAPG = THREADS * GPT;             // groups of 4 entries per chunk
  constexpr int RB = THREADS / BS;                // block rows per workgroup
  constexpr int PERG = GPT;
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  constexpr int kThreads = THREADS;
  __shared__ __attribute__((aligned(16))) T prod[CAPG * 4];

  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();

  const int tid = threadIdx.x;
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  const int64_t ntiles = (a.nb + RB - 1) / RB;
  // Reducing launches are capped at a resident grid (the dot's per-workgroup ticket and
  // the last arriver's partial sweep then cost once per workgroup, not once per tile);
  // each workgroup walks tiles blockIdx.x, blockIdx.x + gridDim.x, ... (or its XCD slice)
  int64_t t_first = blockIdx.x, t_end = ntiles, t_step = gridDim.x;
  if constexpr (XCD) {
    const int64_t per = gridDim.x >> 3;
    const int64_t t8 = (ntiles + 7) >> 3;
    const int64_t x = blockIdx.x & 7;
    t_first = x * t8 + (blockIdx.x >> 3);
    t_end = (x + 1) * t8 < ntiles ? (x + 1) * t8 : ntiles;
    t_step = per;
  }
  for (int64_t tile = t_first; tile < t_end; tile += t_step) {
  const int64_t b0 = tile * RB;
  const int64_t b1 = b0 + RB < a.nb ? b0 + RB : a.nb;
  const int64_t e0 = int64_t(a.rowptr[b0]) * BB;
  const int64_t e1 = int64_t(a.rowptr[b1]) * BB;
  const bool active = tid < (b1 - b0) * BS;
  const int64_t I = b0 + tid / BS;
  const int comp = tid % BS;
  int64_t kb_beg = 0, kb_end = 0;
  if (active) {
    kb_beg = int64_t(a.rowptr[I]) * BB;   // scalar-entry range of this thread's block row
    kb_end = int64_t(a.rowptr[I + 1]) * BB;
  }
  T acc = T(0);
  const int64_t G0 = e0 >> 2;
  const int64_t G1 = (e1 + 3) >> 2;

  for (int64_t gs = G0; gs < G1; gs += CAPG) {
    const int64_t ge = gs + CAPG < G1 ? gs + CAPG : G1;
    if constexpr (LANEC) {
      // entries [4gs, 4ge) clamped to [e0, e1); LDS index = entry - 4gs
      constexpr int PE = 4 * PERG;
      const int64_t lo4 = 4 * gs;
      int64_t hi4 = 4 * ge;
      hi4 = hi4 < e1 ? hi4 : e1;
      const int64_t lo = lo4 > e0 ? lo4 : e0;
      int cidx[PE];
      VT v[PE];
#pragma unroll
      for (int u = 0; u < PE; ++u) {
        int64_t k = lo + tid + int64_t(u) * kThreads;
        k = k < hi4 ? k : hi4 - 1;
        v[u] = gld(a.vals + k);
        if constexpr (BS == 1) {
          cidx[u] = gld(a.colind + k);
        } else {
          const int64_t kb = k / BB;
          const int w = int(k - kb * BB);
          cidx[u] = gld(a.colind + kb) * BS + (w % BS);
        }
      }
      T xv[PE];
#pragma unroll
      for (int u = 0; u < PE; ++u) xv[u] = gx(cidx[u]);
#pragma unroll
      for (int u = 0; u < PE; ++u) {
        int64_t k = lo + tid + int64_t(u) * kThreads;
        k = k < hi4 ? k : hi4 - 1;
        prod[k - lo4] = T(v[u]) * xv[u];
      }
    } else {
    // ---- stage: branch-free 16-B loads, x gather, products -> LDS
    int cidx[PERG][4];
    VT v[PERG][4];
#pragma unroll
    for (int u = 0; u < PERG; ++u) {
      int64_t g = gs + tid + int64_t(u) * kThreads;
      g = g < ge ? g : ge - 1;
      Vec4<VT>::template load<NT>(a.vals + 4 * g, v[u]);
      if constexpr (BS == 1) {
        const i32x4 c = NT ? __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(a.colind) + g)
                           : reinterpret_cast<const i32x4*>(a.colind)[g];
        cidx[u][0] = c.x; cidx[u][1] = c.y; cidx[u][2] = c.z; cidx[u][3] = c.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t k = 4 * g + j;
          const int64_t kb = k / BB;
          const int w = int(k - kb * BB);
          cidx[u][j] = a.colind[kb] * BS + (w % BS);
        }
      }
    }
    T xv[PERG][4];
#pragma unroll
    for (int u = 0; u < PERG; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[u][j] = gx(cidx[u][j]);
#pragma unroll
    for (int u = 0; u < PERG; ++u) {
      int64_t g = gs + tid + int64_t(u) * kThreads;
      g = g < ge ? g : ge - 1;
      T pr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pr[j] = T(v[u][j]) * xv[u][j];  // exact widening of VT
      Vec4<T>::store(prod + 4 * (g - gs), pr);
    }
    __syncthreads();
    }
    // ---- per-row sequential accumulation (scipy order)
    if (active) {
      const int64_t lo = 4 * gs, hi = 4 * ge;
      const int64_t ks = kb_beg > lo ? kb_beg : lo;
      const int64_t ke = kb_end < hi ? kb_end : hi;
      if constexpr (BS == 1) {
        // 4 LDS reads in flight per step (clamped in-bounds index), adds stay sequential
        const T* pp = prod - lo;
        int64_t k = ks;
        for (; k + 4 <= ke; k += 4) {
          const T p0 = pp[k], p1 = pp[k + 1], p2 = pp[k + 2], p3 = pp[k + 3];
          acc = acc + p0;
          acc = acc + p1;
          acc = acc + p2;
          acc = acc + p3;
        }
        for (; k < ke; ++k) acc = acc + pp[k];
      } else {
        // entries of scalar row (I, comp): k = kb*BB + comp*BS + c, blocks in order
        for (int64_t kb = kb_beg; kb < kb_end; kb += BB) {
#pragma unroll
          for (int c = 0; c < BS; ++c) {
            const int64_t k = kb + comp * BS + c;
            if (k >= ks && k < ke) acc = acc + prod[k - lo];
          }
        }
      }
    }
    __syncthreads();
  }
  if (active) epi.row(b0 * BS + tid, acc, d);
  }  // tiles

  finish_epi_dots<Epi>(d, epi);
}

// Production configuration (tuned on MI355X with tools/spmv_probe.py): see DESIGN.md "SpMV".
template <typename T>
struct SpmvCfg {
  static constexpr int THREADS = 256;
  static constexpr int GPT = sizeof(T) == 8 ? 4 : 8;
  static constexpr bool NT = false;
};

template <int THREADS, int BS>
inline int64_t spmv_grid_t(int64_t nb) {
  const int rb = THREADS / BS;
  return (nb + rb - 1) / rb;
}

constexpr int64_t kReduceGridMax = 1024;  // 256 CUs x 4 resident 256-thread workgroups

template <typename T, typename VT, int BS, int THREADS, int GPT, bool NT, class Pro, class Gx, class Epi,
          bool LANEC = false, bool XCD = false>
inline void launch_spmv_cfg(const lspcg_mat* A, Gx gx, Pro pro, Epi epi, hipStream_t st) {
  SpmvArgs<T, VT, BS> a{A->nb, A->rowptr, A->colind, static_cast<const VT*>(A->vals)};
  int64_t grid = spmv_grid_t<THREADS, BS>(A->nb);
  const int64_t cap = std::min<int64_t>(kReduceGridMax * 256 / THREADS, kElemBlocksMax);  // ticket buffer bound
  if (XCD) grid = std::min<int64_t>(((grid + 7) / 8) * 8, cap);
  else if (Epi::NDOT > 0 && grid > cap) grid = cap;
  if (grid > 0)
    LSPCG_LAUNCH_SPMV((k_spmv<T, VT, BS, THREADS, GPT, NT, Pro, Gx, Epi, LANEC, XCD>), dim3(unsigned(grid)),
                       dim3(THREADS), 0, st, a, pro, gx, epi);
}

template <typename T, int BS, class Pro, class Gx, class Epi>
inline void launch_spmv(const lspcg_mat* A, Gx gx, Pro pro, Epi epi, hipStream_t st) {
  if constexpr (sizeof(T) == 8) {
    if (A->storage_dtype() == LSPCG_F32) {
      launch_spmv_cfg<T, float, BS, SpmvCfg<T>::THREADS, SpmvCfg<T>::GPT, SpmvCfg<T>::NT>(A, gx, pro, epi, st);
      return;
    }
  }
  launch_spmv_cfg<T, T, BS, SpmvCfg<T>::THREADS, SpmvCfg<T>::GPT, SpmvCfg<T>::NT>(A, gx, pro, epi, st);
}

// Dispatch on the matrix block size; `gx` is a gather functor.
template <typename T, class Pro, class Gx, class Epi>
inline int launch_spmv_gx(const lspcg_mat* A, Gx gx, Pro pro, Epi epi, hipStream_t st) {
  if (A->block_size == 1) {
    launch_spmv<T, 1>(A, gx, pro, epi, st);
  } else if (A->block_size == 3) {
    launch_spmv<T, 3>(A, gx, pro, epi, st);
  } else {
    set_error("unsupported block size " + std::to_string(A->block_size));
    return LSPCG_ERR_UNSUPPORTED;
  }
  return LSPCG_OK;
}

template <typename T, class Pro, class Epi>
inline int launch_spmv_any(const lspcg_mat* A, const T* x, Pro pro, Epi epi, hipStream_t st) {
  return launch_spmv_gx<T>(A, GatherVec<T>{x}, pro, epi, st);
}

}  // namespace lspcg
