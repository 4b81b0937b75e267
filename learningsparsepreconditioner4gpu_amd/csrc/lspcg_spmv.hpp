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

#include "lspcg_internal.hpp"

namespace lspcg {

template <typename T, int BS>
struct SpmvArgs {
  int64_t nb;             // block rows
  const int32_t* rowptr;  // [nb+1]
  const int32_t* colind;  // [nnzb]
  const T* vals;          // [nnzb*BS*BS]
  const T* x;             // gathered vector
};

template <int BS>
__host__ __device__ constexpr int spmv_rows_per_block() { return kThreads / BS; }

template <typename T, int BS>
__host__ __device__ constexpr int spmv_cap() {
  // fp32 entries are half the size: stage twice as many per chunk (same 32 KiB LDS).
  return ((kSpmvCap * (sizeof(T) == 4 ? 2 : 1)) / (BS * BS)) * (BS * BS);
}

inline int64_t spmv_grid(int64_t nb, int bs) {
  const int rb = kThreads / bs;
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
  __device__ __forceinline__ void row(int64_t r, T s, DD*) const { y[r] = s; }
  __device__ __forceinline__ void fin(const double*) const {}
  double* partials = nullptr;
  unsigned* ticket = nullptr;
};

template <typename T, int BS, class Pro, class Epi>
__global__ void __launch_bounds__(kThreads) k_spmv(SpmvArgs<T, BS> a, Pro pro, Epi epi) {
  constexpr int BB = BS * BS;
  constexpr int CAP = spmv_cap<T, BS>();
  constexpr int RB = spmv_rows_per_block<BS>();
  constexpr int PER = (CAP + kThreads - 1) / kThreads;
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  __shared__ T prod[CAP];

  if (pro.exit()) return;

  const int tid = threadIdx.x;
  const int64_t b0 = int64_t(blockIdx.x) * RB;
  const int64_t b1 = b0 + RB < a.nb ? b0 + RB : a.nb;
  const int64_t e0 = int64_t(a.rowptr[b0]) * BB;
  const int64_t e1 = int64_t(a.rowptr[b1]) * BB;
  const bool active = tid < (b1 - b0) * BS;
  const int64_t I = b0 + tid / BS;
  const int comp = tid % BS;
  int64_t kb_beg = 0, kb_end = 0;
  if (active) {
    kb_beg = a.rowptr[I];
    kb_end = a.rowptr[I + 1];
  }
  T acc = T(0);

  for (int64_t c0 = e0; c0 < e1; c0 += CAP) {
    const int64_t c1 = c0 + CAP < e1 ? c0 + CAP : e1;
    // ---- stage: coalesced value/index loads, x gather, products -> LDS
    int cidx[PER];
    T v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t k = c0 + tid + int64_t(u) * kThreads;
      if (k < c1) {
        if constexpr (BS == 1) {
          cidx[u] = a.colind[k];
        } else {
          const int64_t kb = k / BB;
          const int w = int(k - kb * BB);
          cidx[u] = a.colind[kb] * BS + (w % BS);
        }
        v[u] = a.vals[k];
      }
    }
    T xv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t k = c0 + tid + int64_t(u) * kThreads;
      if (k < c1) xv[u] = a.x[cidx[u]];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int64_t k = c0 + tid + int64_t(u) * kThreads;
      if (k < c1) prod[k - c0] = v[u] * xv[u];
    }
    __syncthreads();
    // ---- per-row sequential accumulation (scipy order)
    if (active) {
      const int64_t lo = c0 / BB, hi = c1 / BB;
      const int64_t kbs = kb_beg > lo ? kb_beg : lo;
      const int64_t kbe = kb_end < hi ? kb_end : hi;
      const T* pp = prod + (kbs - lo) * BB + comp * BS;
      for (int64_t kb = kbs; kb < kbe; ++kb, pp += BB) {
#pragma unroll
        for (int cc = 0; cc < BS; ++cc) acc = acc + pp[cc];
      }
    }
    __syncthreads();
  }

  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  if (active) epi.row(b0 * BS + tid, acc, d);
  if constexpr (Epi::NDOT > 0) {
    grid_reduce_dd<Epi::NDOT>(d, epi.partials, epi.ticket, [&](const double* vals) { epi.fin(vals); });
  }
}

template <typename T, int BS, class Pro, class Epi>
inline void launch_spmv(const lspcg_mat* A, const T* x, Pro pro, Epi epi, hipStream_t st) {
  SpmvArgs<T, BS> a{A->nb, A->rowptr, A->colind, static_cast<const T*>(A->vals), x};
  const int64_t grid = spmv_grid(A->nb, BS);
  if (grid > 0) hipLaunchKernelGGL((k_spmv<T, BS, Pro, Epi>), dim3(unsigned(grid)), dim3(kThreads), 0, st, a, pro, epi);
}

// Dispatch on the matrix block size.
template <typename T, class Pro, class Epi>
inline int launch_spmv_any(const lspcg_mat* A, const T* x, Pro pro, Epi epi, hipStream_t st) {
  if (A->block_size == 1) {
    launch_spmv<T, 1>(A, x, pro, epi, st);
  } else if (A->block_size == 3) {
    launch_spmv<T, 3>(A, x, pro, epi, st);
  } else {
    set_error("unsupported block size " + std::to_string(A->block_size));
    return LSPCG_ERR_UNSUPPORTED;
  }
  return LSPCG_OK;
}

}  // namespace lspcg
