// Sliced-ELL (SELL-64) iteration view of a scalar CSR matrix, for the PCG loop.
//
// Why (DESIGN.md "SpMV formats"): in the staged CSR kernel one gather instruction covers the
// entries of ~17 consecutive rows at ~4 different stencil positions (~30 distinct cache lines),
// and every row tile pays a dependent rowptr load, an LDS round trip and two barriers.  In
// SELL-64 a wave owns a slice of 64 consecutive rows; entry k of row r is stored at
//     256*(gp[slice] + k/4) + 4*r + k%4
// so lane r loads 4 consecutive entries of ITS row with one 16-B load (values) and one 16-B
// load (columns), and one gather instruction reads x at the same in-row position of 64
// consecutive rows (~4 cache lines on banded FEM matrices).  The row sum stays in a register
// and is accumulated in the row's index order -- scipy's csr_matvec order, so results are
// bit-identical to the CSR kernels.  Padding slots (k >= row length) are skipped by a
// predicate, never added (0*inf and -0.0 + 0.0 must not leak into the sum).
#pragma once

#include "lspcg_internal.hpp"
#include "lspcg_spmv.hpp"

#include <algorithm>
#include <cstdlib>

namespace lspcg {

constexpr int kSellC = 64;  // rows per slice = one wave64

// Column storage: 16-bit offsets from the slice's first row when every |col - 64*slice| <=
// 32767 (banded FEM orderings: 6 instead of 8 B per fp32-valued entry), padding marked by the
// sentinel kSellPad16 (row lengths then need no rowptr loads); otherwise int32 columns, padding =
// the row itself, masked with the row length from rowptr.
constexpr int16_t kSellPad16 = -32768;

// Pattern shared by every matrix with the same CSR (rowptr, colind).
struct SellPattern {
  int64_t n = 0;
  int64_t ns = 0;                  // slices
  int64_t groups = 0;              // gp[ns]: 4-entry groups per lane, summed over slices
  int32_t* gp = nullptr;           // [ns+1] exclusive prefix of per-slice groups-per-row
  void* col = nullptr;             // [256*groups] int32 columns or int16 offsets (col_bits)
  int col_bits = 32;
  const int32_t* rowptr = nullptr; // CSR row pointer (row lengths), not owned
  void release() {
    (void)hipFree(gp);
    (void)hipFree(col);
    gp = nullptr;
    col = nullptr;
  }
};

template <typename VT, typename CT>
struct SellArgs {
  int64_t n;
  int64_t ns;
  const int32_t* gp;
  const CT* col;
  const int32_t* rowptr;
  const VT* vals;
};

// ---- the SpMV ----------------------------------------------------------------
template <typename VT>
struct Vec4Ld;
template <>
struct Vec4Ld<float> {
  __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
    const f32x4 a = *(const __attribute__((address_space(1))) f32x4*)(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};
template <>
struct Vec4Ld<double> {
  __device__ static __forceinline__ void load(const double* p, double (&v)[4]) {
    const auto* q = (const __attribute__((address_space(1))) f64x2*)(p);
    const f64x2 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
};

using i16x4 = short __attribute__((ext_vector_type(4)));

// 256-thread workgroups = 4 slices = one 256-row tile (the same row tiles as k_spmv, so the
// prologue / epilogue functors and the dot-product reduction are shared).  QB groups of 4
// entries are loaded per lane before the first gather (branch-free: the group index is
// clamped, the surplus is masked at the add).
template <typename T, typename VT, typename CT, int QB, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(256) k_spmv_sell(SellArgs<VT, CT> a, Pro pro, Gx gx, Epi epi) {
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  constexpr bool C16 = sizeof(CT) == 2;
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t ntiles = (a.n + 255) / 256;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * 4 + w;
    const int64_t i = tile * 256 + threadIdx.x;
    if (s < a.ns) {  // wave-uniform
      const int32_t g0 = a.gp[s];
      const int nq = a.gp[s + 1] - g0;
      int len = 0;
      if constexpr (!C16) len = i < a.n ? gld(a.rowptr + i + 1) - gld(a.rowptr + i) : 0;
      const int32_t base = int32_t(s * kSellC);
      const VT* vp = a.vals + 256 * int64_t(g0) + 4 * lane;
      const CT* cp = a.col + 256 * int64_t(g0) + 4 * lane;
      T acc = T(0);
      for (int q0 = 0; q0 < nq; q0 += QB) {
        VT v[QB][4];
        int c[QB][4];
        bool m[QB][4];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int q = min(q0 + u, nq - 1);
          Vec4Ld<VT>::load(vp + 256 * q, v[u]);
          if constexpr (C16) {
            const i16x4 cc = *(const __attribute__((address_space(1))) i16x4*)(cp + 256 * q);
            const int o[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              m[u][j] = (o[j] != kSellPad16) && (q0 + u < nq);
              c[u][j] = base + (o[j] != kSellPad16 ? o[j] : 0);
            }
          } else {
            const i32x4 cc = *(const __attribute__((address_space(1))) i32x4*)(cp + 256 * q);
            c[u][0] = cc.x; c[u][1] = cc.y; c[u][2] = cc.z; c[u][3] = cc.w;
#pragma unroll
            for (int j = 0; j < 4; ++j) m[u][j] = 4 * (q0 + u) + j < len;
          }
        }
        T xv[QB][4];
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[u][j] = gx(c[u][j]);
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (m[u][j]) acc = acc + T(v[u][j]) * xv[u][j];
      }
      if (i < a.n) epi.row(i, acc, d);
    }
  }
  if constexpr (Epi::NDOT > 0) {
    grid_reduce_dd<Epi::NDOT>(d, epi.partials, epi.ticket, [&](const double* vals) { epi.fin(vals); });
  }
}

constexpr int64_t kSellReduceGridMax = 2048;  // <= the solver's partial slots (>= 4096)

// grid caps (experiment knobs LSPCG_SELL_RCAP / LSPCG_SELL_NCAP, read once)
inline int64_t sell_cap(bool reducing) {
  static const int64_t rcap = [] {
    const char* e = std::getenv("LSPCG_SELL_RCAP");
    const int64_t v = e ? std::atoll(e) : kSellReduceGridMax;
    return std::max<int64_t>(1, std::min<int64_t>(v, 4096));
  }();
  static const int64_t ncap = [] {
    const char* e = std::getenv("LSPCG_SELL_NCAP");
    return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(1) << 40;
  }();
  return reducing ? rcap : ncap;
}

template <typename T, typename VT, class Pro, class Gx, class Epi>
inline void launch_spmv_sell_cfg(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st) {
  int64_t grid = (P.n + 255) / 256;
  grid = std::min<int64_t>(grid, sell_cap(Epi::NDOT > 0));
  if (grid <= 0) return;
  if (P.col_bits == 16) {
    SellArgs<VT, int16_t> a{P.n, P.ns, P.gp, static_cast<const int16_t*>(P.col), P.rowptr,
                            static_cast<const VT*>(vals)};
    hipLaunchKernelGGL((k_spmv_sell<T, VT, int16_t, 4, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(256), 0, st, a, pro,
                       gx, epi);
  } else {
    SellArgs<VT, int32_t> a{P.n, P.ns, P.gp, static_cast<const int32_t*>(P.col), P.rowptr,
                            static_cast<const VT*>(vals)};
    hipLaunchKernelGGL((k_spmv_sell<T, VT, int32_t, 4, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(256), 0, st, a, pro,
                       gx, epi);
  }
}

}  // namespace lspcg

namespace lspcg {
// Host-side construction (lspcg_sell.hip), enqueued on `st`.
// Builds the SELL-64 pattern of a scalar CSR (n rows); fails with LSPCG_ERR_UNSUPPORTED when the
// padded size exceeds max_pad x nnz (irregular row lengths: the CSR kernel is used instead).
// allow16: store 16-bit column offsets when they fit.
int sell_build_pattern(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, double max_pad,
                       bool allow16, hipStream_t st, SellPattern* out);
// Allocates and fills the SELL value array of a CSR with the same pattern.  src_dtype /
// dst_dtype: LSPCG_F32 or LSPCG_F64 (fp64 -> fp32 only for exactly representable values).
int sell_fill_values(const SellPattern& P, const int32_t* colind, const void* src, int src_dtype, int dst_dtype,
                     hipStream_t st, void** out);
}  // namespace lspcg
