// Diagnostics only (not part of liblspcg_hip.so): the SELL-DIA SpMV (csrc/lspcg_sell.hpp) under
// other launch configurations -- slots loaded per batch (SB) x register budget (MINW, minimum
// workgroups per CU in __launch_bounds__) -- timed cold / warm exactly like lspcg_spmv_timed, so a
// sweep can pick the product's configuration.  Built and driven by tools/sell_sweep.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../learningsparsepreconditioner4gpu_amd/csrc/lspcg_sell.hpp"

using namespace lspcg;

namespace {

__global__ void k_flush(const int4* __restrict__ buf, int64_t n, int* sink) {
  int acc = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int4 v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567) sink[0] = acc;
}

template <typename VT, int SB, int MINW>
void launch(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  const int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  SdiaArgs<VT> a{P.n, P.ns, P.gp, static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals)};
  hipLaunchKernelGGL((k_spmv_sdia<double, VT, SB, kSellWG, MINW, ProNone, GatherVec<double>, EpiStore<double>>),
                     dim3(unsigned(grid)), dim3(kSellWG), 0, st, a, ProNone{}, GatherVec<double>{x}, EpiStore<double>{y});
}

// the fused-update cost model: the vector entry of a slot recomputed from two vectors,
// p_new[c] = p_old[c] * beta + z[c] (what a KC with UP folded in would load)
struct GatherFused {
  const double* z;
  const double* p;
  double beta;
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ double operator()(int64_t j) const { return (gld(p + j) * beta) + gld(z + j); }
};

template <typename VT, int SB, int MINW>
void launch_fused(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  const int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  SdiaArgs<VT> a{P.n, P.ns, P.gp, static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals)};
  // z = x, p = y's second half is not available: use x for both streams at distinct offsets (x + 0 / x + 1)
  hipLaunchKernelGGL((k_spmv_sdia<double, VT, SB, kSellWG, MINW, ProNone, GatherFused, EpiStore<double>>),
                     dim3(unsigned(grid)), dim3(kSellWG), 0, st, a, ProNone{}, GatherFused{x, x + P.n, 0.5},
                     EpiStore<double>{y});
}

// bound experiment: every slot's vector entry a constant (no x load): the values-only stream
struct GatherConst {
  __device__ __forceinline__ void prepare() {}
  __device__ __forceinline__ double operator()(int64_t) const { return 1.0; }
};

template <typename VT, int SB, int MINW>
void launch_xconst(const SellPattern& P, const void* vals, const double*, double* y, hipStream_t st) {
  const int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  SdiaArgs<VT> a{P.n, P.ns, P.gp, static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals)};
  hipLaunchKernelGGL((k_spmv_sdia<double, VT, SB, kSellWG, MINW, ProNone, GatherConst, EpiStore<double>>),
                     dim3(unsigned(grid)), dim3(kSellWG), 0, st, a, ProNone{}, GatherConst{}, EpiStore<double>{y});
}

// Experiment (round 4): slots whose offset is the previous slot's + 1 (the stencil's offset clusters,
// e.g. {-1, 0, 1}, {101, 102}) take their vector entries from the previous slot's by a one-lane DPP
// wave shift instead of a load; lane 63's entry comes from one extra per-slice gather (lane k <
// D_s: x[base + 63 + dict[k]]).  MODE 2: the same kernel with every slot loaded (the baseline of
// this structure); MODE 0: shifted slots reuse the previous vector unshifted (wrong, timing bound);
// MODE 1: the DPP shift (bit-identical).  All 16 slots in one batch; cluster heads loaded at clamped
// addresses on every lane so the shifted entries are right wherever the row has the entry.
__device__ __forceinline__ double wave_shl1(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(b), 0x130, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, int(b >> 32), 0x130, 0xf, 0xf, true);
  return __builtin_bit_cast(double, (long long)(unsigned)lo | ((long long)hi << 32));
}

template <typename VT, int MODE, int MINW>
__global__ void __launch_bounds__(256, MINW) k_sdia_clu(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                        const uint16_t* __restrict__ mask,
                                                        const int32_t* __restrict__ dict, const VT* __restrict__ vals,
                                                        const double* __restrict__ x, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t s = int64_t(blockIdx.x) * 4 + w;
  if (s >= ns) return;
  const int g0 = gp[s], nd = gp[s + 1] - g0;
  const unsigned msk = mask[kSellC * s + lane];
  const int32_t* dp = dict + kSdiaMax * s;
  int32_t dct[kSdiaMax];
#pragma unroll
  for (int j = 0; j < kSdiaMax; ++j) dct[j] = dp[j];
  const int32_t base = int32_t(s * kSellC), row = base + lane;
  const int32_t nm1 = int32_t(n - 1);
  double ext = 0.0;
  if constexpr (MODE == 1) {
    const int32_t e = base + 63 + dp[lane & 15];
    ext = gld(x + min(max(e, 0), nm1));
  }
  VT v[kSdiaMax];
  double xv[kSdiaMax];
#pragma unroll
  for (int j = 0; j < kSdiaMax; ++j) v[j] = gld(vals + kSellC * int64_t(g0 + min(j, nd - 1)) + lane);
#pragma unroll
  for (int j = 0; j < kSdiaMax; ++j) {
    if (j >= nd) continue;
    const bool sh = MODE != 2 && j > 0 && dct[j] == dct[j - 1] + 1;
    if (sh) {
      if constexpr (MODE == 0) {
        xv[j] = xv[j - 1];
      } else {
        const double t = wave_shl1(xv[j - 1]);
        const double e = __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(
                             int(__builtin_bit_cast(long long, ext) >> 32), j)) << 32 |
                             (unsigned)__builtin_amdgcn_readlane(int(__builtin_bit_cast(long long, ext)), j)));
        xv[j] = lane == 63 ? e : t;
      }
    } else {
      xv[j] = gld(x + min(max(row + dct[j], 0), nm1));
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < kSdiaMax; ++j) {
    if (j < nd && ((msk >> j) & 1u)) acc = acc + double(v[j]) * xv[j];
  }
  if (row < n) y[row] = acc;
}

template <typename VT, int MODE, int MINW>
void launch_clu(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  hipLaunchKernelGGL((k_sdia_clu<VT, MODE, MINW>), dim3(unsigned((P.ns + 3) / 4)), dim3(256), 0, st, P.n, P.ns, P.gp,
                     static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals), x, y);
}

// Experiment (round 5): each wave takes NS consecutive slices, loading all their metadata at once and
// then every value / vector load of all NS slices before the first add -- one metadata round trip and
// one data round trip per NS slices (the product kernel's one-tile workgroups pay both per slice).
template <typename VT, int NS, int MINW>
__global__ void __launch_bounds__(256, MINW) k_sdia_multi(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                          const uint16_t* __restrict__ mask,
                                                          const int32_t* __restrict__ dict, const VT* __restrict__ vals,
                                                          const double* __restrict__ x, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t s0 = (int64_t(blockIdx.x) * 4 + w) * NS;
  int g0[NS], nd[NS];
  unsigned msk[NS];
  int32_t dct[NS][kSdiaMax];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int64_t s = min(s0 + k, ns - 1);
    g0[k] = gp[s];
    nd[k] = s0 + k < ns ? gp[s + 1] - g0[k] : 0;
    msk[k] = mask[kSellC * s + lane];
    const int32_t* dp = dict + kSdiaMax * s;
#pragma unroll
    for (int j = 0; j < kSdiaMax; ++j) dct[k][j] = dp[j];
  }
  VT v[NS][kSdiaMax];
  double xv[NS][kSdiaMax];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int32_t base = int32_t(min(s0 + k, ns - 1) * kSellC), row = base + lane;
#pragma unroll
    for (int j = 0; j < kSdiaMax; ++j) {
      if (j < nd[k]) {
        const bool m = (msk[k] >> j) & 1u;
        v[k][j] = gld(vals + kSellC * int64_t(g0[k] + j) + lane);
        xv[k][j] = gld(x + (m ? row + dct[k][j] : base));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int64_t row = (s0 + k) * kSellC + lane;
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kSdiaMax; ++j)
      if (j < nd[k] && ((msk[k] >> j) & 1u)) acc = acc + double(v[k][j]) * xv[k][j];
    if (s0 + k < ns && row < n) y[row] = acc;
  }
}

template <typename VT, int NS, int MINW>
void launch_multi(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  const int64_t waves = (P.ns + NS - 1) / NS;
  hipLaunchKernelGGL((k_sdia_multi<VT, NS, MINW>), dim3(unsigned((waves + 3) / 4)), dim3(256), 0, st, P.n, P.ns, P.gp,
                     static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals), x, y);
}

// Experiment (round 5): TWO waves per slice.  Wave h of a pair loads slots [8h, 8h + 8) and forms
// their products; wave 0 folds its products in slot order, hands the partial row sums to wave 1
// through LDS, and wave 1 continues the fold with its own products in slot order -- the same
// sequential sum (products are rounded before each add either way), with twice the waves.
template <typename VT, int MINW>
__global__ void __launch_bounds__(256, MINW) k_sdia_split2(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                           const uint16_t* __restrict__ mask,
                                                           const int32_t* __restrict__ dict, const VT* __restrict__ vals,
                                                           const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double sh[2][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int h = w & 1, pr = w >> 1;
  const int64_t s = int64_t(blockIdx.x) * 2 + pr;
  const bool live = s < ns;  // wave-uniform
  const int64_t sc = live ? s : ns - 1;
  const int g0 = gp[sc], nd = live ? gp[sc + 1] - g0 : 0;
  const unsigned msk = mask[kSellC * sc + lane];
  const int32_t* dp = dict + kSdiaMax * sc + 8 * h;
  int32_t dct[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dct[j] = dp[j];
  const int32_t base = int32_t(sc * kSellC), row = base + lane;
  double prod[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = 8 * h + j;
    const bool m = jj < nd && ((msk >> jj) & 1u);
    const VT v = gld(vals + kSellC * int64_t(g0 + min(jj, max(nd - 1, 0))) + lane);
    const double xv = gld(x + (m ? row + dct[j] : base));
    prod[j] = double(v) * xv;
  }
  double acc = 0.0;
  if (h == 1) {
    __syncthreads();
    acc = sh[pr][lane];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int jj = 8 * h + j;
    if (jj < nd && ((msk >> jj) & 1u)) acc = acc + prod[j];
  }
  if (h == 0) {
    sh[pr][lane] = acc;
    __syncthreads();
  } else if (live && row < n) {
    y[row] = acc;
  }
}

template <typename VT, int MINW>
void launch_split2(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  hipLaunchKernelGGL((k_sdia_split2<VT, MINW>), dim3(unsigned((P.ns + 1) / 2)), dim3(256), 0, st, P.n, P.ns, P.gp,
                     static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals), x, y);
}

using Fn = void (*)(const SellPattern&, const void*, const double*, double*, hipStream_t);

// config id -> (value bytes, slots per batch SB, MINW, transposed)
struct Cfg {
  int vbytes, qb, minw, tr;
  Fn fn;
};
const Cfg kCfgs[] = {
    {8, 4, 1, 0, launch<double, 4, 1>},  {8, 8, 1, 0, launch<double, 8, 1>}, {8, 16, 1, 0, launch<double, 16, 1>},
    {8, 8, 4, 0, launch<double, 8, 4>},  {4, 4, 6, 0, launch<float, 4, 6>},  {4, 8, 6, 0, launch<float, 8, 6>},
    {4, 16, 6, 0, launch<float, 16, 6>}, {4, 8, 8, 0, launch<float, 8, 8>},  {4, 8, 1, 0, launch<float, 8, 1>},
    {4, 8, 6, 1, launch_fused<float, 8, 6>}, {4, 16, 6, 1, launch_fused<float, 16, 6>},
    {8, 8, 1, 3, launch_xconst<double, 8, 1>}, {4, 8, 6, 3, launch_xconst<float, 8, 6>},
    {8, 16, 1, 4, launch_clu<double, 2, 1>}, {8, 16, 1, 5, launch_clu<double, 0, 1>}, {8, 16, 1, 6, launch_clu<double, 1, 1>},
    {4, 16, 6, 4, launch_clu<float, 2, 6>},  {4, 16, 6, 5, launch_clu<float, 0, 6>},  {4, 16, 6, 6, launch_clu<float, 1, 6>},
    {8, 1, 1, 7, launch_multi<double, 1, 1>}, {8, 2, 1, 7, launch_multi<double, 2, 1>}, {8, 3, 1, 7, launch_multi<double, 3, 1>},
    {8, 4, 1, 7, launch_multi<double, 4, 1>},
    {8, 8, 1, 8, launch_split2<double, 1>}, {4, 8, 6, 8, launch_split2<float, 6>}, {4, 8, 8, 8, launch_split2<float, 8>},
};

template <typename VT, int QB, int MINW>
void launch_bsr(const SellPattern& P, const void* vals, const double* x, double* y, hipStream_t st) {
  const int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  SellArgs<VT, int16_t> a{P.n, P.ns, P.gp, static_cast<const int16_t*>(P.col), P.rowptr, static_cast<const VT*>(vals)};
  hipLaunchKernelGGL((k_spmv_bsell3<double, VT, int16_t, QB, kSellWG, MINW, ProNone, GatherVec<double>, EpiStore<double>>),
                     dim3(unsigned(grid)), dim3(kSellWG), 0, st, a, ProNone{}, GatherVec<double>{x}, EpiStore<double>{y});
}

// BSELL-64 (BSR 3x3) configurations: (value bytes, block slots per batch QB, MINW)
const Cfg kBsrCfgs[] = {
    {8, 1, 1, 0, launch_bsr<double, 1, 1>}, {8, 2, 1, 0, launch_bsr<double, 2, 1>}, {8, 4, 1, 0, launch_bsr<double, 4, 1>},
    {8, 8, 1, 0, launch_bsr<double, 8, 1>}, {4, 2, 1, 0, launch_bsr<float, 2, 1>},  {4, 4, 1, 0, launch_bsr<float, 4, 1>},
    {4, 8, 1, 0, launch_bsr<float, 8, 1>},
};

// SELL-DIA with the values of a slice stored in quads (the experiment: 16-B value loads, one per 4
// slots, D_s padded to a multiple of 4): vals[64 gq[s] * 4 + 256 (j / 4) + 4 lane + j % 4]
template <typename T, int QPB>
__global__ void __launch_bounds__(256, 6) k_sdia_quad(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                      const int32_t* __restrict__ gq, const uint16_t* __restrict__ mask,
                                                      const int32_t* __restrict__ dict, const float* __restrict__ vals,
                                                      const T* __restrict__ x, T* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t s = int64_t(blockIdx.x) * 4 + w;
  if (s >= ns) return;
  const int nd = gp[s + 1] - gp[s];
  const int nq = gq[s + 1] - gq[s];
  const int32_t* dp = dict + kSdiaMax * s;
  const unsigned msk = mask[kSellC * s + lane];
  const int32_t base = int32_t(s * kSellC), row = base + lane;
  const float* vp = vals + 256 * int64_t(gq[s]) + 4 * lane;
  T acc = T(0);
#pragma unroll
  for (int j0 = 0; j0 < kSdiaMax; j0 += 4 * QPB) {
    if (j0 >= nd) break;
    float v[4 * QPB];
    T xv[4 * QPB];
    bool m[4 * QPB];
#pragma unroll
    for (int u = 0; u < QPB; ++u) {
      const int g = min(j0 / 4 + u, nq - 1);
      const f32x4 a = *(const __attribute__((address_space(1))) f32x4*)(vp + 256 * g);
      v[4 * u] = a.x; v[4 * u + 1] = a.y; v[4 * u + 2] = a.z; v[4 * u + 3] = a.w;
    }
#pragma unroll
    for (int u = 0; u < 4 * QPB; ++u) {
      const int j = min(j0 + u, nd - 1);
      m[u] = (j0 + u < nd) && ((msk >> (j0 + u)) & 1u);
      xv[u] = gld(x + (m[u] ? row + dp[j] : base));
    }
#pragma unroll
    for (int u = 0; u < 4 * QPB; ++u)
      if (m[u]) acc = acc + T(v[u]) * xv[u];
  }
  if (row < n) y[row] = acc;
}

}  // namespace

extern "C" {

// the quad-layout experiment: builds the SELL-DIA pattern, re-lays its fp32 values into quads on the
// host and times k_sdia_quad (QPB quads per batch: 2 or 4) like sweep_run
int sweep_quad_run(int qpb, int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, const double* vals,
                   const double* x, double* y, int reps, int64_t flush_bytes, double* ms_cold, double* ms_warm) {
  hipStream_t st = nullptr;
  SellPattern P;
  if (sell_build_pattern(n, nnz, rowptr, colind, 1e30, kSellColDia, st, &P) || P.col_bits != 1) return -2;
  void* v = nullptr;
  if (sell_fill_values(P, colind, vals, LSPCG_F64, LSPCG_F32, st, &v)) return -3;
  (void)hipDeviceSynchronize();
  std::vector<int32_t> gp(P.ns + 1), gq(P.ns + 1, 0);
  (void)hipMemcpy(gp.data(), P.gp, sizeof(int32_t) * (P.ns + 1), hipMemcpyDeviceToHost);
  for (int64_t s = 0; s < P.ns; ++s) gq[s + 1] = gq[s] + (gp[s + 1] - gp[s] + 3) / 4;
  std::vector<float> sv(size_t(64) * gp[P.ns]), qv(size_t(256) * gq[P.ns], 0.f);
  (void)hipMemcpy(sv.data(), v, sizeof(float) * sv.size(), hipMemcpyDeviceToHost);
  for (int64_t s = 0; s < P.ns; ++s)
    for (int j = 0; j < gp[s + 1] - gp[s]; ++j)
      for (int l = 0; l < 64; ++l)
        qv[size_t(256) * gq[s] + 256 * (j / 4) + 4 * l + j % 4] = sv[size_t(64) * (gp[s] + j) + l];
  int32_t* dgq = nullptr;
  float* dqv = nullptr;
  (void)hipMalloc(&dgq, sizeof(int32_t) * gq.size());
  (void)hipMalloc(&dqv, sizeof(float) * std::max<size_t>(qv.size(), 1));
  (void)hipMemcpy(dgq, gq.data(), sizeof(int32_t) * gq.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dqv, qv.data(), sizeof(float) * qv.size(), hipMemcpyHostToDevice);
  int4* fl = nullptr;
  int* sink = nullptr;
  (void)hipMalloc(&fl, size_t(flush_bytes) + 64);
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(fl, 1, size_t(flush_bytes));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 g(unsigned((P.ns + 3) / 4)), b(256);
  auto run = [&]() {
    if (qpb == 4)
      hipLaunchKernelGGL((k_sdia_quad<double, 4>), g, b, 0, st, P.n, P.ns, P.gp, dgq,
                         static_cast<const uint16_t*>(P.col), P.dict, dqv, x, y);
    else
      hipLaunchKernelGGL((k_sdia_quad<double, 2>), g, b, 0, st, P.n, P.ns, P.gp, dgq,
                         static_cast<const uint16_t*>(P.col), P.dict, dqv, x, y);
  };
  auto flush = [&]() { hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, st, fl, flush_bytes / 16, sink); };
  float t = 0.f, tp = 0.f, tf = 0.f;
  run();
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < 3 * reps; ++i) run();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms_warm = t / (3 * reps);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) {
    flush();
    run();
  }
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tp, e0, e1);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) flush();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tf, e0, e1);
  *ms_cold = (tp - tf) / reps;
  const hipError_t e = hipDeviceSynchronize();
  for (void* p : {(void*)dgq, (void*)dqv, v, (void*)fl, (void*)sink}) (void)hipFree(p);
  P.release();
  return e == hipSuccess ? 0 : -4;
}

int sweep_bsr_count() { return int(sizeof(kBsrCfgs) / sizeof(kBsrCfgs[0])); }

int sweep_bsr_cfg(int id, int* vbytes, int* qb) {
  if (id < 0 || id >= sweep_bsr_count()) return -1;
  *vbytes = kBsrCfgs[id].vbytes;
  *qb = kBsrCfgs[id].qb;
  return 0;
}

// BSR 3x3: nb block rows, nnzb blocks, rowptr / colind (int32, device), vals [nnzb][3][3] fp64 (device)
int sweep_bsr_run(int id, int64_t nb, int64_t nnzb, const int32_t* rowptr, const int32_t* colind, const double* vals,
                  const double* x, double* y, int reps, int64_t flush_bytes, double* ms_cold, double* ms_warm) {
  if (id < 0 || id >= sweep_bsr_count()) return -1;
  hipStream_t st = nullptr;
  SellPattern P;
  if (bsell_build_pattern(nb, nnzb, rowptr, colind, 1e30, true, false, st, &P) || P.col_bits != 16) return -2;
  void* v = nullptr;
  if (bsell_fill_values(P, vals, LSPCG_F64, kBsrCfgs[id].vbytes == 4 ? LSPCG_F32 : LSPCG_F64, st, &v)) return -3;
  int4* fl = nullptr;
  int* sink = nullptr;
  (void)hipMalloc(&fl, size_t(flush_bytes) + 64);
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(fl, 1, size_t(flush_bytes));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&]() { kBsrCfgs[id].fn(P, v, x, y, st); };
  auto flush = [&]() { hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, st, fl, flush_bytes / 16, sink); };
  float t = 0.f, tp = 0.f, tf = 0.f;
  run();
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < 3 * reps; ++i) run();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms_warm = t / (3 * reps);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) {
    flush();
    run();
  }
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tp, e0, e1);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) flush();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tf, e0, e1);
  *ms_cold = (tp - tf) / reps;
  const hipError_t e = hipDeviceSynchronize();
  (void)hipFree(v);
  (void)hipFree(fl);
  (void)hipFree(sink);
  P.release();
  return e == hipSuccess ? 0 : -4;
}

int sweep_count() { return int(sizeof(kCfgs) / sizeof(kCfgs[0])); }

int sweep_cfg(int id, int* vbytes, int* qb, int* minw, int* tr) {
  if (id < 0 || id >= sweep_count()) return -1;
  *tr = kCfgs[id].tr;
  *vbytes = kCfgs[id].vbytes;
  *qb = kCfgs[id].qb;
  *minw = kCfgs[id].minw;
  return 0;
}

// rowptr / colind (int32, device) / vals (fp64, device) of an n-row CSR with sorted rows; x, y device
// fp64.  Times config `id` (dictionary columns required): ms_cold / ms_warm per launch.
int sweep_run(int id, int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, const double* vals,
              const double* x, double* y, int reps, int64_t flush_bytes, double* ms_cold, double* ms_warm) {
  if (id < 0 || id >= sweep_count()) return -1;
  hipStream_t st = nullptr;
  SellPattern P;
  if (sell_build_pattern(n, nnz, rowptr, colind, 1e30, kSellColDia, st, &P) || P.col_bits != 1) return -2;
  void* v = nullptr;
  const int vb = kCfgs[id].vbytes;
  if (sell_fill_values(P, colind, vals, LSPCG_F64, vb == 4 ? LSPCG_F32 : LSPCG_F64, st, &v)) return -3;
  int4* fl = nullptr;
  int* sink = nullptr;
  (void)hipMalloc(&fl, size_t(flush_bytes) + 64);
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(fl, 1, size_t(flush_bytes));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&]() { kCfgs[id].fn(P, v, x, y, st); };
  auto flush = [&]() { hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, st, fl, flush_bytes / 16, sink); };
  float t = 0.f;
  run();
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < 3 * reps; ++i) run();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms_warm = t / (3 * reps);
  float tp = 0.f, tf = 0.f;
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) {
    flush();
    run();
  }
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tp, e0, e1);
  (void)hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) flush();
  (void)hipEventRecord(e1, st);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&tf, e0, e1);
  *ms_cold = (tp - tf) / reps;
  const hipError_t e = hipDeviceSynchronize();
  (void)hipFree(v);
  (void)hipFree(fl);
  (void)hipFree(sink);
  P.release();
  return e == hipSuccess ? 0 : -4;
}
}
