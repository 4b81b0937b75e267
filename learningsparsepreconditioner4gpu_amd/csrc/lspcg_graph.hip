// Block SpMV as message passing over an edge list -- the GPU form of the reference's
// GraphSpmv (neural_cg/nn/basic_layers.py:112-142) and AATPE (:228-261), the torch twin of
// the ext_spai apply used by training and by neural_pcg.py:649-654.
//
// PyG semantics restated (basic_layers.py:126-142):
//   GraphSpmv(use_transpose=False): flow "target_to_source": x_j = x[edge_index[1]], the
//     message A_e x_j is summed at edge_index[0]        ->  y = A x   (A_e = block (row, col))
//   GraphSpmv(use_transpose=True):  flow "source_to_target": x_j = x[edge_index[0]], the
//     message A_eᵀ x_j is summed at edge_index[1]       ->  y = Aᵀ x
//   forward(..., mask): out * mask after the sum.
//   AATPE.forward(x, ei, A, mask, diag): t = mask ⊙ Aᵀx ; t *= diag ; y = mask ⊙ (A t) + (εx)·diag
// Any edge order, duplicates summed (PyG's scatter-add); the list is sorted once per graph
// (lspcg_graph_create: two radix sorts of 64-bit (row, col) / (col, row) keys) so each output
// row is a deterministic sequential sum over its edges in (row, col) order -- PyG's atomic
// scatter order is arbitrary, so parity is the fp32 tolerance (1e-5), not bits.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <memory>
#include <string>

#include "lspcg_internal.hpp"

struct lspcg_graph {
  lspcg_ctx* ctx = nullptr;
  int64_t N = 0, E = 0;
  int bs = 1;
  // row-major (by edge_index[0]) and column-major (by edge_index[1]) orders of the edges:
  // ptr[N+1] into perm[E] (edge ids) and other[E] (the edge's column, resp. row)
  int32_t *rp = nullptr, *rperm = nullptr, *rother = nullptr;
  int32_t *cp = nullptr, *cperm = nullptr, *cother = nullptr;
};

namespace lspcg {

__global__ void k_graph_keys(int64_t E, int64_t N, const int64_t* __restrict__ ei, uint64_t* __restrict__ krow,
                             uint64_t* __restrict__ kcol, int32_t* __restrict__ ids, int* __restrict__ flag) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = ei[e], c = ei[E + e];
    if (r < 0 || r >= N || c < 0 || c >= N) {
      atomicOr(flag, 1);
      krow[e] = kcol[e] = 0;
    } else {
      krow[e] = uint64_t(r) * uint64_t(N) + uint64_t(c);
      kcol[e] = uint64_t(c) * uint64_t(N) + uint64_t(r);
    }
    ids[e] = int32_t(e);
  }
}

// ptr[i] = first sorted position whose key >= i*N; other[k] = key % N
__global__ void k_graph_ptr(int64_t E, int64_t N, const uint64_t* __restrict__ keys, int32_t* __restrict__ ptr,
                            int32_t* __restrict__ other) {
  const int64_t ts = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i <= N; i += ts) {
    const uint64_t key = uint64_t(i) * uint64_t(N);
    int64_t lo = 0, hi = E;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    ptr[i] = int32_t(lo);
  }
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < E; k += ts) other[k] = int32_t(keys[k] % uint64_t(N));
}

// One thread per scalar output row i = BS*I + a: the sum over the row's edges (sorted order),
// each edge's block row a (TRANS: block column a) against x at the other end.
//   PASS 0 (GraphSpmv / AATPE first half): y = s ; y *= mask ; y *= scale (AATPE's diag)
//   PASS 1 (AATPE second half): y = (s * mask) + (eps * x0) * scale
template <typename T, int BS, bool TRANS, int PASS>
__global__ void __launch_bounds__(256) k_graph_spmv(int64_t N, const int32_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ perm, const int32_t* __restrict__ other,
                                                    const T* __restrict__ vals, const T* __restrict__ x,
                                                    const T* __restrict__ mask, const T* __restrict__ scale,
                                                    const T* __restrict__ x0, T eps, T* __restrict__ y) {
  const int64_t n = N * BS;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t I = i / BS;
    const int a = int(i - I * BS);
    T s = T(0);
    for (int32_t k = ptr[I]; k < ptr[I + 1]; ++k) {
      const int64_t e = perm[k];
      const int64_t J = other[k];
      const T* blk = vals + e * BS * BS;
      T m = T(0);  // the message component: (A_e x_J)[a] or (A_eᵀ x_J)[a]
#pragma unroll
      for (int c = 0; c < BS; ++c) m = m + (TRANS ? blk[c * BS + a] : blk[a * BS + c]) * x[J * BS + c];
      s = s + m;
    }
    if (mask) s = s * mask[i];
    if constexpr (PASS == 0) {
      if (scale) s = s * scale[i];
    } else {
      T ex = eps * x0[i];
      if (scale) ex = ex * scale[i];
      s = s + ex;
    }
    y[i] = s;
  }
}

static int grid_of(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return int(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

template <typename T, int BS>
static void launch(const lspcg_graph* g, bool trans, int pass, const T* vals, const T* x, const T* mask, const T* scale,
                   const T* x0, T eps, T* y) {
  hipStream_t st = g->ctx->stream;
  const dim3 grid(grid_of(g->N * BS)), blk(256);
  const int32_t* ptr = trans ? g->cp : g->rp;
  const int32_t* perm = trans ? g->cperm : g->rperm;
  const int32_t* oth = trans ? g->cother : g->rother;
  if (trans) {
    if (pass == 0)
      hipLaunchKernelGGL((k_graph_spmv<T, BS, true, 0>), grid, blk, 0, st, g->N, ptr, perm, oth, vals, x, mask, scale, x0, eps, y);
    else
      hipLaunchKernelGGL((k_graph_spmv<T, BS, true, 1>), grid, blk, 0, st, g->N, ptr, perm, oth, vals, x, mask, scale, x0, eps, y);
  } else {
    if (pass == 0)
      hipLaunchKernelGGL((k_graph_spmv<T, BS, false, 0>), grid, blk, 0, st, g->N, ptr, perm, oth, vals, x, mask, scale, x0, eps, y);
    else
      hipLaunchKernelGGL((k_graph_spmv<T, BS, false, 1>), grid, blk, 0, st, g->N, ptr, perm, oth, vals, x, mask, scale, x0, eps, y);
  }
}

template <typename T>
static int dispatch(const lspcg_graph* g, bool trans, int pass, const void* vals, const void* x, const void* mask,
                    const void* scale, const void* x0, double eps, void* y) {
  auto v = static_cast<const T*>(vals);
  auto xx = static_cast<const T*>(x);
  auto m = static_cast<const T*>(mask);
  auto sc = static_cast<const T*>(scale);
  auto z = static_cast<const T*>(x0);
  auto yy = static_cast<T*>(y);
  if (g->bs == 1) launch<T, 1>(g, trans, pass, v, xx, m, sc, z, T(eps), yy);
  else launch<T, 3>(g, trans, pass, v, xx, m, sc, z, T(eps), yy);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

static int run(const lspcg_graph* g, int dtype, bool trans, int pass, const void* vals, const void* x,
               const void* mask, const void* scale, const void* x0, double eps, void* y) {
  if (g->N == 0) return LSPCG_OK;
  return dtype == LSPCG_F32 ? dispatch<float>(g, trans, pass, vals, x, mask, scale, x0, eps, y)
                            : dispatch<double>(g, trans, pass, vals, x, mask, scale, x0, eps, y);
}

}  // namespace lspcg

using namespace lspcg;

extern "C" {

int lspcg_graph_create(lspcg_ctx* ctx, int64_t N, int64_t E, int bs, const int64_t* edge_index, lspcg_graph** out) {
  LSPCG_CHECK(ctx && out && (E == 0 || edge_index), LSPCG_ERR_ARG, "graph_create: NULL argument");
  LSPCG_CHECK(bs == 1 || bs == 3, LSPCG_ERR_UNSUPPORTED, "graph_create: block size must be 1 or 3");
  LSPCG_CHECK(N >= 0 && E >= 0 && E < (int64_t(1) << 31) && N * bs < (int64_t(1) << 31), LSPCG_ERR_ARG,
              "graph_create: sizes out of int32 range");
  LSPCG_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  std::unique_ptr<lspcg_graph> g(new lspcg_graph());
  g->ctx = ctx;
  g->N = N;
  g->E = E;
  g->bs = bs;
  const size_t eb = sizeof(int32_t) * size_t(std::max<int64_t>(E, 1));
  for (int32_t** p : {&g->rp, &g->cp}) LSPCG_HIP(hipMalloc(p, sizeof(int32_t) * (N + 1)));
  for (int32_t** p : {&g->rperm, &g->rother, &g->cperm, &g->cother}) LSPCG_HIP(hipMalloc(p, eb));
  if (E == 0) {
    LSPCG_HIP(hipMemsetAsync(g->rp, 0, sizeof(int32_t) * (N + 1), st));
    LSPCG_HIP(hipMemsetAsync(g->cp, 0, sizeof(int32_t) * (N + 1), st));
    LSPCG_HIP(hipStreamSynchronize(st));
    *out = g.release();
    return LSPCG_OK;
  }
  uint64_t *kr = nullptr, *kc = nullptr, *ks = nullptr;
  int32_t* ids = nullptr;
  int* flag = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&]() {
    for (void* p : {(void*)kr, (void*)kc, (void*)ks, (void*)ids, (void*)flag, tmp}) (void)hipFree(p);
  };
  struct Guard {
    decltype(cleanup)& f;
    ~Guard() { f(); }
  } guard{cleanup};
  LSPCG_HIP(hipMalloc(&kr, sizeof(uint64_t) * E));
  LSPCG_HIP(hipMalloc(&kc, sizeof(uint64_t) * E));
  LSPCG_HIP(hipMalloc(&ks, sizeof(uint64_t) * E));
  LSPCG_HIP(hipMalloc(&ids, sizeof(int32_t) * E));
  LSPCG_HIP(hipMalloc(&flag, sizeof(int)));
  LSPCG_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_graph_keys, dim3(grid_of(E)), dim3(256), 0, st, E, N, edge_index, kr, kc, ids, flag);
  int bits = 1;
  while (bits < 64 && (uint64_t(1) << bits) < uint64_t(N) * uint64_t(N)) ++bits;
  size_t tb = 0;
  LSPCG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kr, ks, ids, g->rperm, int(E), 0, bits, st));
  LSPCG_HIP(hipMalloc(&tmp, tb > 0 ? tb : 1));
  LSPCG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kr, ks, ids, g->rperm, int(E), 0, bits, st));
  hipLaunchKernelGGL(k_graph_ptr, dim3(grid_of(std::max<int64_t>(N + 1, E))), dim3(256), 0, st, E, N, ks, g->rp,
                     g->rother);
  LSPCG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kc, ks, ids, g->cperm, int(E), 0, bits, st));
  hipLaunchKernelGGL(k_graph_ptr, dim3(grid_of(std::max<int64_t>(N + 1, E))), dim3(256), 0, st, E, N, ks, g->cp,
                     g->cother);
  int h = 0;
  LSPCG_HIP(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  if (h) {
    lspcg_graph_destroy(g.release());
    set_error("graph_create: edge_index out of range [0, N)");
    return LSPCG_ERR_FORMAT;
  }
  *out = g.release();
  return LSPCG_OK;
}

int lspcg_graph_destroy(lspcg_graph* g) {
  if (!g) return LSPCG_OK;
  (void)hipSetDevice(g->ctx->device);
  for (int32_t* p : {g->rp, g->rperm, g->rother, g->cp, g->cperm, g->cother}) (void)hipFree(p);
  delete g;
  return LSPCG_OK;
}

int lspcg_graph_spmv(lspcg_graph* g, const void* vals, int dtype, int transpose, const void* x, const void* mask,
                     void* y) {
  LSPCG_CHECK(g && (g->E == 0 || vals) && x && y, LSPCG_ERR_ARG, "graph_spmv: NULL argument");
  LSPCG_CHECK(dtype == LSPCG_F32 || dtype == LSPCG_F64, LSPCG_ERR_ARG, "graph_spmv: bad dtype");
  LSPCG_CHECK(x != y, LSPCG_ERR_ARG, "graph_spmv: x and y must not alias");
  LSPCG_HIP(hipSetDevice(g->ctx->device));
  return run(g, dtype, transpose != 0, 0, vals, x, mask, nullptr, nullptr, 0.0, y);
}

int lspcg_graph_aatpe(lspcg_graph* g, const void* vals, int dtype, double epsilon, const void* x, const void* mask,
                      const void* diag, void* t, void* y) {
  LSPCG_CHECK(g && (g->E == 0 || vals) && x && t && y, LSPCG_ERR_ARG, "graph_aatpe: NULL argument");
  LSPCG_CHECK(dtype == LSPCG_F32 || dtype == LSPCG_F64, LSPCG_ERR_ARG, "graph_aatpe: bad dtype");
  LSPCG_CHECK(x != y && x != t && t != y, LSPCG_ERR_ARG, "graph_aatpe: x, t and y must not alias");
  LSPCG_HIP(hipSetDevice(g->ctx->device));
  if (int rc = run(g, dtype, true, 0, vals, x, mask, diag, nullptr, 0.0, t)) return rc;
  return run(g, dtype, false, 1, vals, t, mask, diag, x, epsilon, y);
}

}  // extern "C"
