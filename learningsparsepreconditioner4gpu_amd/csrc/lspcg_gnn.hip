// GNN that infers the SPAI factor L: NodeEdgeProcessing.forward (neural_cg/nn/gnns.py:77-97)
// with FeedForward (basic_layers.py:73-109, num_layers = 2 -> Linear/GELU/Linear/GELU/Linear)
// and MPLayer (basic_layers.py:145-225, PyG 2.6.1 source_to_target flow: x_i = x[dst =
// edge_index[1]], x_j = x[src = edge_index[0]], messages summed at dst).  fp32.
//
// Layout (DESIGN.md "GNN"): edges are kept in CSC order (sorted by dst, then by original
// edge id) for the whole forward.  One message-passing layer is ONE kernel: a 256-thread
// workgroup owns 256 destination nodes and streams their incoming edges in chunks of 512
// (coalesced edge-feature reads/writes, x rows gathered).  Per edge a thread computes the
// shared LayerNorm(48) statistics, the message MLP and the edge MLP, writes the updated
// edge feature in place and drops the message into LDS; after a barrier every node thread
// sums its messages in CSC order (deterministic, no atomics), applies LayerNorm(16) + the
// node MLP + residual and writes the next node state.  Messages never touch HBM.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <memory>
#include <string>
#include <vector>

#include "lspcg_internal.hpp"

namespace lspcg {

constexpr int H = 16;        // hidden = node_features = edge_features
constexpr int CE = 512;      // edges per LDS chunk (512 x 16 x 4 B = 32 KiB)
constexpr int kMaxIn = 32;   // encoder input features supported

// FeedForward(in, out, hidden=16, num_layers=2) parameter block:
//   [W1 (16 x in) | b1 (16) | W2 (16 x 16) | b2 (16) | W3 (out x 16) | b3 (out)]
__host__ __device__ constexpr int ff_size(int in, int out) { return H * in + H + H * H + H + out * H + out; }

__device__ __forceinline__ float gelu(float v) { return 0.5f * v * (1.0f + erff(v * 0.7071067811865476f)); }

template <int IN>
__device__ __forceinline__ void linear16(const float* __restrict__ W, const float* __restrict__ b, const float* in,
                                         float* out) {
#pragma unroll
  for (int o = 0; o < H; ++o) {
    float acc = b[o];
#pragma unroll
    for (int i = 0; i < IN; ++i) acc = __builtin_fmaf(in[i], W[o * IN + i], acc);
    out[o] = acc;
  }
}

// hidden part of the FF after its first layer: GELU -> Linear16 -> GELU -> Linear(out)
template <int OUT>
__device__ __forceinline__ void ff_tail(const float* __restrict__ w2, const float* h1, float* out) {
  float a[H], h2[H];
#pragma unroll
  for (int o = 0; o < H; ++o) a[o] = gelu(h1[o]);
  linear16<H>(w2, w2 + H * H, a, h2);
#pragma unroll
  for (int o = 0; o < H; ++o) a[o] = gelu(h2[o]);
  const float* W3 = w2 + H * H + H;
  const float* b3 = W3 + OUT * H;
#pragma unroll
  for (int o = 0; o < OUT; ++o) {
    float acc = b3[o];
#pragma unroll
    for (int i = 0; i < H; ++i) acc = __builtin_fmaf(a[i], W3[o * H + i], acc);
    out[o] = acc;
  }
}

// Encoder with a runtime input width, input row read straight from global memory
// (loop over inputs outermost so no runtime-indexed register array is needed).
__device__ __forceinline__ void ff_encode(const float* __restrict__ w, int in_n, const float* __restrict__ in,
                                          float* out) {
  float h1[H];
#pragma unroll
  for (int o = 0; o < H; ++o) h1[o] = w[H * in_n + o];
  for (int i = 0; i < in_n; ++i) {
    const float v = in[i];
#pragma unroll
    for (int o = 0; o < H; ++o) h1[o] = __builtin_fmaf(v, w[o * in_n + i], h1[o]);
  }
  ff_tail<H>(w + H * in_n + H, h1, out);
}

__device__ __forceinline__ void ld16(const float* __restrict__ p, float* v) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 t = q[j];
    v[4 * j] = t.x;
    v[4 * j + 1] = t.y;
    v[4 * j + 2] = t.z;
    v[4 * j + 3] = t.w;
  }
}
__device__ __forceinline__ void st16(float* __restrict__ p, const float* v) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
}

// ---------------------------------------------------------------------------
// CSC build: count by dst, scan, slot fill, per-node insertion sort by edge id
// ---------------------------------------------------------------------------
__global__ void k_csc_count(int64_t E, const int64_t* __restrict__ ei, int32_t* __restrict__ cnt) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += int64_t(gridDim.x) * blockDim.x)
    atomicAdd(&cnt[ei[E + e]], 1);
}
__global__ void k_csc_fill(int64_t E, const int64_t* __restrict__ ei, const int32_t* __restrict__ ptr,
                           int32_t* __restrict__ fill, int32_t* __restrict__ perm) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t d = ei[E + e];
    perm[ptr[d] + atomicAdd(&fill[d], 1)] = int32_t(e);
  }
}
__global__ void k_csc_sort(int64_t N, const int64_t* __restrict__ ei, int64_t E, const int32_t* __restrict__ ptr,
                           int32_t* __restrict__ perm, int32_t* __restrict__ inv, int32_t* __restrict__ src,
                           int32_t* __restrict__ dst) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t b = ptr[i], e = ptr[i + 1];
    for (int32_t k = b + 1; k < e; ++k) {
      const int32_t v = perm[k];
      int32_t m = k - 1;
      while (m >= b && perm[m] > v) {
        perm[m + 1] = perm[m];
        --m;
      }
      perm[m + 1] = v;
    }
    for (int32_t k = b; k < e; ++k) {
      const int32_t oe = perm[k];
      inv[oe] = k;
      src[k] = int32_t(ei[oe]);
      dst[k] = int32_t(i);
    }
  }
}

// ---------------------------------------------------------------------------
// Encoders / decoder
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_node_enc(int64_t N, int fin, const float* __restrict__ w,
                                                       const float* __restrict__ x, float* __restrict__ h) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    float out[H];
    ff_encode(w, fin, x + i * fin, out);
    st16(h + i * H, out);
  }
}

__global__ void __launch_bounds__(kThreads) k_edge_enc(int64_t E, int fe, const float* __restrict__ w,
                                                       const float* __restrict__ ea, const int32_t* __restrict__ perm,
                                                       float* __restrict__ ecsc) {
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < E; k += int64_t(gridDim.x) * blockDim.x) {
    float out[H];
    const int64_t oe = perm[k];
    ff_encode(w, fe, ea + oe * fe, out);
    st16(ecsc + k * H, out);
  }
}

// out[e] = edge_dec(cat[e_attr, x[src], x[dst]])  (gnns.py:88-95; original edge order)
template <int OUT>
__global__ void __launch_bounds__(kThreads) k_edge_dec(int64_t E, const float* __restrict__ w,
                                                       const int64_t* __restrict__ ei, const int32_t* __restrict__ inv,
                                                       const float* __restrict__ ecsc, const float* __restrict__ x,
                                                       float* __restrict__ out) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += int64_t(gridDim.x) * blockDim.x) {
    float in[3 * H], h1[H], o[OUT];
    ld16(ecsc + int64_t(inv[e]) * H, in);
    ld16(x + ei[e] * H, in + H);
    ld16(x + ei[E + e] * H, in + 2 * H);
    linear16<3 * H>(w, w + 3 * H * H, in, h1);
    ff_tail<OUT>(w + 3 * H * H + H, h1, o);
#pragma unroll
    for (int j = 0; j < OUT; ++j) out[e * OUT + j] = o[j];
  }
}

// ---------------------------------------------------------------------------
// One MPLayer (basic_layers.py:193-225) as one kernel
// ---------------------------------------------------------------------------
struct LayerW {
  const float* node;  // [ln_g 16 | ln_b 16 | FF(16 -> 16)]
  const float* edge;  // [ln_g 48 | ln_b 48 | FF(48 -> 16)]
  const float* msg;   // [ln_g 48 | ln_b 48 | FF(48 -> 16)]
};

__device__ __forceinline__ void ln_ff48(const float* __restrict__ p, const float* xn, float* out) {
  const float* g = p;
  const float* bb = p + 3 * H;
  const float* w = p + 6 * H;
  float in[3 * H], h1[H];
#pragma unroll
  for (int i = 0; i < 3 * H; ++i) in[i] = __builtin_fmaf(xn[i], g[i], bb[i]);
  linear16<3 * H>(w, w + 3 * H * H, in, h1);
  ff_tail<H>(w + 3 * H * H + H, h1, out);
}

__global__ void __launch_bounds__(kThreads) k_mp_layer(int64_t N, LayerW lw, int node_res, int edge_res,
                                                       const int32_t* __restrict__ ptr, const int32_t* __restrict__ src,
                                                       const int32_t* __restrict__ dst, const float* __restrict__ x,
                                                       float* __restrict__ e, float* __restrict__ xout) {
  __shared__ float msg[CE * H];
  const int tid = threadIdx.x;
  const int64_t n0 = int64_t(blockIdx.x) * kThreads;
  const int64_t n1 = n0 + kThreads < N ? n0 + kThreads : N;
  const int64_t k0 = ptr[n0], k1 = ptr[n1];
  const int64_t i = n0 + tid;
  const bool active = i < n1;
  int64_t my_b = 0, my_e = 0;
  if (active) {
    my_b = ptr[i];
    my_e = ptr[i + 1];
  }
  float agg[H];
#pragma unroll
  for (int o = 0; o < H; ++o) agg[o] = 0.f;

  for (int64_t c0 = k0; c0 < k1; c0 += CE) {
    const int64_t c1 = c0 + CE < k1 ? c0 + CE : k1;
    for (int64_t k = c0 + tid; k < c1; k += kThreads) {
      float h[3 * H];
      ld16(x + int64_t(dst[k]) * H, h);          // x_i (target)
      ld16(x + int64_t(src[k]) * H, h + H);      // x_j (source)
      ld16(e + k * H, h + 2 * H);                // edge attr
      float mean = 0.f;
#pragma unroll
      for (int q = 0; q < 3 * H; ++q) mean += h[q];
      mean *= (1.0f / (3 * H));
      float var = 0.f;
#pragma unroll
      for (int q = 0; q < 3 * H; ++q) {
        const float dv = h[q] - mean;
        var = __builtin_fmaf(dv, dv, var);
      }
      var *= (1.0f / (3 * H));
      const float rstd = 1.0f / sqrtf(var + 1e-5f);
      float xn[3 * H];
#pragma unroll
      for (int q = 0; q < 3 * H; ++q) xn[q] = (h[q] - mean) * rstd;
      float m[H], u[H];
      ln_ff48(lw.msg, xn, m);
      ln_ff48(lw.edge, xn, u);
      if (edge_res) {
#pragma unroll
        for (int o = 0; o < H; ++o) u[o] += h[2 * H + o];
      }
      st16(e + k * H, u);
      float* ms = msg + (k - c0) * H;
#pragma unroll
      for (int o = 0; o < H; ++o) ms[o] = m[o];
    }
    __syncthreads();
    if (active) {
      const int64_t kb = my_b > c0 ? my_b : c0;
      const int64_t ke = my_e < c1 ? my_e : c1;
      for (int64_t k = kb; k < ke; ++k) {
        const float* ms = msg + (k - c0) * H;
#pragma unroll
        for (int o = 0; o < H; ++o) agg[o] += ms[o];
      }
    }
    __syncthreads();
  }
  if (!active) return;
  // update(): node_mlp(aggr) with LayerNorm(16) pre-norm; residual (basic_layers.py:203-206, 224-225)
  float mean = 0.f;
#pragma unroll
  for (int o = 0; o < H; ++o) mean += agg[o];
  mean *= (1.0f / H);
  float var = 0.f;
#pragma unroll
  for (int o = 0; o < H; ++o) {
    const float dv = agg[o] - mean;
    var = __builtin_fmaf(dv, dv, var);
  }
  var *= (1.0f / H);
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
  float in[H], h1[H], out[H];
#pragma unroll
  for (int o = 0; o < H; ++o) in[o] = __builtin_fmaf((agg[o] - mean) * rstd, lw.node[o], lw.node[H + o]);
  const float* w = lw.node + 2 * H;
  linear16<H>(w, w + H * H, in, h1);
  ff_tail<H>(w + H * H + H, h1, out);
  if (node_res) {
    float xo[H];
    ld16(x + i * H, xo);
#pragma unroll
    for (int o = 0; o < H; ++o) out[o] += xo[o];
  }
  st16(xout + i * H, out);
}

static int egrid(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  return int(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace lspcg

using namespace lspcg;

struct lspcg_gnn {
  lspcg_ctx* ctx = nullptr;
  lspcg_gnn_desc d{};
  float* w = nullptr;
  int64_t nw = 0;
  // offsets into w
  int64_t o_node_enc = 0, o_edge_enc = 0, o_dec = 0;
  std::vector<int64_t> o_layer;  // per layer: node, edge, msg
  // workspace
  int64_t capN = -1, capE = -1;
  float *xa = nullptr, *xb = nullptr, *ecsc = nullptr;
  int32_t *ptr = nullptr, *cnt = nullptr, *perm = nullptr, *inv = nullptr, *src = nullptr, *dst = nullptr;
  void* scan_tmp = nullptr;
  size_t scan_bytes = 0;
};

static int64_t gnn_weight_count(const lspcg_gnn_desc& d) {
  int64_t n = ff_size(d.node_in, H) + ff_size(d.edge_in, H);
  n += int64_t(d.num_mp_layers) * ((2 * H + ff_size(H, H)) + 2 * (6 * H + ff_size(3 * H, H)));
  n += ff_size(3 * H, d.edge_out);
  return n;
}

static void gnn_free_ws(lspcg_gnn* g) {
  for (void* p : {(void*)g->xa, (void*)g->xb, (void*)g->ecsc, (void*)g->ptr, (void*)g->cnt, (void*)g->perm,
                  (void*)g->inv, (void*)g->src, (void*)g->dst, g->scan_tmp})
    (void)hipFree(p);
  g->xa = g->xb = g->ecsc = nullptr;
  g->ptr = g->cnt = g->perm = g->inv = g->src = g->dst = nullptr;
  g->scan_tmp = nullptr;
  g->capN = g->capE = -1;
}

static int gnn_reserve(lspcg_gnn* g, int64_t N, int64_t E) {
  if (N <= g->capN && E <= g->capE) return LSPCG_OK;
  gnn_free_ws(g);
  const int64_t n = N > 0 ? N : 1, e = E > 0 ? E : 1;
  LSPCG_HIP(hipMalloc(&g->xa, sizeof(float) * n * H));
  LSPCG_HIP(hipMalloc(&g->xb, sizeof(float) * n * H));
  LSPCG_HIP(hipMalloc(&g->ecsc, sizeof(float) * e * H));
  LSPCG_HIP(hipMalloc(&g->ptr, sizeof(int32_t) * (n + 1)));
  LSPCG_HIP(hipMalloc(&g->cnt, sizeof(int32_t) * (n + 1)));
  LSPCG_HIP(hipMalloc(&g->perm, sizeof(int32_t) * e));
  LSPCG_HIP(hipMalloc(&g->inv, sizeof(int32_t) * e));
  LSPCG_HIP(hipMalloc(&g->src, sizeof(int32_t) * e));
  LSPCG_HIP(hipMalloc(&g->dst, sizeof(int32_t) * e));
  g->scan_bytes = 0;
  LSPCG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, g->scan_bytes, g->cnt, g->ptr, int(n + 1), g->ctx->stream));
  LSPCG_HIP(hipMalloc(&g->scan_tmp, g->scan_bytes ? g->scan_bytes : 1));
  g->capN = N;
  g->capE = E;
  return LSPCG_OK;
}

extern "C" {

int lspcg_gnn_create(lspcg_ctx* ctx, const lspcg_gnn_desc* desc, const float* weights, int64_t nweights,
                     lspcg_gnn** out) {
  LSPCG_CHECK(ctx && desc && weights && out, LSPCG_ERR_ARG, "gnn_create: NULL argument");
  const lspcg_gnn_desc& d = *desc;
  LSPCG_CHECK(d.hidden == H, LSPCG_ERR_UNSUPPORTED, "gnn_create: hidden must be 16 (gnn.yaml gnn_features)");
  LSPCG_CHECK(d.mlp_layers == 2, LSPCG_ERR_UNSUPPORTED, "gnn_create: FeedForward num_layers must be 2");
  LSPCG_CHECK(d.node_in >= 1 && d.node_in <= kMaxIn && d.edge_in >= 1 && d.edge_in <= kMaxIn, LSPCG_ERR_UNSUPPORTED,
              "gnn_create: node_in / edge_in must be in [1, 32]");
  LSPCG_CHECK(d.edge_out == 1 || d.edge_out == 4 || d.edge_out == 9, LSPCG_ERR_UNSUPPORTED,
              "gnn_create: edge_out must be block_size^2 with block_size in {1,2,3}");
  LSPCG_CHECK(d.num_mp_layers >= 0 && d.num_mp_layers <= 64, LSPCG_ERR_ARG, "gnn_create: bad num_mp_layers");
  const int64_t need = gnn_weight_count(d);
  LSPCG_CHECK(nweights == need, LSPCG_ERR_ARG,
              "gnn_create: weight blob has " + std::to_string(nweights) + " floats, expected " + std::to_string(need));
  LSPCG_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<lspcg_gnn> g(new lspcg_gnn());
  g->ctx = ctx;
  g->d = d;
  g->nw = need;
  LSPCG_HIP(hipMalloc(&g->w, sizeof(float) * need));
  LSPCG_HIP(hipMemcpyAsync(g->w, weights, sizeof(float) * need, hipMemcpyDefault, ctx->stream));
  LSPCG_HIP(hipStreamSynchronize(ctx->stream));
  int64_t o = 0;
  g->o_node_enc = o;
  o += ff_size(d.node_in, H);
  g->o_edge_enc = o;
  o += ff_size(d.edge_in, H);
  for (int l = 0; l < d.num_mp_layers; ++l) {
    g->o_layer.push_back(o);
    o += 2 * H + ff_size(H, H);
    g->o_layer.push_back(o);
    o += 6 * H + ff_size(3 * H, H);
    g->o_layer.push_back(o);
    o += 6 * H + ff_size(3 * H, H);
  }
  g->o_dec = o;
  *out = g.release();
  return LSPCG_OK;
}

int lspcg_gnn_forward(lspcg_gnn* g, int64_t N, int64_t E, const float* x, const int64_t* edge_index,
                      const float* edge_attr, float* out) {
  LSPCG_CHECK(g && (N == 0 || x) && (E == 0 || (edge_index && edge_attr && out)), LSPCG_ERR_ARG,
              "gnn_forward: NULL argument");
  LSPCG_CHECK(N >= 0 && E >= 0 && N < (int64_t(1) << 31) && E < (int64_t(1) << 31), LSPCG_ERR_ARG,
              "gnn_forward: sizes out of range");
  LSPCG_HIP(hipSetDevice(g->ctx->device));
  int rc = gnn_reserve(g, N, E);
  if (rc) return rc;
  if (E == 0 || N == 0) return LSPCG_OK;
  hipStream_t st = g->ctx->stream;
  const lspcg_gnn_desc& d = g->d;
  // CSC of the edges by destination
  LSPCG_HIP(hipMemsetAsync(g->cnt, 0, sizeof(int32_t) * (N + 1), st));
  hipLaunchKernelGGL(k_csc_count, dim3(egrid(E)), dim3(kThreads), 0, st, E, edge_index, g->cnt);
  size_t tb = g->scan_bytes;
  LSPCG_HIP(hipcub::DeviceScan::ExclusiveSum(g->scan_tmp, tb, g->cnt, g->ptr, int(N + 1), st));
  LSPCG_HIP(hipMemsetAsync(g->cnt, 0, sizeof(int32_t) * (N + 1), st));
  hipLaunchKernelGGL(k_csc_fill, dim3(egrid(E)), dim3(kThreads), 0, st, E, edge_index, g->ptr, g->cnt, g->perm);
  hipLaunchKernelGGL(k_csc_sort, dim3(egrid(N)), dim3(kThreads), 0, st, N, edge_index, E, g->ptr, g->perm, g->inv,
                     g->src, g->dst);
  // encoders
  hipLaunchKernelGGL(k_node_enc, dim3(egrid(N)), dim3(kThreads), 0, st, N, d.node_in, g->w + g->o_node_enc, x, g->xa);
  hipLaunchKernelGGL(k_edge_enc, dim3(egrid(E)), dim3(kThreads), 0, st, E, d.edge_in, g->w + g->o_edge_enc,
                     edge_attr, g->perm, g->ecsc);
  // message passing
  float* xc = g->xa;
  float* xn = g->xb;
  const unsigned lg = unsigned((N + kThreads - 1) / kThreads);
  for (int l = 0; l < d.num_mp_layers; ++l) {
    LayerW lw{g->w + g->o_layer[3 * l], g->w + g->o_layer[3 * l + 1], g->w + g->o_layer[3 * l + 2]};
    hipLaunchKernelGGL(k_mp_layer, dim3(lg), dim3(kThreads), 0, st, N, lw, d.node_residual, d.edge_residual, g->ptr,
                       g->src, g->dst, xc, g->ecsc, xn);
    std::swap(xc, xn);
  }
  // decoder
  const float* wd = g->w + g->o_dec;
  if (d.edge_out == 1)
    hipLaunchKernelGGL(k_edge_dec<1>, dim3(egrid(E)), dim3(kThreads), 0, st, E, wd, edge_index, g->inv, g->ecsc, xc, out);
  else if (d.edge_out == 4)
    hipLaunchKernelGGL(k_edge_dec<4>, dim3(egrid(E)), dim3(kThreads), 0, st, E, wd, edge_index, g->inv, g->ecsc, xc, out);
  else
    hipLaunchKernelGGL(k_edge_dec<9>, dim3(egrid(E)), dim3(kThreads), 0, st, E, wd, edge_index, g->inv, g->ecsc, xc, out);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_gnn_destroy(lspcg_gnn* g) {
  if (!g) return LSPCG_OK;
  (void)hipSetDevice(g->ctx->device);
  gnn_free_ws(g);
  (void)hipFree(g->w);
  delete g;
  return LSPCG_OK;
}

}  // extern "C"
