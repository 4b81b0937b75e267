// GNN that infers the SPAI factor L: NodeEdgeProcessing.forward (neural_cg/nn/gnns.py:77-97)
// with FeedForward (basic_layers.py:73-109, num_layers = 2 -> Linear/GELU/Linear/GELU/Linear)
// and MPLayer (basic_layers.py:145-225, PyG 2.6.1 source_to_target flow: x_i = x[dst =
// edge_index[1]], x_j = x[src = edge_index[0]], messages summed at dst).  fp32.
//
// MFMA design (DESIGN.md "GNN"): every MLP runs on v_mfma_f32_16x16x4_f32 (exact fp32
// FMA chains).  A wave owns a tile of 16 items (edges or nodes); lane l = (item l&15,
// quarter q = l>>4).  Layers compute H^T = W * IN^T: the weights are the A operand (one f32
// per lane per 4-deep K step, pre-arranged on the host into per-lane "fragments" held in
// LDS), the activations the B operand.  The 16x16 accumulator of one layer (lane l: rows
// 4q..4q+3 of item l&15) is directly the next layer's B operand with K slot q of step s =
// hidden unit 4q+s -- no data movement between layers.  Input features are laid out so a
// lane's 4 K-slots of each 16-wide block are 4 contiguous floats: every row read/write is a
// 16-B access.  LayerNorm affine parameters are folded into the first Linear on the host.
//
// One message-passing layer is ONE kernel: a 256-thread workgroup owns 256 destination
// nodes and streams their incoming edges (kept in CSC order for the whole forward) in
// chunks of 256; per edge tile it computes the shared LayerNorm(48) statistics, the message
// MLP and the edge MLP (two interleaved MFMA chains), writes the updated edge feature in
// place and drops the message into LDS; after a barrier every node lane sums its messages
// in CSC order (deterministic, no atomics).  The node MLP then runs on 16-node tiles.
// Messages never touch HBM.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "lspcg_internal.hpp"

namespace lspcg {

constexpr int H = 16;        // hidden = node_features = edge_features
constexpr int CE = 256;      // edges per LDS chunk (256 x 16 x 4 B = 16 KiB)
constexpr int kMaxIn = 32;   // encoder input features supported

using f4 = float __attribute__((ext_vector_type(4)));

// FeedForward(in, out, hidden=16, num_layers=2) parameter block of the packed blob:
//   [W1 (16 x in) | b1 (16) | W2 (16 x 16) | b2 (16) | W3 (out x 16) | b3 (out)]
__host__ __device__ constexpr int ff_size(int in, int out) { return H * in + H + H * H + H + out * H + out; }

// Fragment block of one FeedForward (floats): [A1 (S1 x 64) | C1 (64 x 4) | A2 (4 x 64) |
// C2 (64 x 4) | A3 (4 x 64) | C3 (64 x 4)]
__host__ __device__ constexpr int frag_size(int s1) { return s1 * 64 + 5 * 256; }

// GELU(v) = v Phi(v) = max(v, 0) - |v| m(|v|),  m(a) = Phi(-a) = erfc(a / sqrt2) / 2 (either sign
// of v; nn.GELU's exact-erf form).  log2 m(a) on [0, 5.75] is a degree-6 polynomial (fp32
// coefficients fitted to the absolute GELU error a m(a); a clamps at 5.75, where m < 5e-9), so a
// value costs one exp2 and 6 FMAs -- no reciprocal (round 2's erfcc took rcp + exp2 + 10 FMAs):
// |GELU error| <= 5.2e-7 absolute against the exact erf GELU with fp32 evaluation, at the fp32
// rounding of GELU(v) itself (4.8e-7 at |v| = 9; round 3's unweighted degree-8 fit 4.1e-7,
// round 4's degree-7 one 5.3e-7), and the forward stays
// within ~1e-7 of the reference's (tests/test_gpu_gnn.py, 1e-5).  Two values at a time in packed fp32
// (v_pk_fma_f32); |v| and the clamp are one v_med3_f32 with the abs modifier.
using f2 = float __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, float c) { return __builtin_elementwise_fma(a, b, (f2)(c)); }
constexpr float kGeluClamp = 5.75f;
constexpr int kGeluDeg = 6;  // fitted to the GELU's absolute error |v| m(|v|) (iteratively reweighted
                              // least squares toward minimax): 5.1e-8 in exact arithmetic, 5.2e-7 with fp32
                              // evaluation -- the fp32 rounding of GELU(v) itself is 4.8e-7 at |v| = 9
constexpr float kGeluC[7] = {-0.999993085861206f,   -1.1512017250061035f,    -0.4587709605693817f,
                             -0.05341210961341858f, 0.008080719038844109f,   -0.0007692205253988504f,
                             3.309291059849784e-05f};
// max(v, 0) as one v_max_i32 on the bit pattern (negative floats, -0 included, are negative
// integers); fmaxf would add a canonicalising v_max
__device__ __forceinline__ float relu(float v) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0));
}
// min(|v|, clamp) as one v_med3_f32 with the abs modifier (fminf would add a canonicalising v_max)
__device__ __forceinline__ float abs_clamp(float v) { return __builtin_amdgcn_fmed3f(__builtin_fabsf(v), 0.0f, kGeluClamp); }
// K independent pairs, every step interleaved across them: a dependent packed op needs a wait
// state on gfx950, so one chain alone would issue an s_nop between every Horner step.
template <int K>
__device__ __forceinline__ void gelu_n(f2 (&v)[K]) {
  f2 a[K], p[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    a[k] = (f2){abs_clamp(v[k].x), abs_clamp(v[k].y)};
    p[k] = pfma(a[k], (f2)(kGeluC[kGeluDeg]), kGeluC[kGeluDeg - 1]);
  }
#pragma unroll
  for (int c = kGeluDeg - 2; c >= 0; --c)
#pragma unroll
    for (int k = 0; k < K; ++k) p[k] = pfma(a[k], p[k], kGeluC[c]);
  // the clamped |v| (a) multiplies m: for |v| > 5.75 that changes |v| m(|v|) < 2.6e-8 |v| / 5.75 by less
  // than its own size -- below fp32's half ulp of GELU(v) for v > 0 and 2.6e-8 absolute for v < 0 --
  // and the pair's last step is one v_pk_fma_f32 with a neg modifier (|v| would need two v_and)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const f2 e = (f2){__builtin_amdgcn_exp2f(p[k].x), __builtin_amdgcn_exp2f(p[k].y)};
    v[k] = __builtin_elementwise_fma(-a[k], e, (f2){relu(v[k].x), relu(v[k].y)});
  }
}
__device__ __forceinline__ f4 gelu4(f4 a) {
  f2 v[2] = {(f2){a.x, a.y}, (f2){a.z, a.w}};
  gelu_n<2>(v);
  return f4{v[0].x, v[0].y, v[1].x, v[1].y};
}
__device__ __forceinline__ void gelu4x2(f4& a, f4& b) {
  f2 v[4] = {(f2){a.x, a.y}, (f2){a.z, a.w}, (f2){b.x, b.y}, (f2){b.z, b.w}};
  gelu_n<4>(v);
  a = f4{v[0].x, v[0].y, v[1].x, v[1].y};
  b = f4{v[2].x, v[2].y, v[3].x, v[3].y};
}

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float comp(f4 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// One FeedForward's fragment block held in this lane's registers (the fused edge encoder of the
// first MP layer: its ~21 floats per lane fit beside the layer, whose occupancy is LDS-bound, so
// the per-tile weight reads leave the dependency chain)
template <int S1>
struct FragRegs {
  float a1[S1], a2[4], a3[4];
  f4 c1, c2, c3;
  __device__ __forceinline__ void load(const float* fr, int lane) {
#pragma unroll
    for (int s = 0; s < S1; ++s) a1[s] = fr[s * 64 + lane];
    const float* p = fr + S1 * 64;
    c1 = *reinterpret_cast<const f4*>(p + lane * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) a2[s] = p[256 + s * 64 + lane];
    c2 = *reinterpret_cast<const f4*>(p + 512 + lane * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) a3[s] = p[768 + s * 64 + lane];
    c3 = *reinterpret_cast<const f4*>(p + 1024 + lane * 4);
  }
};

// layers 2 and 3 of an FF on the layer-1 pre-activation `h` (in accumulator layout)
__device__ __forceinline__ f4 ff_tail(const float* fr, int s1, f4 h, int lane) {
  const float* a2 = fr + s1 * 64 + 256;
  const float* c2 = a2 + 256;
  const float* a3 = c2 + 256;
  const float* c3 = a3 + 256;
  h = gelu4(h);
  f4 h2 = *reinterpret_cast<const f4*>(c2 + lane * 4);
#pragma unroll
  for (int s = 0; s < 4; ++s) h2 = mfma(a2[s * 64 + lane], comp(h, s), h2);
  h2 = gelu4(h2);
  f4 o = *reinterpret_cast<const f4*>(c3 + lane * 4);
#pragma unroll
  for (int s = 0; s < 4; ++s) o = mfma(a3[s * 64 + lane], comp(h2, s), o);
  return o;
}

// Two FFs with 48 inputs sharing the same B operand (message + edge MLP of an MPLayer): the
// two dependent MFMA chains and the two GELU blocks are interleaved so they overlap (f32 MFMA:
// the F32 kernels, chosen by lspcg_gnn_create for weights past the split-f16 range; the default
// runs the split-f16 version below).
__device__ __forceinline__ void ff2_48(const float* fa, const float* fb, const float (&in)[12], int lane, f4& oa,
                                       f4& ob) {
  f4 ha = *reinterpret_cast<const f4*>(fa + 12 * 64 + lane * 4);
  f4 hb = *reinterpret_cast<const f4*>(fb + 12 * 64 + lane * 4);
#pragma unroll
  for (int s = 0; s < 12; ++s) {
    ha = mfma(fa[s * 64 + lane], in[s], ha);
    hb = mfma(fb[s * 64 + lane], in[s], hb);
  }
  const float* a2 = fa + 12 * 64 + 256;
  const float* b2 = fb + 12 * 64 + 256;
  gelu4x2(ha, hb);
  f4 h2a = *reinterpret_cast<const f4*>(a2 + 256 + lane * 4);
  f4 h2b = *reinterpret_cast<const f4*>(b2 + 256 + lane * 4);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    h2a = mfma(a2[s * 64 + lane], comp(ha, s), h2a);
    h2b = mfma(b2[s * 64 + lane], comp(hb, s), h2b);
  }
  gelu4x2(h2a, h2b);
  const float* a3 = a2 + 512;
  const float* b3 = b2 + 512;
  oa = *reinterpret_cast<const f4*>(a3 + 256 + lane * 4);
  ob = *reinterpret_cast<const f4*>(b3 + 256 + lane * 4);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    oa = mfma(a3[s * 64 + lane], comp(h2a, s), oa);
    ob = mfma(b3[s * 64 + lane], comp(h2b, s), ob);
  }
}

// ---- The message + edge MLPs of an MPLayer on f16 MFMAs with split operands -----------------
// On gfx950 an f32 MFMA and a vector instruction never execute together on a SIMD (the layer's PMC:
// SQ_VALU_MFMA_COEXEC_CYCLES = 0, MFMA 47 % + VALU 44 % of the cycles; tools/coexec_probe.hip: one
// f32 MFMA plus 8 FMAs take the sum of both), while an f16 MFMA runs beside the VALU.  So the two
// MLPs' products go to v_mfma_f32_16x16x32_f16 / 16x16x16f16 with every fp32 operand split into an
// f16 pair, x = xh + xl (RNE; x - xh is exact in fp32): W x ~ Wl xh + Wh xl + Wh xh (the dropped
// Wl xl is ~2^-22 relative), products exact and summed in fp32.  Each weight matrix is scaled by a
// power of two 2^s (max |W| 2^s in [2^10, 2^11): its low halves stay normal f16) and the
// accumulator by 2^-s after the chain.  Error vs an fp64 forward ~5e-8 at kuhn / Poisson sizes,
// the same order as the fp32 forward's own (2e-8; tests/test_gpu_gnn.py holds it to 1e-5).
// Activations must stay below f16's 65504 (LayerNorm outputs are |v| <= 6.9; hidden layers are
// GELU outputs of O(1..10) pre-activations).
using h4 = _Float16 __attribute__((ext_vector_type(4)));
using hf2 = _Float16 __attribute__((ext_vector_type(2)));

// f16 block of one FeedForward(48 -> 16 -> 16 -> out) (dwords, 64 lanes): [W1 hi, K block 0 / 1 / 2
// (2 dwords = 4 halves per lane each) | W1 lo, blocks 0 / 1 / 2 | C1 (4 floats / lane) | W2 hi | W2 lo |
// C2 | W3 hi | W3 lo | C3 | 2^-s1, 2^-s2, 2^-s3, pad].  Every product is a v_mfma_f32_16x16x16f16:
// K slot (q, j) of block i is the lane's in[4i + j] (feature 16i + 4q + j, as feat48); C = 2^s b in
// accumulator layout.  (v_mfma_f32_16x16x32_f16 -- one instruction for blocks 0 and 1 -- lost its
// operands: hipcc reused its A / B registers for VALU results right after issue, and the products
// went missing in the edge decoder; 16x16x16 has no such hazard gap.)
constexpr int kH48 = 2052;
constexpr int kH48W1h = 0, kH48W1l = 384, kH48C1 = 768;
constexpr int kH48W2h = 1024, kH48W2l = 1152, kH48C2 = 1280, kH48W3h = 1536, kH48W3l = 1664, kH48C3 = 1792;
constexpr int kH48S = 2048;

// (a, b) -> packed f16 pairs hi = RNE(a, b), lo = RNE(a - hi, b - hi) (x - hi is exact in fp32).
// The residuals come straight from the f16 halves: v_fma_mix_f32 reads src0 as f16 (lo or hi half
// by op_sel), so hi is never converted back to f32 and there is no packed subtract -- 4 instead of 5
// instructions per pair, 2 of them packed-rate fewer (the compiler does not select the mix form
// itself).  Exact, so the same bits; the asm results feed a compiler-emitted conversion, never an
// MFMA operand (an MFMA reading a VGPR written inside inline asm needs wait states hipcc does not
// insert -- round 4's v_fma_mix{lo,hi}_f16 form, which wrote the f16 operand itself, measured no
// faster for that reason).  Forward 4.49 vs 4.63 ms at kuhn101 (profiles/r5_gnn_ab_mix.jsonl).
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
  const hf2 h = __builtin_convertvector((f2){a, b}, hf2);
  hi = __builtin_bit_cast(unsigned, h);
  float ra, rb;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(ra) : "v"(hi), "v"(a));
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(rb) : "v"(hi), "v"(b));
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f2){ra, rb}, hf2));
}
__device__ __forceinline__ void split4(const float* v, h4& hi, h4& lo) {
  unsigned h[2], l[2];
  split2(v[0], v[1], h[0], l[0]);
  split2(v[2], v[3], h[1], l[1]);
  hi = __builtin_bit_cast(h4, (unsigned __attribute__((ext_vector_type(2)))){h[0], h[1]});
  lo = __builtin_bit_cast(h4, (unsigned __attribute__((ext_vector_type(2)))){l[0], l[1]});
}
__device__ __forceinline__ h4 ldh4(const float* p) { return *reinterpret_cast<const h4*>(p); }
__device__ __forceinline__ f4 mfma16h(h4 a, h4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }

// layer 1 of a 48-input FeedForward: acc = C + sum over the 3 K blocks of Wl xh, then Wh xl, then Wh xh
__device__ __forceinline__ f4 layer48h(const float* w, const h4 (&xh)[3], const h4 (&xl)[3], int lane,
                                      float cmul = 1.0f) {
  h4 wh[3], wlo[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    wh[i] = ldh4(w + kH48W1h + 128 * i + 2 * lane);
    wlo[i] = ldh4(w + kH48W1l + 128 * i + 2 * lane);
  }
  f4 acc = ld4(w + kH48C1 + 4 * lane) * cmul;  // cmul: a power of two (1 but for ff1_48's guard)
#pragma unroll
  for (int i = 0; i < 3; ++i) acc = mfma16h(wlo[i], xh[i], acc);
#pragma unroll
  for (int i = 0; i < 3; ++i) acc = mfma16h(wh[i], xl[i], acc);
#pragma unroll
  for (int i = 0; i < 3; ++i) acc = mfma16h(wh[i], xh[i], acc);
  return acc;
}

// one 16x16 layer on split operands: acc = C + Wl xh + Wh xl + Wh xh (small terms first)
__device__ __forceinline__ f4 layer16h(const float* w, int oh, int ol, int oc, float unscale, h4 xh, h4 xl,
                                       int lane) {
  const h4 wh = ldh4(w + oh + 2 * lane), wlo = ldh4(w + ol + 2 * lane);
  f4 acc = ld4(w + oc + 4 * lane);
  acc = mfma16h(wlo, xh, acc);
  acc = mfma16h(wh, xl, acc);
  acc = mfma16h(wh, xh, acc);
  return acc * unscale;
}

// us[0..2] / us[3..5]: the unscale factors 2^-s of the message / edge MLP's three layers (uniform:
// read once per kernel from the global blob, so they live in SGPRs)
__device__ __forceinline__ void ff2_48(const float* fa, const float* fb, const float (&in)[12], int lane, f4& oa,
                                       f4& ob, const float (&us)[6]) {
  h4 xh[3], xl[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) split4(in + 4 * i, xh[i], xl[i]);
  f4 ha = layer48h(fa, xh, xl, lane);
  f4 hb = layer48h(fb, xh, xl, lane);
  ha *= us[0];
  hb *= us[3];
  gelu4x2(ha, hb);
  h4 xah, xal, xbh, xbl;
  {
    const float va[4] = {ha.x, ha.y, ha.z, ha.w}, vb[4] = {hb.x, hb.y, hb.z, hb.w};
    split4(va, xah, xal);
    split4(vb, xbh, xbl);
  }
  f4 h2a = layer16h(fa, kH48W2h, kH48W2l, kH48C2, us[1], xah, xal, lane);
  f4 h2b = layer16h(fb, kH48W2h, kH48W2l, kH48C2, us[4], xbh, xbl, lane);
  gelu4x2(h2a, h2b);
  {
    const float va[4] = {h2a.x, h2a.y, h2a.z, h2a.w}, vb[4] = {h2b.x, h2b.y, h2b.z, h2b.w};
    split4(va, xah, xal);
    split4(vb, xbh, xbl);
  }
  // the last layer's accumulators are returned as they stand (2^s3 times the outputs): the
  // caller folds the unscale into the message aggregation / the edge residual's FMA
  oa = layer16h(fa, kH48W3h, kH48W3l, kH48C3, 1.0f, xah, xal, lane);
  ob = layer16h(fb, kH48W3h, kH48W3l, kH48C3, 1.0f, xbh, xbl, lane);
}

// FeedForward(16 -> 16 -> 16 -> 16) (the node MLP) on split operands: block [W1 hi | W1 lo | C1 | W2 hi |
// W2 lo | C2 | W3 hi | W3 lo | C3 | 2^-s1..3, pad | the encoder's magnitude bounds B1, c1, B2, c2
// (ff1_16_enc)] (kH16 dwords; K slot (q, j) = the lane's in[j], i.e.
// feature 4q + j, as feat16); us = its 2^-s factors
constexpr int kH16 = 1548;
constexpr int kH16S = 1536;
__device__ __forceinline__ f4 ff1_16(const float* fa, const float (&in)[4], int lane, const float (&us)[3]) {
  h4 xh, xl;
  split4(in, xh, xl);
  f4 h = gelu4(layer16h(fa, 0, 128, 256, us[0], xh, xl, lane));
  {
    const float va[4] = {h.x, h.y, h.z, h.w};
    split4(va, xh, xl);
  }
  h = gelu4(layer16h(fa, 512, 640, 768, us[1], xh, xl, lane));
  {
    const float va[4] = {h.x, h.y, h.z, h.w};
    split4(va, xh, xl);
  }
  return layer16h(fa, 1024, 1152, 1280, us[2], xh, xl, lane);
}

// 2^t as a float (t in [-126, 127])
__device__ __forceinline__ float exp2i(int t) { return __builtin_bit_cast(float, unsigned(t + 127) << 23); }

// max over the 4 lanes of an item (l, l^16, l^32, l^48): row-swap permutes, as swap_sum16 / 32 below
__device__ __forceinline__ float swap_max16(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const unsigned long long r = __builtin_bit_cast(unsigned long long, __builtin_amdgcn_permlane16_swap(u, u, false, false));
  return fmaxf(__builtin_bit_cast(float, unsigned(r)), __builtin_bit_cast(float, unsigned(r >> 32)));
}
__device__ __forceinline__ float swap_max32(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const unsigned long long r = __builtin_bit_cast(unsigned long long, __builtin_amdgcn_permlane32_swap(u, u, false, false));
  return fmaxf(__builtin_bit_cast(float, unsigned(r)), __builtin_bit_cast(float, unsigned(r >> 32)));
}

// Per-edge power-of-two input scale of the fused edge encoder.  Raw edge features (the matrix
// values, any magnitude: data.py:247-267 allows normalize_matrix="none") are multiplied by 2^t,
// t chosen per edge so the largest |feature| of the edge lands in [2^10, 2^11); the bias of that
// edge's output column is scaled alike and the column unscaled after the chain (an MFMA column is
// one edge, and lane l holds edge l & 15's inputs and outputs, so no lane exchange beyond the
// edge's own 4 lanes).  Without it an input >= 65520 splits into an infinite f16 and inputs below
// 2^-14 lose their low bits in f16 subnormals; with it the split's error is relative to the edge's
// largest feature, like an fp32 dot product's.  Exact (powers of two): inputs already in f16's
// normal range give the same bits as unscaled, and the scale depends on the edge alone.
__device__ __forceinline__ int enc_scale_exp(float m) {
  // m in [2^(e-127), 2^(e-126)) -> [2^10, 2^11); clamped to [-60, 60]: a zero edge (e = 0) keeps its
  // bias finite (|C| 2^60 < 2^128), an inf / NaN one (e = 255) stays inf / NaN
  const int e = int(__builtin_bit_cast(unsigned, m) >> 23);  // m >= 0: no sign bit
  return min(max(137 - e, -60), 60);  // v_med3_i32
}

// hidden activations of the edge decoder follow the raw edge features' magnitude (through the edge
// residuals): an EDGE whose largest |h| reaches 2^15 has its hidden values scaled by 2^t (t < 0, so
// its largest lands in [2^14, 2^15)) and the next layer undoes it for that edge's column (its bias
// times 2^t, its product times 2^-t), so no split overflows f16 -- per edge, like the input scale,
// so a small edge sharing a tile with a huge one keeps its own relative accuracy (a wave-wide
// factor would push its low halves into f16 subnormals).  The check is 3 VALU + a wave-uniform
// branch that normal magnitudes never take; returns this lane's edge's t (0: none).
__device__ __forceinline__ int enc_guard(f4& h) {
  const float m = fmaxf(fmaxf(fabsf(h.x), fabsf(h.y)), fmaxf(fabsf(h.z), fabsf(h.w)));
  if (!__builtin_amdgcn_ballot_w64(!(m < 32768.0f))) return 0;  // NaN takes the slow path too
  const float w = swap_max32(swap_max16(m));                   // the edge's 4 lanes
  const int e = int(__builtin_bit_cast(unsigned, w) >> 23) & 0xff;
  const int t = (w >= 32768.0f && e != 0xff) ? 141 - e : 0;   // -113 <= t <= -1; inf / NaN propagate
  h *= exp2i(t);
  return t;
}

// one 16x16 layer on split operands: acc = C cmul + Wl xh + Wh xl + Wh xh, times omul (cmul / omul
// powers of two: the input's scale and the weights' unscale with the input's scale undone)
__device__ __forceinline__ f4 layer16h_sc(const float* w, int oh, int ol, int oc, float cmul, float omul, h4 xh,
                                          h4 xl, int lane) {
  const h4 wh = ldh4(w + oh + 2 * lane), wlo = ldh4(w + ol + 2 * lane);
  f4 acc = ld4(w + oc + 4 * lane) * cmul;
  acc = mfma16h(wlo, xh, acc);
  acc = mfma16h(wh, xl, acc);
  acc = mfma16h(wh, xh, acc);
  return acc * omul;
}
__device__ __forceinline__ f4 layer16h_guarded(const float* w, int oh, int ol, int oc, float unscale, int t, h4 xh,
                                               h4 xl, int lane) {
  if (!__builtin_amdgcn_ballot_w64(t != 0)) return layer16h(w, oh, ol, oc, unscale, xh, xl, lane);  // wave-uniform
  return layer16h_sc(w, oh, ol, oc, exp2i(t), unscale * exp2i(-t), xh, xl, lane);  // per lane = per edge
}

// the fused edge encoder FeedForward(fin -> 16 -> 16 -> 16) (kH16 block) on raw features `in`
// (this lane's features 4q .. 4q+3 of edge lane & 15), scaled per edge (enc_scale_exp)
__device__ __forceinline__ f4 ff1_16_enc(const float* fa, const float (&in)[4], int lane, const float (&us)[3],
                                         const float (&bd)[5]) {
  const float m = swap_max32(swap_max16(fmaxf(fmaxf(fabsf(in[0]), fabsf(in[1])), fmaxf(fabsf(in[2]), fabsf(in[3])))));
  const unsigned scb = unsigned(enc_scale_exp(m) + 127) << 23;
  const float sc = __builtin_bit_cast(float, scb), isc = __builtin_bit_cast(float, 0x7f000000u - scb);  // 2^t, 2^-t
  h4 xh, xl;
  {
    const float v[4] = {in[0] * sc, in[1] * sc, in[2] * sc, in[3] * sc};
    split4(v, xh, xl);
  }
  const f4 z1 = layer16h_sc(fa, 0, 128, 256, sc, us[0] * isc, xh, xl, lane);
  // the hidden layers' scale: |h1| <= B1 m + c1 and |h2| <= B2 |h1| + c2 (B = max row sum of |W|,
  // c = max |bias| + 0.17 for GELU's negative lobe; host constants bd), so 2^k with k = min(0, 14 -
  // exponent of the larger bound) keeps every split below 2^15.  bd[4] holds the largest m
  // for which k = 0: a wave with no larger edge maximum (every wave on normal data) skips it.
  if (!__builtin_amdgcn_ballot_w64(!(m <= bd[4]))) {
    f4 h = gelu4(z1);
    {
      const float va[4] = {h.x, h.y, h.z, h.w};
      split4(va, xh, xl);
    }
    h = gelu4(layer16h(fa, 512, 640, 768, us[1], xh, xl, lane));
    {
      const float va[4] = {h.x, h.y, h.z, h.w};
      split4(va, xh, xl);
    }
    return layer16h(fa, 1024, 1152, 1280, us[2], xh, xl, lane);
  }
  const float h1b = fmaf(bd[0], m, bd[1]);
  const float hb = fmaxf(h1b, fmaf(bd[2], h1b, bd[3]));
  const int ke = int(__builtin_bit_cast(unsigned, hb) >> 23);
  const unsigned hsb = unsigned(min(max(141 - ke, -100), 0) + 127) << 23;
  const float hs = __builtin_bit_cast(float, hsb), ihs = __builtin_bit_cast(float, 0x7f000000u - hsb);
  f4 h = gelu4(z1) * hs;
  {
    const float va[4] = {h.x, h.y, h.z, h.w};
    split4(va, xh, xl);
  }
  h = gelu4(layer16h_sc(fa, 512, 640, 768, hs, us[1] * ihs, xh, xl, lane)) * hs;
  {
    const float va[4] = {h.x, h.y, h.z, h.w};
    split4(va, xh, xl);
  }
  return layer16h_sc(fa, 1024, 1152, 1280, hs, us[2] * ihs, xh, xl, lane);
}

// one FeedForward(48 -> 16 -> 16 -> out) on split operands (the edge decoder); us = its 2^-s
// factors.  Its input -- the edge state and both endpoints' node states -- has no LayerNorm in
// front (gnns.py:88-95), so it carries the magnitude of the raw edge features through the edge
// residuals: an edge whose largest |input| reaches 2^15 is scaled down by a power of two (its bias
// column alike, its output column back; exact), and each hidden layer by enc_guard.  Normal
// magnitudes never leave the fast path (a max and a compare per value pair).
__device__ __forceinline__ f4 ff1_48(const float* fa, const float (&in)[12], int lane, const float (&us)[3]) {
  float v[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) v[i] = in[i];
  float cmul = 1.0f, omul = us[0];
  {
    float m = fmaxf(fabsf(v[0]), fabsf(v[1]));
#pragma unroll
    for (int i = 2; i < 12; ++i) m = fmaxf(m, fabsf(v[i]));
    if (__builtin_amdgcn_ballot_w64(!(m < 32768.0f))) {  // wave-uniform; rare
      m = swap_max32(swap_max16(m));
      const int e = int(__builtin_bit_cast(unsigned, m) >> 23) & 0xff;
      const int t = (m >= 32768.0f && e != 0xff) ? 141 - e : 0;  // this edge's largest -> [2^14, 2^15)
      cmul = exp2i(t);
      omul = us[0] * exp2i(-t);
#pragma unroll
      for (int i = 0; i < 12; ++i) v[i] *= cmul;
    }
  }
  h4 xh[3], xl[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) split4(v + 4 * i, xh[i], xl[i]);
  f4 ha = gelu4(layer48h(fa, xh, xl, lane, cmul) * omul);
  int tg = enc_guard(ha);
  h4 xah, xal;
  {
    const float va[4] = {ha.x, ha.y, ha.z, ha.w};
    split4(va, xah, xal);
  }
  f4 h2 = gelu4(layer16h_guarded(fa, kH48W2h, kH48W2l, kH48C2, us[1], tg, xah, xal, lane));
  tg = enc_guard(h2);
  {
    const float va[4] = {h2.x, h2.y, h2.z, h2.w};
    split4(va, xah, xal);
  }
  return layer16h_guarded(fa, kH48W3h, kH48W3l, kH48C3, us[2], tg, xah, xal, lane);
}

template <int S1>
__device__ __forceinline__ f4 ff_tile_regs(const FragRegs<S1>& w, const float (&in)[S1]) {
  f4 h = w.c1;
#pragma unroll
  for (int s = 0; s < S1; ++s) h = mfma(w.a1[s], in[s], h);
  h = gelu4(h);
  f4 h2 = w.c2;
#pragma unroll
  for (int s = 0; s < 4; ++s) h2 = mfma(w.a2[s], comp(h, s), h2);
  h2 = gelu4(h2);
  f4 o = w.c3;
#pragma unroll
  for (int s = 0; s < 4; ++s) o = mfma(w.a3[s], comp(h2, s), o);
  return o;
}

template <int S1>
__device__ __forceinline__ f4 ff_tile(const float* fr, const float (&in)[S1], int lane) {
  f4 h = *reinterpret_cast<const f4*>(fr + S1 * 64 + lane * 4);
#pragma unroll
  for (int s = 0; s < S1; ++s) h = mfma(fr[s * 64 + lane], in[s], h);
  return ff_tail(fr, S1, h, lane);
}



__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// Sum over the 4 K-quarters of an item (lanes l, l^16, l^32, l^48), every lane gets the total:
// gfx950's row-swap permutes (VALU, no LDS round trip like ds_bpermute).  swap(v, v) returns the
// own row's value in one register and the partner row's in the other.  (The pair is read through
// a 64-bit bit_cast: subscripting the builtin's result folds both halves into element 0.)
__device__ __forceinline__ float swap_sum16(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const unsigned long long r = __builtin_bit_cast(unsigned long long, __builtin_amdgcn_permlane16_swap(u, u, false, false));
  return __builtin_bit_cast(float, unsigned(r)) + __builtin_bit_cast(float, unsigned(r >> 32));
}
__device__ __forceinline__ float swap_sum32(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const unsigned long long r = __builtin_bit_cast(unsigned long long, __builtin_amdgcn_permlane32_swap(u, u, false, false));
  return __builtin_bit_cast(float, unsigned(r)) + __builtin_bit_cast(float, unsigned(r >> 32));
}
__device__ __forceinline__ float quad_sum(float v) { return swap_sum32(swap_sum16(v)); }

// 48-feature block layout of a lane: in[s], s = 4*block + c  <->  feature 16*block + 4q + c
__device__ __forceinline__ void pack12(f4 b0, f4 b1, f4 b2, float (&v)[12]) {
  v[0] = b0.x; v[1] = b0.y; v[2] = b0.z; v[3] = b0.w;
  v[4] = b1.x; v[5] = b1.y; v[6] = b1.z; v[7] = b1.w;
  v[8] = b2.x; v[9] = b2.y; v[10] = b2.z; v[11] = b2.w;
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

// Fast path for row-major sorted edges with a symmetric pattern (every matrix graph of the
// reference: edge_index comes from a CSR, data.py:471-536): the incoming edges of node c, in
// ascending source order, are exactly the outgoing edges of c, so edge e = (r -> c) takes CSC slot
// p = position of r in row c -- a binary search, no atomics and no sort.  flag bit 1: edges
// not row-major strictly sorted, bit 2: pattern not symmetric (-> generic path).
__global__ void k_csc_rowstart(int64_t N, int64_t E, const int64_t* __restrict__ ei, int32_t* __restrict__ ptr,
                               int* flag) {
  // ptr[r] = first edge with src >= r: edge e writes it for the rows src[e-1] < r <= src[e] (and
  // the virtual edge E for the rows after the last source), one coalesced pass over the sources
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e <= E; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = e < E ? ei[e] : N;
    const int64_t rp = e > 0 ? ei[e - 1] : -1;
    if (e < E) {
      if (r < 0 || r >= N) atomicOr(flag, 1);
      if (e + 1 < E) {
        const int64_t r1 = ei[e + 1];
        if (r > r1 || (r == r1 && ei[E + e] >= ei[E + e + 1])) atomicOr(flag, 1);
      }
    }
    const int64_t lo = rp + 1 > 0 ? rp + 1 : 0, hi = r < N ? r : N;
    for (int64_t rr = lo; rr <= hi; ++rr) ptr[rr] = int32_t(e);
  }
}

// Symmetric, strictly sorted pattern (k_csc_rowstart's check): the CSC slots of destination c
// are CSR row c's own slots, and the slot of edge e = (r, c) is the position of r in row c --
// the slot <-> edge map is an involution (perm, slot -> edge, is its own inverse), and slot k's
// endpoints are (src, dst) = (ei[E+k], ei[k]).  Every
// write is therefore at the thread's own index (coalesced); only the search in row c gathers.
__global__ void k_csc_sym(int64_t E, const int64_t* __restrict__ ei, const int32_t* __restrict__ ptr,
                          int32_t* __restrict__ perm, int32_t* __restrict__ src, int32_t* __restrict__ dst,
                          int* flag) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = ei[e], c = ei[E + e];
    const int32_t end = ptr[c + 1];
    int32_t lo = ptr[c], hi = end;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (ei[E + mid] < r) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= end || ei[E + lo] != r) atomicOr(flag, 2);
    perm[e] = lo;
    src[e] = int32_t(c);
    dst[e] = int32_t(r);
  }
}

// ---------------------------------------------------------------------------
// Encoders / decoder (16-item MFMA tiles, 4 waves per workgroup, grid-stride over tiles)
// ---------------------------------------------------------------------------
// Encoder input layout: K slot q of step s = input feature 4s + q (zero past `fin`).  Items are
// visited in output order, so the 64-B output rows are written coalesced; EDGE: CSC slot m reads
// the (few-float) input row of its edge perm[m] -- a gather from a small, cache-resident array
// instead of a scatter of 64-B rows into the [E,16] edge state.
template <bool EDGE>
__global__ void __launch_bounds__(256) k_encode(int64_t M, int fin, const float* __restrict__ fr,
                                               const float* __restrict__ in, const int32_t* __restrict__ inidx,
                                               float* __restrict__ out) {
  const int lane = threadIdx.x & 63, it = lane & 15, q = lane >> 4;
  const int s1 = (fin + 3) / 4;
  const int64_t ntiles = (M + 15) / 16;
  for (int64_t t = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); t < ntiles; t += int64_t(gridDim.x) * 4) {
    const int64_t m = t * 16 + it;
    const bool valid = m < M;
    const int64_t mm = valid ? m : M - 1;
    const int64_t irow = EDGE ? int64_t(inidx[mm]) : mm;
    f4 h = ld4(fr + s1 * 64 + lane * 4);
    for (int s = 0; s < s1; ++s) {
      const int f = 4 * s + q;
      const float v = f < fin ? in[irow * fin + f] : 0.f;
      h = mfma(fr[s * 64 + lane], v, h);
    }
    const f4 o = ff_tail(fr, s1, h, lane);
    if (valid) st4(out + mm * H + 4 * q, o);
  }
}

// out[e] = edge_dec(cat[e_attr, x[src], x[dst]])  (gnns.py:88-95; original edge order).  Visits
// edges e, gathering each 64-B edge-state row from its CSC slot inv[e]: measured faster than
// visiting slots and scattering the OUT-float results (0.59 vs 0.67 ms at E = 15.2 M).
template <bool F32, int OUT, typename IT>
__global__ void __launch_bounds__(256) k_edge_dec(int64_t E, const float* __restrict__ fr,
                                                 const IT* __restrict__ ra, const IT* __restrict__ rb,
                                                 const int32_t* __restrict__ inv,
                                                 const float* __restrict__ ecsc, const float* __restrict__ x,
                                                 float* __restrict__ out) {
  // the decoder's fragment block in LDS (8 KiB): the per-tile weight reads stay off the gathers'
  // memory queue
  constexpr int kDec = F32 ? frag_size(12) : kH48;  // f32 fragments / split-f16 block (ff1_48)
  const float us[3] = {F32 ? 1.f : fr[kH48S], F32 ? 1.f : fr[kH48S + 1], F32 ? 1.f : fr[kH48S + 2]};
  __shared__ __attribute__((aligned(16))) float wd[kDec];
  for (int i = threadIdx.x; i < kDec / 4; i += 256) reinterpret_cast<f4*>(wd)[i] = ld4(fr + 4 * i);
  __syncthreads();
  const int lane = threadIdx.x & 63, it = lane & 15, q = lane >> 4;
  const int64_t ntiles = (E + 15) / 16;
  for (int64_t t = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); t < ntiles; t += int64_t(gridDim.x) * 4) {
    const int64_t e = t * 16 + it;
    const bool valid = e < E;
    const int64_t ee = valid ? e : E - 1;
    float in[12];
    pack12(ld4(ecsc + int64_t(inv[ee]) * H + 4 * q), ld4(x + int64_t(ra[ee]) * H + 4 * q), ld4(x + int64_t(rb[ee]) * H + 4 * q), in);
    f4 o;
    if constexpr (F32) o = ff_tile<12>(wd, in, lane);
    else o = ff1_48(wd, in, lane, us);
    if (valid) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * q + r < OUT) out[ee * OUT + 4 * q + r] = comp(o, r);
    }
  }
}

// ---------------------------------------------------------------------------
// One MPLayer (basic_layers.py:193-225) as one kernel
// ---------------------------------------------------------------------------
// fragment blocks of one layer, [msg | edge | node]: f32 fragments or split-f16 blocks (ff2_48, ff1_16)
constexpr int frag48(bool f32) { return f32 ? frag_size(12) : kH48; }
constexpr int frag16(bool f32) { return f32 ? frag_size(4) : kH16; }
constexpr int layer_frag(bool f32) { return 2 * frag48(f32) + frag16(f32); }

// S1E > 0 (first layer): the edge encoder is fused in -- the layer's input edge state is computed
// from the raw edge features (fin <= 4 S1E floats of edge perm[k], fragment block `fenc` read
// through the cache, not LDS) instead of read back from an [E,16] pass of k_encode<true>.
template <bool F32, int S1E>
__global__ void __launch_bounds__(256, 4) k_mp_layer(int64_t N, const float* __restrict__ frag, int node_res,
                                                 int edge_res, const int32_t* __restrict__ ptr,
                                                 const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                                 const float* __restrict__ x, float* __restrict__ e,
                                                 float* __restrict__ xout, const float* __restrict__ fenc, int fin,
                                                 const float* __restrict__ eattr, const int32_t* __restrict__ perm) {
  [[maybe_unused]] constexpr int SE = S1E > 0 ? S1E : 1;
  constexpr int kLayerFrag = layer_frag(F32), kFrag48 = frag48(F32);
  __shared__ __attribute__((aligned(16))) float wl[kLayerFrag];
  __shared__ __attribute__((aligned(16))) float msg[CE * H];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, it = lane & 15, q = lane >> 4;
  for (int i = tid; i < kLayerFrag / 4; i += 256) reinterpret_cast<f4*>(wl)[i] = ld4(frag + 4 * i);
  __syncthreads();
  [[maybe_unused]] FragRegs<SE> wenc;
  if constexpr (F32 && S1E > 0) wenc.load(fenc, lane);
  const float* fmsg = wl;
  // split-f16 unscale factors (unused by the F32 kernels, whose blob has none at these offsets)
  const float us[6] = {F32 ? 1.f : frag[kH48S], F32 ? 1.f : frag[kH48S + 1], F32 ? 1.f : frag[kH48S + 2],
                       F32 ? 1.f : frag[kH48 + kH48S], F32 ? 1.f : frag[kH48 + kH48S + 1],
                       F32 ? 1.f : frag[kH48 + kH48S + 2]};
  const float usn[3] = {F32 ? 1.f : frag[2 * kH48 + kH16S], F32 ? 1.f : frag[2 * kH48 + kH16S + 1],
                        F32 ? 1.f : frag[2 * kH48 + kH16S + 2]};
  const float* fedge = wl + kFrag48;
  const float* fnode = wl + 2 * kFrag48;
  const int n0 = blockIdx.x * 256;
  const int n1 = n0 + 256 < N ? n0 + 256 : int(N);
  const int k0 = ptr[n0], k1 = ptr[n1];
  f4 agg[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) agg[j] = f4{0.f, 0.f, 0.f, 0.f};

  // Edge tiles T = 0..NT-1 of this workgroup (16 CSC edges each); wave w takes T = w, w+4, ...
  // Software pipeline: while tile T is computed, the gathers of tile T+4 and the index loads of
  // tile T+8 are in flight.  Prefetches past the last tile are clamped to the last edge (issued
  // unconditionally: no exec-mask branches), indices are 32-bit (E < 2^31, checked by the host),
  // and the 4 tiles of a chunk are unrolled so the prefetch registers rotate without moves.
  const int NT = (k1 - k0 + 15) / 16;
  const int klast = k1 - 1;
  auto edge_of = [&](int T) { const int k = k0 + T * 16 + it; return k < k1 ? k : klast; };
  int qd = 0, qs = 0, qe = 0;
  f4 pxd{}, pxs{}, pea{};
  // fused encoder, this lane's raw input features of the prefetched edge: F32, K slot q of step s =
  // feature 4s + q (f32 fragments); split-f16, features 4q .. 4q+3 (the kH16 block fenc)
  constexpr int NPIN = F32 ? SE : 4;
  float pin[NPIN];
  auto load_in = [&](int row) {
#pragma unroll
    for (int s = 0; s < NPIN; ++s) {
      const int f = F32 ? 4 * s + q : 4 * q + s;
      pin[s] = f < fin ? eattr[row * fin + f] : 0.f;
    }
  };
  float use[3] = {0.f, 0.f, 0.f}, ebd[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (!F32 && S1E > 0) {
    use[0] = fenc[kH16S];
    use[1] = fenc[kH16S + 1];
    use[2] = fenc[kH16S + 2];
#pragma unroll
    for (int j = 0; j < 5; ++j) ebd[j] = fenc[kH16S + 4 + j];
  }
  if (wave < NT) {
    const int kk = edge_of(wave);
    qd = dst[kk];
    qs = src[kk];
    pxd = ld4(x + qd * H + 4 * q);
    pxs = ld4(x + qs * H + 4 * q);
    if constexpr (S1E > 0) load_in(perm[kk]);
    else pea = ld4(e + int64_t(kk) * H + 4 * q);
    const int kn = edge_of(wave + 4);
    qd = dst[kn];
    qs = src[kn];
    if constexpr (S1E > 0) qe = perm[kn];
  }
  const int nchunk = (NT + 15) / 16;
  for (int c = 0; c < nchunk; ++c) {
    const int c0 = k0 + c * CE;
    const int c1 = c0 + CE < k1 ? c0 + CE : k1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int T = c * 16 + wave + 4 * i;
      if (T >= NT) break;  // wave-uniform: MFMA needs EXEC all ones
      const int k = k0 + T * 16 + it;
      const bool valid = k < k1;
      const f4 xd = pxd, xs = pxs;  // x_i (target), x_j (source)
      f4 ea;                         // edge attr
      if constexpr (S1E > 0 && F32) {
        float iv[SE];
#pragma unroll
        for (int s = 0; s < SE; ++s) iv[s] = pin[s];
        ea = ff_tile_regs<SE>(wenc, iv);  // k_encode<true>'s MLP on this edge
      } else if constexpr (S1E > 0) {
        const float iv[4] = {pin[0], pin[1], pin[2], pin[3]};
        ea = ff1_16_enc(fenc, iv, lane, use, ebd);  // k_encode<true>'s MLP on this edge (split-f16 block, read
                                               // through the cache)
      } else {
        ea = pea;
      }
      {  // prefetch tile T+4 (clamped), indices of tile T+8 (clamped)
        pxd = ld4(x + qd * H + 4 * q);
        pxs = ld4(x + qs * H + 4 * q);
        if constexpr (S1E > 0) load_in(qe);
        else pea = ld4(e + int64_t(edge_of(T + 4)) * H + 4 * q);
        const int kn = edge_of(T + 8);
        qd = dst[kn];
        qs = src[kn];
        if constexpr (S1E > 0) qe = perm[kn];
      }
      // LayerNorm(48) statistics: 12 values per lane, 4 lanes per edge, packed fp32 pairs
      f2 w[6] = {(f2){xd.x, xd.y}, (f2){xd.z, xd.w}, (f2){xs.x, xs.y},
                 (f2){xs.z, xs.w}, (f2){ea.x, ea.y}, (f2){ea.z, ea.w}};
      const f2 s2 = ((w[0] + w[1]) + (w[2] + w[3])) + (w[4] + w[5]);
      const float mean = quad_sum(s2.x + s2.y) * (1.0f / 48.0f);
      f2 q2 = (f2)(0.f);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        w[j] -= (f2)(mean);
        q2 = __builtin_elementwise_fma(w[j], w[j], q2);
      }
      const float rstd = __builtin_amdgcn_rsqf(quad_sum(q2.x + q2.y) * (1.0f / 48.0f) + 1e-5f);
      float v[12];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        w[j] *= (f2)(rstd);
        v[2 * j] = w[j].x;
        v[2 * j + 1] = w[j].y;
      }
      f4 m, u;
      if constexpr (F32) {
        ff2_48(fmsg, fedge, v, lane, m, u);
        if (edge_res) u += ea;
      } else {
        // m stays 2^s3 times the message (unscaled once per node after the sum: power-of-two
        // scaling commutes with every rounding of the sum, so the same bits); the edge output's
        // unscale is exact, so unscale + residual is one FMA with the same result
        ff2_48(fmsg, fedge, v, lane, m, u, us);
        if (edge_res) u = __builtin_elementwise_fma(u, (f4)(us[5]), ea);
        else u *= us[5];
      }
      if (valid) {
        st4(e + int64_t(k) * H + 4 * q, u);
        st4(msg + (k - c0) * H + 4 * q, m);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = n0 + (wave + 4 * j) * 16 + it;
      if (i < n1) {
        const int kb = ptr[i] > c0 ? ptr[i] : c0;
        const int ke = ptr[i + 1] < c1 ? ptr[i + 1] : c1;
        for (int kq = kb; kq < ke; ++kq) agg[j] += ld4(msg + (kq - c0) * H + 4 * q);
      }
    }
    __syncthreads();
  }
  // update(): node_mlp(aggr) with LayerNorm(16) pre-norm; residual (basic_layers.py:203-206, 224-225)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = n0 + (wave + 4 * j) * 16 + it;
    const f4 a = F32 ? agg[j] : agg[j] * us[2];  // split-f16: the messages were summed 2^s3-scaled
    const float mean = quad_sum((a.x + a.y) + (a.z + a.w)) * (1.0f / 16.0f);
    float v[4] = {a.x - mean, a.y - mean, a.z - mean, a.w - mean};
    const float sq = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
    const float rstd = __builtin_amdgcn_rsqf(quad_sum(sq) * (1.0f / 16.0f) + 1e-5f);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= rstd;
    f4 o;
    if constexpr (F32) o = ff_tile<4>(fnode, v, lane);
    else o = ff1_16(fnode, v, lane, usn);
    if (i < n1) {
      if (node_res) o += ld4(x + int64_t(i) * H + 4 * q);
      st4(xout + int64_t(i) * H + 4 * q, o);
    }
  }
}

static int egrid(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  return int(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

static int tgrid(int64_t items) {  // 64 items (4 waves x 16) per workgroup
  int64_t g = (items + 63) / 64;
  return int(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace lspcg

using namespace lspcg;

// ---------------------------------------------------------------------------
// Host-side fragment preparation
// ---------------------------------------------------------------------------
namespace {

struct FF {  // views into the packed (reference-layout) blob
  const float* W1;
  const float* b1;
  const float* W2;
  const float* b2;
  const float* W3;
  const float* b3;
  int in, out;
};

FF ff_at(const float* w, int in, int out) {
  FF f;
  f.in = in;
  f.out = out;
  f.W1 = w;
  f.b1 = w + H * in;
  f.W2 = f.b1 + H;
  f.b2 = f.W2 + H * H;
  f.W3 = f.b2 + H;
  f.b3 = f.W3 + out * H;
  return f;
}

// Append the fragment block of `f` (LayerNorm affine gamma/beta folded into layer 1 when given).
// feat(s, q) = input feature in K slot q of step s (-1 = zero).
template <class Feat>
void emit_frag(std::vector<float>& o, const FF& f, int s1, Feat feat, const float* gamma, const float* beta) {
  std::vector<double> W1(H * f.in), b1(H);
  for (int i = 0; i < H; ++i) {
    double bb = f.b1[i];
    for (int k = 0; k < f.in; ++k) {
      const double w = f.W1[i * f.in + k];
      W1[i * f.in + k] = gamma ? w * gamma[k] : w;
      if (beta) bb += w * beta[k];
    }
    b1[i] = bb;
  }
  for (int s = 0; s < s1; ++s)
    for (int l = 0; l < 64; ++l) {
      const int fi = feat(s, l >> 4);
      o.push_back(fi >= 0 && fi < f.in ? float(W1[(l & 15) * f.in + fi]) : 0.f);
    }
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) o.push_back(float(b1[4 * (l >> 4) + r]));
  for (int s = 0; s < 4; ++s)
    for (int l = 0; l < 64; ++l) o.push_back(f.W2[(l & 15) * H + 4 * (l >> 4) + s]);
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) o.push_back(f.b2[4 * (l >> 4) + r]);
  for (int s = 0; s < 4; ++s)
    for (int l = 0; l < 64; ++l) {
      const int i = l & 15;
      o.push_back(i < f.out ? f.W3[i * H + 4 * (l >> 4) + s] : 0.f);
    }
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * (l >> 4) + r;
      o.push_back(i < f.out ? f.b3[i] : 0.f);
    }
}

auto feat48 = [](int s, int q) { return (s >> 2) * 16 + 4 * q + (s & 3); };

// The split-f16 block of a FeedForward(48 -> 16 -> 16 -> out) (ff2_48; layout at kH48): weights
// scaled by 2^s per matrix (max |W| 2^s in [2^10, 2^11)), split into RNE f16 pairs.
void emit_frag_h_any(std::vector<float>& o, const FF& f, const float* gamma, const float* beta, bool in48) {
  std::vector<float> W1(H * f.in), b1(H);
  for (int i = 0; i < H; ++i) {
    double bb = f.b1[i];
    for (int k = 0; k < f.in; ++k) {
      const double w = f.W1[i * f.in + k];
      W1[i * f.in + k] = float(gamma ? w * gamma[k] : w);
      if (beta) bb += w * beta[k];
    }
    b1[i] = float(bb);
  }
  auto scale_exp = [](auto get, int rows, int cols) {
    double mx = 0;
    for (int i = 0; i < rows; ++i)
      for (int k = 0; k < cols; ++k) mx = std::max(mx, std::fabs(double(get(i, k))));
    if (mx == 0) return 0;
    int e;
    std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
    return 11 - e;       // max |W| 2^s in [2^10, 2^11)
  };
  auto w1 = [&](int i, int k) { return k < f.in ? W1[i * f.in + k] : 0.f; };  // 16-slot blocks pad fin < 16
  auto w2 = [&](int i, int k) { return f.W2[i * H + k]; };
  auto w3 = [&](int i, int k) { return i < f.out ? f.W3[i * H + k] : 0.f; };
  const int s1 = scale_exp(w1, H, f.in), s2 = scale_exp(w2, H, H), s3 = scale_exp(w3, H, H);
  auto push_pairs = [&](auto get, int s, int per_lane, auto kidx, bool lo) {  // per lane: per_lane halves
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < per_lane; j += 2) {
        unsigned u = 0;
        for (int t = 0; t < 2; ++t) {
          const int k = kidx(l >> 4, j + t);
          const float x = k >= 0 ? std::ldexp(get(l & 15, k), s) : 0.f;
          const _Float16 h = static_cast<_Float16>(x);
          const _Float16 v = lo ? static_cast<_Float16>(x - static_cast<float>(h)) : h;
          u |= unsigned(__builtin_bit_cast(unsigned short, v)) << (16 * t);
        }
        o.push_back(__builtin_bit_cast(float, u));
      }
  };
  auto push_bias = [&](auto get, int s) {
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) o.push_back(std::ldexp(get(4 * (l >> 4) + r), s));
  };
  auto kh = [](int q, int j) { return 4 * q + j; };  // 16-wide inputs / hidden layers
  if (in48) {  // three K blocks of 16: block i, slot (q, j) = feature 16 i + 4 q + j = feat48(4 i + j, q)
    for (bool lo : {false, true})
      for (int i = 0; i < 3; ++i) push_pairs(w1, s1, 4, [i](int q, int j) { return feat48(4 * i + j, q); }, lo);
  } else {  // 16 inputs: one 16x16x16 product, K slot (q, j) = feature 4q + j
    push_pairs(w1, s1, 4, kh, false);
    push_pairs(w1, s1, 4, kh, true);
  }
  push_bias([&](int i) { return b1[i]; }, s1);
  push_pairs(w2, s2, 4, kh, false);
  push_pairs(w2, s2, 4, kh, true);
  push_bias([&](int i) { return f.b2[i]; }, s2);
  push_pairs(w3, s3, 4, kh, false);
  push_pairs(w3, s3, 4, kh, true);
  push_bias([&](int i) { return i < f.out ? f.b3[i] : 0.f; }, s3);
  for (int s : {s1, s2, s3}) o.push_back(std::ldexp(1.0f, -s));
  o.push_back(0.f);
  if (!in48) {  // magnitude bounds for ff1_16_enc: max row sum of |W|, max |bias| + GELU's 0.17
    auto rowsum = [](auto get, int rows, int cols) {
      double mx = 0;
      for (int i = 0; i < rows; ++i) {
        double r = 0;
        for (int k = 0; k < cols; ++k) r += std::fabs(double(get(i, k)));
        mx = std::max(mx, r);
      }
      return float(mx);
    };
    auto absmax = [](auto get, int n) {
      double mx = 0;
      for (int i = 0; i < n; ++i) mx = std::max(mx, std::fabs(double(get(i))));
      return float(mx + 0.17);
    };
    const float B1 = rowsum(w1, H, f.in), c1 = absmax([&](int i) { return b1[i]; }, H);
    const float B2 = rowsum(w2, H, H), c2 = absmax([&](int i) { return f.b2[i]; }, H);
    o.push_back(B1);
    o.push_back(c1);
    o.push_back(B2);
    o.push_back(c2);
    // the largest edge maximum m with max(B1 m + c1, B2 (B1 m + c1) + c2) < 2^14 (no hidden scale);
    // half the device threshold, so the float rounding of the bounds cannot matter
    const double lim = 16384.0, h1 = std::min(lim, (lim - c2) / std::max(double(B2), 1e-30));
    const double ms = (h1 - c1) / std::max(double(B1), 1e-30);
    o.push_back(float(std::max(0.0, ms)));
    o.push_back(0.f);
    o.push_back(0.f);
    o.push_back(0.f);
  }
}
// Largest |hidden activation| a LayerNorm-fed FeedForward can produce: LayerNorm outputs are at most
// sqrt(n - 1) in magnitude (gamma / beta folded into layer 1), |GELU(z)| <= max(|z|, 0.17), so
// |h1| <= ||W1'||_inf sqrt(n - 1) + max |b1'| + 0.17 and |h2| <= ||W2||_inf |h1| + max |b2| + 0.17.
// The split-f16 products need it below 2^15 (f16 holds 65504): gnn_create runs the fp32-MFMA
// kernels for weights past it.
double ln_ff_hidden_bound(const FF& f, const float* gamma, const float* beta) {
  double h1 = 0, h2 = 0, b2 = 0;
  for (int i = 0; i < H; ++i) {
    double r = 0, bb = f.b1[i];
    for (int k = 0; k < f.in; ++k) {
      r += std::fabs(double(f.W1[i * f.in + k]) * gamma[k]);
      bb += double(f.W1[i * f.in + k]) * beta[k];
    }
    h1 = std::max(h1, r * std::sqrt(double(f.in - 1)) + std::fabs(bb) + 0.17);
  }
  for (int i = 0; i < H; ++i) {
    double r = 0;
    for (int k = 0; k < H; ++k) r += std::fabs(double(f.W2[i * H + k]));
    h2 = std::max(h2, r);
    b2 = std::max(b2, std::fabs(double(f.b2[i])));
  }
  return std::max(h1, h2 * h1 + b2 + 0.17);
}
// The split-f16 GEMMs carry each layer's result scaled by 2^s (s: emit_frag_h_any's exponent, max |W|
// 2^s in [2^10, 2^11)); the last layer's messages are summed over a node's edges while still scaled.
// A matrix of tiny weights beside O(1) biases (2^s large, the bias scaled alike) could push those
// scaled values past fp32's range, which the per-message unscale never reached.  Returns
// the largest scaled magnitude, 2^s x (|W| row bound x input bound + max |bias|), over the three
// layers; gnn_create runs the fp32-MFMA kernels (no scaling) when it exceeds 2^96, which leaves 2^32
// for a node's message sum.  (Seeded / trained weights: ~2^20.)
double ln_ff_scaled_bound(const FF& f, const float* gamma, const float* beta) {
  auto sexp = [](double mx) {
    if (mx == 0) return 0;
    int e;
    std::frexp(mx, &e);
    return 11 - e;
  };
  double w1 = 0, w2 = 0, w3 = 0, r1 = 0, r2 = 0, r3 = 0, b1 = 0, b2 = 0, b3 = 0;
  for (int i = 0; i < H; ++i) {
    double r = 0, bb = f.b1[i];
    for (int k = 0; k < f.in; ++k) {
      const double w = double(f.W1[i * f.in + k]) * gamma[k];
      w1 = std::max(w1, std::fabs(w));
      r += std::fabs(w);
      bb += double(f.W1[i * f.in + k]) * beta[k];
    }
    r1 = std::max(r1, r);
    b1 = std::max(b1, std::fabs(bb));
    double q2 = 0, q3 = 0;
    for (int k = 0; k < H; ++k) {
      w2 = std::max(w2, std::fabs(double(f.W2[i * H + k])));
      q2 += std::fabs(double(f.W2[i * H + k]));
      if (i < f.out) {
        w3 = std::max(w3, std::fabs(double(f.W3[i * H + k])));
        q3 += std::fabs(double(f.W3[i * H + k]));
      }
    }
    r2 = std::max(r2, q2);
    r3 = std::max(r3, q3);
    b2 = std::max(b2, std::fabs(double(f.b2[i])));
    if (i < f.out) b3 = std::max(b3, std::fabs(double(f.b3[i])));
  }
  const double x1 = std::sqrt(double(f.in - 1));            // LayerNorm output bound
  const double h1 = r1 * x1 + b1 + 0.17, h2 = r2 * h1 + b2 + 0.17;  // GELU outputs
  return std::max({std::ldexp(r1 * x1 + b1, sexp(w1)), std::ldexp(r2 * h1 + b2, sexp(w2)),
                   std::ldexp(r3 * h2 + b3, sexp(w3))});
}
void emit_frag_h(std::vector<float>& o, const FF& f, const float* gamma, const float* beta) {
  emit_frag_h_any(o, f, gamma, beta, true);  // kH48 dwords
}
void emit_frag_h16(std::vector<float>& o, const FF& f, const float* gamma, const float* beta) {
  emit_frag_h_any(o, f, gamma, beta, false);  // kH16 dwords
}
auto feat16 = [](int s, int q) { return 4 * q + s; };
auto featenc = [](int s, int q) { return 4 * s + q; };

}  // namespace

struct lspcg_gnn {
  lspcg_ctx* ctx = nullptr;
  lspcg_gnn_desc d{};
  float* frag = nullptr;  // device fragment blob
  int64_t o_node_enc = 0, o_edge_enc = 0, o_dec = 0;
  int64_t o_edge_enc_h = 0;  // split-f16 block of the edge encoder (the first layer's fused copy)
  bool f32 = false;          // fp32-MFMA kernels (weights past the split-f16 range, or LSPCG_GNN_F32=1)
  double hidden_bound = 0;   // largest ln_ff_hidden_bound over the layers (what chose f32)
  std::vector<int64_t> o_layer;  // per layer: [msg | edge | node] fragment block
  // workspace
  int64_t capN = -1, capE = -1;
  float *xa = nullptr, *xb = nullptr, *ecsc = nullptr;
  int32_t *ptr = nullptr, *cnt = nullptr, *perm = nullptr, *inv = nullptr, *src = nullptr, *dst = nullptr;
  int* flag = nullptr;
  void* scan_tmp = nullptr;
  size_t scan_bytes = 0;
  // the CSC of the last graph (lspcg_gnn_set_graph): reused while forward gets the same
  // (edge_index pointer, N, E); gflag != 0: the generic (unsorted / asymmetric) path built it
  const int64_t* gei = nullptr;
  int64_t gN = -1, gE = -1;
  int gflag = 0;
};

static int64_t gnn_weight_count(const lspcg_gnn_desc& d) {
  int64_t n = ff_size(d.node_in, H) + ff_size(d.edge_in, H);
  n += int64_t(d.num_mp_layers) * ((2 * H + ff_size(H, H)) + 2 * (6 * H + ff_size(3 * H, H)));
  n += ff_size(3 * H, d.edge_out);
  return n;
}

static void gnn_free_ws(lspcg_gnn* g) {
  for (void* p : {(void*)g->xa, (void*)g->xb, (void*)g->ecsc, (void*)g->ptr, (void*)g->cnt, (void*)g->perm, (void*)g->inv,
                  (void*)g->src, (void*)g->dst, g->scan_tmp})
    (void)hipFree(p);
  g->xa = g->xb = g->ecsc = nullptr;
  g->ptr = g->cnt = g->perm = g->inv = g->src = g->dst = nullptr;
  (void)hipFree(g->flag);
  g->flag = nullptr;
  g->scan_tmp = nullptr;
  g->capN = g->capE = -1;
  g->gei = nullptr;  // the cached CSC lived in the freed workspace
  g->gN = g->gE = -1;
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
  LSPCG_HIP(hipMalloc(&g->flag, sizeof(int)));
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
  std::vector<float> w(need);
  LSPCG_HIP(hipMemcpy(w.data(), weights, sizeof(float) * need, hipMemcpyDefault));  // host or device source
  // precision: the split-f16 GEMMs hold hidden activations below 2^15; weights whose LayerNorm-fed
  // MLPs could exceed that run the exact fp32-MFMA kernels instead (same results to ~1e-7, 1.2x slower)
  {
    int64_t ob = ff_size(d.node_in, H) + ff_size(d.edge_in, H);
    double scaled = 0;  // ln_ff_scaled_bound over the layers
    for (int l = 0; l < d.num_mp_layers; ++l) {
      const float* node = w.data() + ob;
      const float* edge = node + 2 * H + ff_size(H, H);
      const float* msgp = edge + 6 * H + ff_size(3 * H, H);
      ob += 2 * H + ff_size(H, H) + 2 * (6 * H + ff_size(3 * H, H));
      g->hidden_bound = std::max({g->hidden_bound, ln_ff_hidden_bound(ff_at(msgp + 6 * H, 3 * H, H), msgp, msgp + 3 * H),
                                  ln_ff_hidden_bound(ff_at(edge + 6 * H, 3 * H, H), edge, edge + 3 * H),
                                  ln_ff_hidden_bound(ff_at(node + 2 * H, H, H), node, node + H)});
      scaled = std::max({scaled, ln_ff_scaled_bound(ff_at(msgp + 6 * H, 3 * H, H), msgp, msgp + 3 * H),
                         ln_ff_scaled_bound(ff_at(edge + 6 * H, 3 * H, H), edge, edge + 3 * H),
                         ln_ff_scaled_bound(ff_at(node + 2 * H, H, H), node, node + H)});
    }
    const char* ev = std::getenv("LSPCG_GNN_F32");
    g->f32 = !(g->hidden_bound < 32768.0) || !(scaled <= std::ldexp(1.0, 96)) || (ev && ev[0] == '1');
  }
  const bool f32 = g->f32;
  std::vector<float> fr;
  int64_t o = 0;
  g->o_node_enc = int64_t(fr.size());
  emit_frag(fr, ff_at(w.data() + o, d.node_in, H), (d.node_in + 3) / 4, featenc, nullptr, nullptr);
  o += ff_size(d.node_in, H);
  g->o_edge_enc = int64_t(fr.size());
  emit_frag(fr, ff_at(w.data() + o, d.edge_in, H), (d.edge_in + 3) / 4, featenc, nullptr, nullptr);
  const float* enc_w = w.data() + o;
  o += ff_size(d.edge_in, H);
  for (int l = 0; l < d.num_mp_layers; ++l) {
    const float* node = w.data() + o;  // [ln_g 16 | ln_b 16 | FF(16->16)]
    o += 2 * H + ff_size(H, H);
    const float* edge = w.data() + o;  // [ln_g 48 | ln_b 48 | FF(48->16)]
    o += 6 * H + ff_size(3 * H, H);
    const float* msgp = w.data() + o;
    o += 6 * H + ff_size(3 * H, H);
    g->o_layer.push_back(int64_t(fr.size()));
    if (f32) {
      emit_frag(fr, ff_at(msgp + 6 * H, 3 * H, H), 12, feat48, msgp, msgp + 3 * H);
      emit_frag(fr, ff_at(edge + 6 * H, 3 * H, H), 12, feat48, edge, edge + 3 * H);
      emit_frag(fr, ff_at(node + 2 * H, H, H), 4, feat16, node, node + H);
    } else {
      emit_frag_h(fr, ff_at(msgp + 6 * H, 3 * H, H), msgp, msgp + 3 * H);
      emit_frag_h(fr, ff_at(edge + 6 * H, 3 * H, H), edge, edge + 3 * H);
      emit_frag_h16(fr, ff_at(node + 2 * H, H, H), node, node + H);
    }
  }
  g->o_dec = int64_t(fr.size());
  if (f32) {
    emit_frag(fr, ff_at(w.data() + o, 3 * H, d.edge_out), 12, feat48, nullptr, nullptr);
  } else {
    emit_frag_h(fr, ff_at(w.data() + o, 3 * H, d.edge_out), nullptr, nullptr);
    g->o_edge_enc_h = int64_t(fr.size());
    if (d.edge_in <= 16) emit_frag_h16(fr, ff_at(enc_w, d.edge_in, H), nullptr, nullptr);
  }
  LSPCG_HIP(hipMalloc(&g->frag, sizeof(float) * fr.size()));
  LSPCG_HIP(hipMemcpy(g->frag, fr.data(), sizeof(float) * fr.size(), hipMemcpyHostToDevice));
  *out = g.release();
  return LSPCG_OK;
}

// CSC of the edges by destination (the structure analysis of one graph; lspcg_gnn_set_graph)
static int gnn_build_csc(lspcg_gnn* g, int64_t N, int64_t E, const int64_t* edge_index) {
  g->gei = nullptr;
  if (int rc = gnn_reserve(g, N, E)) return rc;
  g->gei = nullptr;
  g->gN = g->gE = -1;
  if (E == 0 || N == 0) {
    g->gei = edge_index;
    g->gN = N;
    g->gE = E;
    return LSPCG_OK;
  }
  hipStream_t st = g->ctx->stream;
  LSPCG_HIP(hipMemsetAsync(g->cnt, 0, sizeof(int32_t) * (N + 1), st));
  LSPCG_HIP(hipMemsetAsync(g->flag, 0, sizeof(int), st));
  // unsorted input leaves row starts unwritten (flagged): zeroed, k_csc_sym's searches stay in range
  LSPCG_HIP(hipMemsetAsync(g->ptr, 0, sizeof(int32_t) * (N + 1), st));
  hipLaunchKernelGGL(k_csc_rowstart, dim3(egrid(E + 1)), dim3(kThreads), 0, st, N, E, edge_index, g->ptr,
                     g->flag);
  hipLaunchKernelGGL(k_csc_sym, dim3(egrid(E)), dim3(kThreads), 0, st, E, edge_index, g->ptr, g->perm, g->src, g->dst,
                     g->flag);
  int hflag = 0;
  LSPCG_HIP(hipMemcpyAsync(&hflag, g->flag, sizeof(int), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  if (hflag) {  // generic: count by dst, scan, slot fill, per-node sort by edge id
    LSPCG_HIP(hipMemsetAsync(g->cnt, 0, sizeof(int32_t) * (N + 1), st));
    hipLaunchKernelGGL(k_csc_count, dim3(egrid(E)), dim3(kThreads), 0, st, E, edge_index, g->cnt);
    size_t tb = g->scan_bytes;
    LSPCG_HIP(hipcub::DeviceScan::ExclusiveSum(g->scan_tmp, tb, g->cnt, g->ptr, int(N + 1), st));
    LSPCG_HIP(hipMemsetAsync(g->cnt, 0, sizeof(int32_t) * (N + 1), st));
    hipLaunchKernelGGL(k_csc_fill, dim3(egrid(E)), dim3(kThreads), 0, st, E, edge_index, g->ptr, g->cnt, g->perm);
    hipLaunchKernelGGL(k_csc_sort, dim3(egrid(N)), dim3(kThreads), 0, st, N, edge_index, E, g->ptr, g->perm, g->inv,
                       g->src, g->dst);
  }
  LSPCG_HIP(hipGetLastError());
  g->gei = edge_index;
  g->gN = N;
  g->gE = E;
  g->gflag = hflag;
  return LSPCG_OK;
}

int lspcg_gnn_set_graph(lspcg_gnn* g, int64_t N, int64_t E, const int64_t* edge_index) {
  LSPCG_CHECK(g && (E == 0 || edge_index), LSPCG_ERR_ARG, "gnn_set_graph: NULL argument");
  LSPCG_CHECK(N >= 0 && E >= 0 && N < (int64_t(1) << 31) && E < (int64_t(1) << 31), LSPCG_ERR_ARG,
              "gnn_set_graph: sizes out of range");
  LSPCG_HIP(hipSetDevice(g->ctx->device));
  return gnn_build_csc(g, N, E, edge_index);
}

int lspcg_gnn_forward(lspcg_gnn* g, int64_t N, int64_t E, const float* x, const int64_t* edge_index,
                      const float* edge_attr, float* out) {
  LSPCG_CHECK(g && (N == 0 || x) && (E == 0 || (edge_index && edge_attr && out)), LSPCG_ERR_ARG,
              "gnn_forward: NULL argument");
  LSPCG_CHECK(N >= 0 && E >= 0 && N < (int64_t(1) << 31) && E < (int64_t(1) << 31), LSPCG_ERR_ARG,
              "gnn_forward: sizes out of range");
  LSPCG_HIP(hipSetDevice(g->ctx->device));
  if (!(g->gei == edge_index && g->gN == N && g->gE == E && N <= g->capN && E <= g->capE))
    if (int rc = gnn_build_csc(g, N, E, edge_index)) return rc;
  if (E == 0 || N == 0) return LSPCG_OK;
  hipStream_t st = g->ctx->stream;
  const lspcg_gnn_desc& d = g->d;
  const int hflag = g->gflag;
  const int32_t* inv = hflag ? g->inv : g->perm;  // edge -> CSC slot (the involution is its own inverse)
  // encoders (the edge encoder is fused into the first layer when there is one and edge_in <= 12)
  hipLaunchKernelGGL(k_encode<false>, dim3(tgrid(N)), dim3(256), 0, st, N, d.node_in, g->frag + g->o_node_enc, x,
                     static_cast<const int32_t*>(nullptr), g->xa);
  const int s1e = (d.edge_in + 3) / 4;
  const bool fuse_enc = d.num_mp_layers > 0 && s1e <= 3;
  if (!fuse_enc)
    hipLaunchKernelGGL(k_encode<true>, dim3(tgrid(E)), dim3(256), 0, st, E, d.edge_in, g->frag + g->o_edge_enc,
                       edge_attr, g->perm, g->ecsc);
  // message passing
  float* xc = g->xa;
  float* xn = g->xb;
  const unsigned lg = unsigned((N + 255) / 256);
  // the fused copy reads the split-f16 block (f32: the f32 fragments, held in registers)
  const float* fenc = g->frag + (g->f32 ? g->o_edge_enc : g->o_edge_enc_h);
  for (int l = 0; l < d.num_mp_layers; ++l) {
    const int se = (l == 0 && fuse_enc) ? s1e : 0;
    auto kern = g->f32 ? (se == 1   ? k_mp_layer<true, 1>
                          : se == 2 ? k_mp_layer<true, 2>
                          : se == 3 ? k_mp_layer<true, 3>
                                    : k_mp_layer<true, 0>)
                       : (se == 1   ? k_mp_layer<false, 1>
                          : se == 2 ? k_mp_layer<false, 2>
                          : se == 3 ? k_mp_layer<false, 3>
                                    : k_mp_layer<false, 0>);
    hipLaunchKernelGGL(kern, dim3(lg), dim3(256), 0, st, N, g->frag + g->o_layer[l], d.node_residual, d.edge_residual,
                       g->ptr, g->src, g->dst, xc, g->ecsc, xn, fenc, d.edge_in, edge_attr,
                       static_cast<const int32_t*>(g->perm));
    std::swap(xc, xn);
  }
  // decoder
  const float* fd = g->frag + g->o_dec;
  // endpoints in edge order: the symmetric fast path's int32 dst / src are exactly edge_index's
  // rows (k_csc_sym: slot e's endpoints are (ei[E+e], ei[e])), half the index bytes of the int64 rows
  if (!hflag) {
    auto dec = g->f32 ? (d.edge_out == 1   ? k_edge_dec<true, 1, int32_t>
                         : d.edge_out == 4 ? k_edge_dec<true, 4, int32_t>
                                           : k_edge_dec<true, 9, int32_t>)
                      : (d.edge_out == 1   ? k_edge_dec<false, 1, int32_t>
                         : d.edge_out == 4 ? k_edge_dec<false, 4, int32_t>
                                           : k_edge_dec<false, 9, int32_t>);
    hipLaunchKernelGGL(dec, dim3(tgrid(E)), dim3(256), 0, st, E, fd, static_cast<const int32_t*>(g->dst),
                       static_cast<const int32_t*>(g->src), inv, g->ecsc, xc, out);
  } else {
    auto dec = g->f32 ? (d.edge_out == 1   ? k_edge_dec<true, 1, int64_t>
                         : d.edge_out == 4 ? k_edge_dec<true, 4, int64_t>
                                           : k_edge_dec<true, 9, int64_t>)
                      : (d.edge_out == 1   ? k_edge_dec<false, 1, int64_t>
                         : d.edge_out == 4 ? k_edge_dec<false, 4, int64_t>
                                           : k_edge_dec<false, 9, int64_t>);
    hipLaunchKernelGGL(dec, dim3(tgrid(E)), dim3(256), 0, st, E, fd, edge_index, edge_index + E, inv, g->ecsc, xc,
                       out);
  }
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int lspcg_gnn_precision(const lspcg_gnn* g, int* f32, double* hidden_bound) {
  LSPCG_CHECK(g && f32, LSPCG_ERR_ARG, "gnn_precision: NULL argument");
  *f32 = g->f32 ? 1 : 0;
  if (hidden_bound) *hidden_bound = g->hidden_bound;
  return LSPCG_OK;
}

int lspcg_gnn_destroy(lspcg_gnn* g) {
  if (!g) return LSPCG_OK;
  (void)hipSetDevice(g->ctx->device);
  gnn_free_ws(g);
  (void)hipFree(g->frag);
  delete g;
  return LSPCG_OK;
}

}  // extern "C"
