// Checks the pieces of the GNN's split-f16 MLPs (lspcg_gnn.hip, ff2_48) on the GPU against the host:
// (1) split2: hi + lo reproduces x to ~2^-22; (2) the operand layouts of v_mfma_f32_16x16x32_f16 and
// v_mfma_f32_16x16x16f16 (A[m][k = 8q + j] / B[k][n] per lane l = (n | m) + 16 q, D[4q + r][n]).
// Measurement / debugging only.  hipcc -O3 --offload-arch=gfx950 tools/f16split_probe.hip -o exp/f16split_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

using f4 = float __attribute__((ext_vector_type(4)));
using h4 = _Float16 __attribute__((ext_vector_type(4)));
using h8 = _Float16 __attribute__((ext_vector_type(8)));

template <int V>
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
  using hf2 = _Float16 __attribute__((ext_vector_type(2)));
  using fl2 = float __attribute__((ext_vector_type(2)));
  if constexpr (V == 0) {  // plain conversions
    const hf2 h = __builtin_convertvector((fl2){a, b}, hf2);
    const fl2 r = (fl2){a, b} - __builtin_convertvector(h, fl2);
    hi = __builtin_bit_cast(unsigned, h);
    lo = __builtin_bit_cast(unsigned, __builtin_convertvector(r, hf2));
  } else if constexpr (V == 1) {  // mixlo / mixhi, constant 1.0
    unsigned h, l;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(a), "v"(b));
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(h), "v"(a));
    asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(h), "v"(b));
    hi = h;
    lo = l;
  } else if constexpr (V == 2) {  // v_fma_mix_f32 residuals, then one pack
    unsigned h;
    float ra, rb;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(a), "v"(b));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(ra) : "v"(h), "v"(a));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(rb) : "v"(h), "v"(b));
    hi = h;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(lo) : "v"(ra), "v"(rb));
  } else {  // mixlo / mixhi with the 1.0 in a VGPR
    unsigned h, l;
    const float one = 1.0f;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h) : "v"(a), "v"(b));
    asm("v_fma_mixlo_f16 %0, -%1, %3, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(h), "v"(a), "v"(one));
    asm("v_fma_mixhi_f16 %0, -%1, %3, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(h), "v"(b), "v"(one));
    hi = h;
    lo = l;
  }
}

template <int V>
__global__ void k_split(const float* x, float* rec, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned h, l;
  split2<V>(x[2 * i], x[2 * i + 1], h, l);
  const auto hh = __builtin_bit_cast(_Float16 __attribute__((ext_vector_type(2))), h);
  const auto ll = __builtin_bit_cast(_Float16 __attribute__((ext_vector_type(2))), l);
  rec[2 * i] = float(hh.x) + float(ll.x);
  rec[2 * i + 1] = float(hh.y) + float(ll.y);
}

// A (16 x 48) row-major, B (48 x 16) row-major (k, n) -> D (16 x 16) with a 16x16x32 over k < 32 and a
// 16x16x16 over k = 32..47, operands in the assumed lane layouts
__global__ void k_mfma(const float* A, const float* B, float* D) {
  const int l = threadIdx.x, q = l >> 4, r16 = l & 15;
  h8 a8, b8;
  h4 a4, b4;
  for (int j = 0; j < 8; ++j) {
    a8[j] = _Float16(A[r16 * 48 + 8 * q + j]);
    b8[j] = _Float16(B[(8 * q + j) * 16 + r16]);
  }
  for (int j = 0; j < 4; ++j) {
    a4[j] = _Float16(A[r16 * 48 + 32 + 4 * q + j]);
    b4[j] = _Float16(B[(32 + 4 * q + j) * 16 + r16]);
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * q + r) * 16 + r16] = acc[r];
}

int main() {
  const int n = 1 << 16;
  float *x, *rec;
  (void)hipMallocManaged(&x, sizeof(float) * n);
  (void)hipMallocManaged(&rec, sizeof(float) * n);
  srand(1);
  for (int i = 0; i < n; ++i) x[i] = (float(rand()) / float(RAND_MAX) - 0.5f) * std::ldexp(1.0f, (i % 20) - 12);
  auto check = [&](int v) {
    double worst = 0, w_lo = 0, w_hi = 0;
    for (int i = 0; i < n; ++i) {
      if (x[i] == 0) continue;
      const double e = std::fabs(double(rec[i]) - x[i]) / std::fabs(double(x[i]));
      worst = std::fmax(worst, e);
      if (i % 2 == 0) w_lo = std::fmax(w_lo, e);
      else w_hi = std::fmax(w_hi, e);
    }
    std::printf("{\"split_variant\": %d, \"max_rel_err\": %.3e, \"even\": %.3e, \"odd\": %.3e}\n", v, worst, w_lo, w_hi);
  };
  hipLaunchKernelGGL(k_split<0>, dim3(n / 512), dim3(256), 0, 0, x, rec, n);
  (void)hipDeviceSynchronize();
  check(0);
  hipLaunchKernelGGL(k_split<1>, dim3(n / 512), dim3(256), 0, 0, x, rec, n);
  (void)hipDeviceSynchronize();
  check(1);
  hipLaunchKernelGGL(k_split<2>, dim3(n / 512), dim3(256), 0, 0, x, rec, n);
  (void)hipDeviceSynchronize();
  check(2);
  hipLaunchKernelGGL(k_split<3>, dim3(n / 512), dim3(256), 0, 0, x, rec, n);
  (void)hipDeviceSynchronize();
  check(3);
  float *A, *B, *D;
  (void)hipMallocManaged(&A, sizeof(float) * 16 * 48);
  (void)hipMallocManaged(&B, sizeof(float) * 48 * 16);
  (void)hipMallocManaged(&D, sizeof(float) * 16 * 16);
  for (int i = 0; i < 16 * 48; ++i) A[i] = float((i * 7) % 13 - 6);
  for (int i = 0; i < 48 * 16; ++i) B[i] = float((i * 5) % 11 - 5);
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, A, B, D);
  (void)hipDeviceSynchronize();
  double derr = 0;
  for (int m = 0; m < 16; ++m)
    for (int c = 0; c < 16; ++c) {
      double s = 0;
      for (int k = 0; k < 48; ++k) s += double(A[m * 48 + k]) * B[k * 16 + c];
      derr = std::fmax(derr, std::fabs(s - D[m * 16 + c]));
    }
  std::printf("{\"mfma_layout_max_abs_err\": %.3e}\n", derr);
  return 0;
}
