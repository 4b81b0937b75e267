// Does an MFMA execute beside independent VALU work on gfx950?  Measurement only.
// (1) one wave per SIMD: a loop of 4 independent MFMA chains with K independent f32 FMAs after each
//     MFMA (inline asm, in that order); cycles per MFMA as K grows say whether the FMAs hide under the
//     MFMA (co-execution: flat until the issue slots run out) or add to it (serialised).
// (2) two waves per SIMD (hardware wave slot parity): one runs MFMAs only, its partner FMAs only;
//     each reports its own cycles -- beside the partner vs alone.
// For v_mfma_f32_16x16x4_f32 (the GNN's) and v_mfma_f32_16x16x32_f16.
//   hipcc -O3 --offload-arch=gfx950 tools/coexec_probe.hip -o exp/coexec_probe && exp/coexec_probe
#include <hip/hip_runtime.h>

#include <cstdio>

using f4 = float __attribute__((ext_vector_type(4)));
using h8 = _Float16 __attribute__((ext_vector_type(8)));

template <int MODE>
__device__ __forceinline__ void mfma(f4& acc, float a, float b, h8 ha, h8 hb) {
  if constexpr (MODE == 0) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(ha), "v"(hb));
}
__device__ __forceinline__ void fma1(float& x, float m, float c) {
  asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(c));
}

// MODE 0 f32 MFMA, 1 f16 MFMA, 2 none; K FMAs after every MFMA (8 rotating registers)
template <int MODE, int K>
__global__ void __launch_bounds__(64) k_single(int iters, float seed, float* out, long long* cyc) {
  const int lane = threadIdx.x;
  f4 acc[4] = {};
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = seed + lane + k;
  const float a = seed * 0.5f + lane, b = seed + 1.0f, m = 0.999f + seed * 1e-9f, c = 0.001f * seed;
  h8 ha, hb;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ha[i] = _Float16(a + i);
    hb[i] = _Float16(b - i);
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (MODE < 2) mfma<MODE>(acc[u], a, b, ha, hb);
#pragma unroll
      for (int k = 0; k < K; ++k) fma1(v[k & 7], m, c);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) s += acc[u].x + acc[u].y + acc[u].z + acc[u].w;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += v[k];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// two single-wave workgroups per SIMD: the wave in an even hardware slot runs MFMAs only (4 chains),
// the odd one FMAs only (K per step, same step count); role < 0: every wave runs its slot's role,
// role 0 / 1: every wave runs MFMA / FMA (the "alone" baselines at the same occupancy)
template <int MODE, int K>
__global__ void __launch_bounds__(64) k_pair(int iters, int role, float seed, float* out, long long* cyc,
                                             int* kind) {
  const int lane = threadIdx.x;
  const unsigned hwid = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4);  // HW_ID[3:0] = wave slot
  const int r = role >= 0 ? role : int(hwid & 1u);
  f4 acc[4] = {};
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = seed + lane + k;
  const float a = seed * 0.5f + lane, b = seed + 1.0f, m = 0.999f + seed * 1e-9f, c = 0.001f * seed;
  h8 ha, hb;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ha[i] = _Float16(a + i);
    hb[i] = _Float16(b - i);
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (r == 0) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int u = 0; u < 4; ++u) mfma<MODE>(acc[u], a, b, ha, hb);
  } else {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) fma1(v[k & 7], m, c);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) s += acc[u].x + acc[u].y + acc[u].z + acc[u].w;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += v[k];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) {
    cyc[blockIdx.x] = t1 - t0;
    kind[blockIdx.x] = r;
  }
}

static long long hcyc[8192];
static int hkind[8192];

template <int MODE, int K>
static void single(const char* name, float* out, long long* cyc, int nb, int iters) {
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_single<MODE, K>), dim3(nb), dim3(64), 0, 0, iters, 1.0f, out, cyc);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(hcyc, cyc, sizeof(long long) * nb, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < nb; ++i) s += double(hcyc[i]);
  s /= nb;
  std::printf("{\"test\": \"single\", \"mfma\": \"%s\", \"fma_per_mfma\": %d, \"cycles_per_step\": %.2f}\n", name, K,
              s / iters / 4.0);
}

template <int MODE, int K>
static void pair(const char* name, float* out, long long* cyc, int* kind, int nb, int iters) {
  const char* rn[3] = {"mfma_alone", "fma_alone", "mixed"};
  for (int role : {0, 1, -1}) {
    for (int rep = 0; rep < 2; ++rep)
      hipLaunchKernelGGL((k_pair<MODE, K>), dim3(nb), dim3(64), 0, 0, iters, role, 1.0f, out, cyc, kind);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(hcyc, cyc, sizeof(long long) * nb, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hkind, kind, sizeof(int) * nb, hipMemcpyDeviceToHost);
    double s[2] = {0, 0};
    int c[2] = {0, 0};
    for (int i = 0; i < nb; ++i) {
      s[hkind[i]] += double(hcyc[i]);
      ++c[hkind[i]];
    }
    std::printf("{\"test\": \"pair\", \"mfma\": \"%s\", \"fma_per_step\": %d, \"run\": \"%s\", "
                "\"mfma_wave_cycles_per_step\": %.2f, \"fma_wave_cycles_per_step\": %.2f, \"waves\": [%d, %d]}\n",
                name, K, rn[role < 0 ? 2 : role], c[0] ? s[0] / c[0] / iters / 4.0 : -1.0,
                c[1] ? s[1] / c[1] / iters / 4.0 : -1.0, c[0], c[1]);
  }
}

int main() {
  const int iters = 4096;
  float* out;
  long long* cyc;
  int* kind;
  (void)hipMalloc(&out, sizeof(float) * 8192 * 64);
  (void)hipMalloc(&cyc, sizeof(long long) * 8192);
  (void)hipMalloc(&kind, sizeof(int) * 8192);
  const int nb1 = 1024;  // one single-wave workgroup per SIMD
  single<0, 0>("f32_16x16x4", out, cyc, nb1, iters);
  single<0, 2>("f32_16x16x4", out, cyc, nb1, iters);
  single<0, 4>("f32_16x16x4", out, cyc, nb1, iters);
  single<0, 8>("f32_16x16x4", out, cyc, nb1, iters);
  single<0, 16>("f32_16x16x4", out, cyc, nb1, iters);
  single<1, 0>("f16_16x16x32", out, cyc, nb1, iters);
  single<1, 2>("f16_16x16x32", out, cyc, nb1, iters);
  single<1, 4>("f16_16x16x32", out, cyc, nb1, iters);
  single<1, 8>("f16_16x16x32", out, cyc, nb1, iters);
  single<1, 16>("f16_16x16x32", out, cyc, nb1, iters);
  single<2, 2>("none", out, cyc, nb1, iters);
  single<2, 4>("none", out, cyc, nb1, iters);
  single<2, 8>("none", out, cyc, nb1, iters);
  single<2, 16>("none", out, cyc, nb1, iters);
  const int nb2 = 2048;  // two single-wave workgroups per SIMD
  pair<0, 8>("f32_16x16x4", out, cyc, kind, nb2, iters);
  pair<0, 16>("f32_16x16x4", out, cyc, kind, nb2, iters);
  pair<1, 4>("f16_16x16x32", out, cyc, kind, nb2, iters);
  pair<1, 8>("f16_16x16x32", out, cyc, kind, nb2, iters);
  (void)hipFree(out);
  (void)hipFree(cyc);
  (void)hipFree(kind);
  return 0;
}
