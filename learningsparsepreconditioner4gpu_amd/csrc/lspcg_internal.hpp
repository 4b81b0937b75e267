// Internal declarations shared by the lspcg HIP translation units (gfx950 / CDNA4).
//
// Numerics contract (DESIGN.md "Parity"): every translation unit is compiled with
// -ffp-contract=off so that elementwise updates and the sequential row sums of the
// SpMV round exactly like scipy's csr_matvec / numpy ufuncs (product rounded, then
// added).  Dot products use a compensated (Dot2, Ogita-Rump-Oishi) fp64 accumulation
// reduced in a fixed order, i.e. they are deterministic and almost always equal to
// the correctly rounded dot.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>

#include "../../include/lspcg.h"

namespace lspcg {

// ---------------------------------------------------------------------------
// Error handling
// ---------------------------------------------------------------------------
void set_error(const std::string& msg);

#define LSPCG_HIP(call)                                                                    \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess) {                                                                \
      ::lspcg::set_error(std::string(#call) + " failed: " + hipGetErrorString(_e) + " at " \
                         + __FILE__ + ":" + std::to_string(__LINE__));                     \
      return LSPCG_ERR_HIP;                                                                \
    }                                                                                      \
  } while (0)

#define LSPCG_CHECK(cond, code, msg)   \
  do {                                 \
    if (!(cond)) {                     \
      ::lspcg::set_error(msg);         \
      return (code);                   \
    }                                  \
  } while (0)

// ---------------------------------------------------------------------------
// Submission lock.  Independent solves may run on several host threads at once
// (linalg.solve_many); each solver owns its stream, but with GPU_MAX_HW_QUEUES = 4 the
// streams share hardware queues.  Every solve enqueues (launches, graph captures and
// launches, async copies, event records) under this one process-wide lock and releases it
// around each host wait, so no two threads of this library write packets into a queue at
// the same time; the GPU still runs the solves concurrently.  Round 4 found a SIGSEGV in
// the rocprofv3 kernel-trace packet interceptor (rocprofiler-sdk reading past the end of
// the HSA intercept queue's ring, called from hipGraphLaunch) that fired only while four
// threads submitted concurrently ("Concurrent solves").
// ---------------------------------------------------------------------------
std::mutex& submit_mutex();

// ---------------------------------------------------------------------------
// Launch geometry
// ---------------------------------------------------------------------------
// One-shot kernel timing for the standalone SpMV measurement (spmv_timed_impl): while set, the next
// SpMV launch of this host thread goes through hipExtLaunchKernelGGL with these events, which the
// runtime stamps at that kernel's own start and end -- the duration rocprofv3's kernel trace
// reports, without the in-stream kernel boundaries an event pair around the launch would add.
struct KernelTimer {
  hipEvent_t start = nullptr, stop = nullptr;
};
inline KernelTimer*& kernel_timer() {
  thread_local KernelTimer* t = nullptr;
  return t;
}
#define LSPCG_LAUNCH_SPMV(kernel, grid, block, shmem, stream, ...)                                      \
  do {                                                                                                   \
    if (::lspcg::KernelTimer* kt_ = ::lspcg::kernel_timer()) {                                           \
      ::lspcg::kernel_timer() = nullptr;                                                                 \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, kt_->start, kt_->stop, 0, __VA_ARGS__);  \
    } else {                                                                                             \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                               \
    }                                                                                                    \
  } while (0)

constexpr int kThreads = 256;       // 4 wave64 per workgroup
constexpr int kElemBlocksMax = 2048;  // grid cap for streaming elementwise kernels
// grid_reduce_dd ticket buffer: [top | group 0 | group 1 | ...], one 128-B line each
constexpr int kTicketGroup = 32;
constexpr int kTicketStride = 32;
constexpr int kReduceBlocksMax = 8192;  // largest grid of a reducing launch (ticket buffer bound)
constexpr int kTicketWords = kTicketStride * (1 + kReduceBlocksMax / kTicketGroup);
constexpr int kEntryPad = 16;       // zeroed padding entries after colind / vals (branch-free SpMV loads)

// ---------------------------------------------------------------------------
// Compensated (double-double) accumulation
// ---------------------------------------------------------------------------
struct DD {
  double s, c;
};

__device__ __forceinline__ DD dd_zero() { return DD{0.0, 0.0}; }

__device__ __forceinline__ DD dd_add(DD a, DD b) {
  const double s = a.s + b.s;
  const double bb = s - a.s;
  const double e = (a.s - (s - bb)) + (b.s - bb);
  return DD{s, (a.c + b.c) + e};
}

// a += x*y with an exact product (FMA TwoProduct) and TwoSum.
__device__ __forceinline__ void dd_fma(DD& a, double x, double y) {
  const double p = x * y;
  const double e = __builtin_fma(x, y, -p);
  const double s = a.s + p;
  const double bb = s - a.s;
  const double t = (a.s - (s - bb)) + (p - bb);
  a.s = s;
  a.c = a.c + (t + e);
}

__device__ __forceinline__ double dd_value(DD a) { return a.s + a.c; }

__device__ __forceinline__ DD dd_shfl_xor(DD a, int m) {
  DD r;
  r.s = __shfl_xor(a.s, m, 64);
  r.c = __shfl_xor(a.c, m, 64);
  return r;
}

// Fixed-order workgroup reduction of N DD values; the result is valid in thread 0.
template <int N>
__device__ __forceinline__ void block_reduce_dd(DD (&v)[N], DD* lds /* >= waves*N */) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < N; ++j) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v[j] = dd_add(v[j], dd_shfl_xor(v[j], m));
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) lds[wid * N + j] = v[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      DD a = lds[j];
      for (int w = 1; w < nw; ++w) a = dd_add(a, lds[w * N + j]);
      v[j] = a;
    }
  }
}

// ---------------------------------------------------------------------------
// Agent-scope helpers (MI355X_MICROARCH.md "Valid forms", table row 1): partials are
// published with sc1 (atomic) stores, drained, then one relaxed ticket add; the last
// arriver reads every partial with sc1 loads.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void st_agent_f64(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent_f64(const double* p) {
  unsigned long long u = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double(static_cast<long long>(u));
}

// Grid-wide deterministic reduction of N dot products.  Every workgroup of the launch
// must call it exactly once (uniformly).  The workgroup that arrives last sums all
// partials in block-index order and calls fin(values) on thread 0.
template <int N, class Fin>
__device__ __forceinline__ void grid_reduce_dd(DD (&v)[N], double* partials, unsigned* ticket, Fin fin) {
  __shared__ DD lds[16 * N];  // up to 16 waves (1024 threads)
  __shared__ int s_last;
  block_reduce_dd<N>(v, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      st_agent_f64(&partials[(size_t(blockIdx.x) * N + j) * 2 + 0], v[j].s);
      st_agent_f64(&partials[(size_t(blockIdx.x) * N + j) * 2 + 1], v[j].c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // two-level ticket: same-address device-scope atomics serialise at the memory side, so
    // each group of kTicketGroup workgroups counts on its own cache line and only the group's
    // last arriver touches the top-level ticket (<= G/32 + 32 serialised atomics, not G)
    const unsigned G = gridDim.x;
    const unsigned g = blockIdx.x / kTicketGroup;
    const unsigned gsize = min(unsigned(kTicketGroup), G - g * kTicketGroup);
    const unsigned ng = (G + kTicketGroup - 1) / kTicketGroup;
    unsigned* gt = ticket + kTicketStride * (1 + g);
    int last = 0;
    if (__hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  // Last arriver: every partial is read with sc1 loads, issued in batches of PB per lane
  // before any of them is consumed (one round trip per batch, not one per partial), and
  // summed in block-index order -> the result does not depend on which block was last.
  constexpr int PB = N >= 2 ? 4 : 8;  // <= 16 doubles in flight per thread (VGPR budget of the host kernel)
  DD acc[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = dd_zero();
  const unsigned G = gridDim.x;
  for (unsigned base = 0; base < G; base += blockDim.x * PB) {
    double ps[PB][N], pc[PB][N];
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      unsigned b = base + threadIdx.x + u * blockDim.x;
      b = b < G ? b : G - 1;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        ps[u][j] = ld_agent_f64(&partials[(size_t(b) * N + j) * 2 + 0]);
        pc[u][j] = ld_agent_f64(&partials[(size_t(b) * N + j) * 2 + 1]);
      }
    }
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const bool ok = base + threadIdx.x + u * blockDim.x < G;
#pragma unroll
      for (int j = 0; j < N; ++j) acc[j] = dd_add(acc[j], DD{ok ? ps[u][j] : 0.0, ok ? pc[u][j] : 0.0});
    }
  }
  __syncthreads();
  block_reduce_dd<N>(acc, lds);
  if (threadIdx.x == 0) {
    double out[N];
#pragma unroll
    for (int j = 0; j < N; ++j) out[j] = dd_value(acc[j]);
    fin(out);
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// Split grid reduction (no serialized grid-wide tail): the producing launch only pre-reduces
// its workgroup partials in groups of `gsz` consecutive workgroups -- each group's last
// arriver (one relaxed agent-scope ticket per group) sums the group's partials in block order
// with one wave and stores the group total -- and the CONSUMING launches finish the sum over
// the <= 64 group totals themselves (group_sum_dd, every wave redundantly, same order: every
// consumer sees the identical value).  The group totals are read after a kernel boundary, so
// plain stores / loads suffice for them.  (The measured cost of the last-arriver tail of
// grid_reduce_dd was ~4.3 us per reduction at 1536 workgroups.)
// ---------------------------------------------------------------------------
constexpr int kNoGroupGrid = 512;  // reducing grids up to this size skip the groups (see lspcg_solver_set_spai)
constexpr int kMaxGroups = 64;  // also the largest group SIZE grid_partial_groups handles (one wave sums a group):
                                 // gsz = ceil(grid / 64) <= 64 for every reducing grid <= 4096 (sell_cap); 32 groups measured 90.2 vs 89.1 us

// fixed-order butterfly over a wave; lane 0 ends with the tree sum (lanes >= cnt contribute 0)
template <int N>
__device__ __forceinline__ void wave_reduce_dd(DD (&v)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v[j] = dd_add(v[j], dd_shfl_xor(v[j], m));
  }
}

template <int N>
__device__ __forceinline__ void grid_partial_groups(DD (&v)[N], double* partials, unsigned* ticket, int gsz,
                                                    double* group_out) {
  __shared__ DD lds[16 * N];
  __shared__ int s_last;
  block_reduce_dd<N>(v, lds);
  const unsigned b = blockIdx.x;
  if (gsz <= 1) {  // no groups: every workgroup total is itself a "group" (consumers sum them all)
    if (threadIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        group_out[(size_t(b) * N + j) * 2 + 0] = v[j].s;
        group_out[(size_t(b) * N + j) * 2 + 1] = v[j].c;
      }
    }
    return;
  }
  const unsigned g = b / unsigned(gsz);
  const unsigned g0 = g * unsigned(gsz);
  const unsigned gn = min(unsigned(gsz), gridDim.x - g0);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      st_agent_f64(&partials[(size_t(b) * N + j) * 2 + 0], v[j].s);
      st_agent_f64(&partials[(size_t(b) * N + j) * 2 + 1], v[j].c);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* gt = ticket + kTicketStride * (1 + g);
    const int last = __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1;
    if (last) __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= 64) return;
  const unsigned lane = threadIdx.x;
  DD a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool ok = lane < gn;
    const size_t k = (size_t(g0 + (ok ? lane : 0)) * N + j) * 2;
    const double s = ld_agent_f64(&partials[k + 0]);
    const double c = ld_agent_f64(&partials[k + 1]);
    a[j] = ok ? DD{s, c} : dd_zero();
  }
  wave_reduce_dd<N>(a);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      group_out[(size_t(g) * N + j) * 2 + 0] = a[j].s;
      group_out[(size_t(g) * N + j) * 2 + 1] = a[j].c;
    }
  }
}

// Consumer side: the N sums over the ng group totals, identical in every wave of every launch
// (same tree); returns the DD values collapsed to double.  ng <= 512: one wave, redundantly in
// every wave (lane l sums entries l, l + 64, l + 128, ... in that order, then the butterfly);
// ng > 512: the whole workgroup (fixed strided order + block tree, LDS broadcast; every thread of
// the workgroup must call it).
template <int N>
__device__ __forceinline__ void group_sum_dd(const double* group_in, int ng, double (&out)[N]) {
  if (ng > 64 && ng <= 512) {
    const int lane = threadIdx.x & 63;
    DD a[N];
#pragma unroll
    for (int j = 0; j < N; ++j) a[j] = dd_zero();
    for (int u0 = 0; u0 < 8 && 64 * u0 < ng; u0 += 4) {  // wave-uniform: 1 or 2 rounds of 4 loads
      double gs[4][N], gc[4][N];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = lane + 64 * (u0 + u);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const size_t k = (size_t(g < ng ? g : 0) * N + j) * 2;
          gs[u][j] = group_in[k + 0];
          gc[u][j] = group_in[k + 1];
        }
      }
#pragma unroll
      for (int j = 0; j < N; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (lane + 64 * (u0 + u) < ng) a[j] = dd_add(a[j], DD{gs[u][j], gc[u][j]});
    }
    wave_reduce_dd<N>(a);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double s = __shfl(a[j].s, 0, 64);
      const double c = __shfl(a[j].c, 0, 64);
      out[j] = dd_value(DD{s, c});
    }
    return;
  }
  if (ng > 64) {
    __shared__ DD lds[16 * N];
    __shared__ double res[N];
    DD a[N];
#pragma unroll
    for (int j = 0; j < N; ++j) a[j] = dd_zero();
    for (int g = threadIdx.x; g < ng; g += blockDim.x) {
#pragma unroll
      for (int j = 0; j < N; ++j) a[j] = dd_add(a[j], DD{group_in[(size_t(g) * N + j) * 2], group_in[(size_t(g) * N + j) * 2 + 1]});
    }
    block_reduce_dd<N>(a, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < N; ++j) res[j] = dd_value(a[j]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < N; ++j) out[j] = res[j];
    return;
  }
  const int lane = threadIdx.x & 63;
  DD a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool ok = lane < ng;
    const size_t k = (size_t(ok ? lane : 0) * N + j) * 2;
    const double s = group_in[k + 0];
    const double c = group_in[k + 1];
    a[j] = ok ? DD{s, c} : dd_zero();
  }
  wave_reduce_dd<N>(a);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double s = __shfl(a[j].s, 0, 64);
    const double c = __shfl(a[j].c, 0, 64);
    out[j] = dd_value(DD{s, c});
  }
}

// Explicit global (address space 1) accesses: pointers picked at run time (ping-pong buffers,
// pointers inside structs) otherwise compile to flat_* instructions, which can only be waited
// for with vmcnt(0)+lgkmcnt(0) and serialise a gather loop.
template <typename T>
using gptr_t = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)(p);
}
template <typename T>
__device__ __forceinline__ void gst(T* p, T v) {
  *(__attribute__((address_space(1))) T*)(p) = v;
}

template <typename T>
__device__ __forceinline__ double round_to(double v) {
  return static_cast<double>(static_cast<T>(v));
}

}  // namespace lspcg

struct lspcg_mat;
namespace lspcg {
// (Re)allocate m->colind / m->vals for nnzb stored blocks with zeroed kEntryPad padding.
int mat_alloc_entries(lspcg_mat* m, int64_t nnzb);
// New handle with rowptr[nb+1] and padded entry arrays (contents uninitialised).
int mat_alloc(lspcg_ctx* ctx, int64_t nb, int64_t nnzb, int bs, int dtype, lspcg_mat** out);
// lspcg_mat_transpose; *same_pattern (optional) <- the symmetric-pattern path ran, i.e. Aᵀ has
// A's rowptr / colind and its values are a permutation of A's
// reuse: an owned matrix of A's shape to overwrite instead of allocating (kept by the caller when
// not taken: *out != reuse)
int mat_transpose(const lspcg_mat* A, lspcg_mat** out, bool* same_pattern, lspcg_mat* reuse);
bool mat_reusable(const lspcg_mat* old, const lspcg_mat* like);

// Bandwidth-reducing row placement (lspcg_reorder.hip): perm[i'] = original (block) row of row
// i', iperm its inverse (device arrays, nb entries); off_* = mean |col - row| of the pattern in the
// original / the permuted numbering.
struct Reorder {
  int32_t* perm = nullptr;
  int32_t* iperm = nullptr;
  int64_t nb = 0;
  double off_before = 0, off_after = 0;
  void release();
};
// mean |col - row| over the stored (block) entries
int mean_abs_offset(const lspcg_mat* A, double* out);
// Reverse Cuthill-McKee of A's graph.  mode 0: never, 1: always, -1: auto (only numberings far from
// banded, and only if RCM halves the mean offset).  *applied <- out holds a permutation.
int rcm_reorder(const lspcg_mat* A, int mode, Reorder* out, bool* applied);
// P M P^T with every row's entries in their original order (columns renamed): same row sums
int mat_permute(const lspcg_mat* M, const Reorder& R, lspcg_mat** out, lspcg_mat* reuse = nullptr);
// dst[i'] = src[perm[i']] (scatter = false) or dst[perm[i']] = src[i'] (scatter = true), bs scalars per row
int vec_permute(int dtype, int64_t nb, int bs, const int32_t* perm, const void* src, void* dst, bool scatter,
                hipStream_t st);

}  // namespace lspcg

// ---------------------------------------------------------------------------
// Handle structs (opaque in the C ABI)
// ---------------------------------------------------------------------------
struct lspcg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
};

struct lspcg_mat {
  lspcg_ctx* ctx = nullptr;
  int block_size = 1;   // 1 = scalar CSR, 3 = BSR 3x3
  int dtype = LSPCG_F64;
  int64_t n = 0;        // scalar rows (= cols)
  int64_t nb = 0;       // block rows
  int64_t nnzb = 0;     // stored blocks (scalar nnz when block_size == 1)
  int32_t* rowptr = nullptr;  // [nb+1]
  int32_t* colind = nullptr;  // [nnzb]
  void* vals = nullptr;       // [nnzb*bs*bs], row-major blocks
  // storage type of vals: equals dtype, or LSPCG_F32 for an fp64 matrix whose values are all
  // exactly representable in fp32 (compact storage, fp64 arithmetic: bit-identical results)
  int val_dtype = -1;
  int storage_dtype() const { return val_dtype < 0 ? dtype : val_dtype; }
  // optional SELL-64 copy for lspcg_spmv (lspcg_mat_prepare_spmv; lspcg_sell.hpp), owned
  struct SellCopy* sell = nullptr;
};
