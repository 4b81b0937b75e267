// Baseline preconditioners of the reference's comparison rows (infer.py:310-321, pymathprim
// "ic" / "ainv") on the GPU:
//
//   IC(0)   A ≈ L Lᵀ, L with the pattern of tril(A)          -> lspcg_ic0, applied by two
//           level-scheduled triangular solves (lspcg_solver_set_ic / LSPCG_PRECOND_IC)
//   AINV(0) A⁻¹ ≈ Z D⁻¹ Zᵀ, Z unit upper with the pattern of triu(A) (Benzi & Tůma incomplete
//           A-biconjugation)                                  -> lspcg_ainv0 returns L = Z D^{-1/2},
//           applied as the ext_spai operator L Lᵀ (+ 0·r) by the SpMV path
//
// Arithmetic (operation order per entry) is fixed by oracle/precond.py; pymathprim's own
// versions are unvendored (parity unpinned).  All factorizations are level scheduled: a row
// (column) depends only on rows of earlier levels, so one launch per level computes every row
// of that level in parallel, one thread per row, with the sequential operation order of the
// oracle.  Levels come from relaxation sweeps (lev[i] = 1 + max lev over dependencies) and a
// stable radix sort of (level, row).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <memory>
#include <string>
#include <vector>

#include "lspcg_factor.hpp"
#include "lspcg_internal.hpp"

namespace lspcg {

static int fgrid(int64_t n) {
  const int64_t g = (n + kThreads - 1) / kThreads;
  return int(std::max<int64_t>(1, std::min<int64_t>(g, 8192)));
}

// ---------------------------------------------------------------------------
// tril pattern (scalar CSR, sorted rows): count / fill; flag 1 = a row without its diagonal
// ---------------------------------------------------------------------------
__global__ void k_tril_count(int64_t n, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                             int32_t* __restrict__ cnt, int* flag) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int c = 0;
    bool diag = false;
    for (int p = rp[i]; p < rp[i + 1]; ++p) {
      const int j = ci[p];
      c += j <= i;
      diag |= j == i;
    }
    cnt[i] = c;
    if (!diag) atomicOr(flag, 1);
  }
}

template <typename T>
__global__ void k_tril_fill(int64_t n, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                            const T* __restrict__ v, const int32_t* __restrict__ orp, int32_t* __restrict__ oci,
                            T* __restrict__ ov) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int o = orp[i];
    for (int p = rp[i]; p < rp[i + 1]; ++p) {
      const int j = ci[p];
      if (j <= i) {
        oci[o] = j;
        if (ov) ov[o] = v[p];
        ++o;
      }
    }
  }
}

// host exclusive scan of cnt[0..n) into a device rowptr (setup path, like lspcg_mat_transpose)
static int scan_to_rowptr(const int32_t* cnt, int64_t n, int32_t* rowptr, int64_t* total, hipStream_t st) {
  std::vector<int32_t> h(n + 1);
  if (n) LSPCG_HIP(hipMemcpyAsync(h.data(), cnt, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  int64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t c = h[i];
    h[i] = int32_t(acc);
    acc += c;
  }
  LSPCG_CHECK(acc < (int64_t(1) << 31), LSPCG_ERR_ARG, "pattern too large for int32 indices");
  h[n] = int32_t(acc);
  LSPCG_HIP(hipMemcpyAsync(rowptr, h.data(), sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  *total = acc;
  return LSPCG_OK;
}

static int flag_value(int* dflag, hipStream_t st, int* out) {
  LSPCG_HIP(hipMemcpyAsync(out, dflag, sizeof(int), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  return LSPCG_OK;
}

// L <- tril(A) (values copied when with_vals)
static int tril_of(const lspcg_mat* A, bool with_vals, lspcg_mat** out) {
  LSPCG_CHECK(A->block_size == 1, LSPCG_ERR_UNSUPPORTED, "tril: scalar CSR required (expand BSR first)");
  hipStream_t st = A->ctx->stream;
  const int64_t n = A->n;
  int32_t* cnt = nullptr;
  int* flag = nullptr;
  LSPCG_HIP(hipMalloc(&cnt, sizeof(int32_t) * std::max<int64_t>(n, 1)));
  LSPCG_HIP(hipMalloc(&flag, sizeof(int)));
  LSPCG_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_tril_count, dim3(fgrid(n)), dim3(kThreads), 0, st, n, A->rowptr, A->colind, cnt, flag);
  int f = 0;
  int rc = flag_value(flag, st, &f);
  if (!rc && f) {
    set_error("factor: a row of A has no stored diagonal entry");
    rc = LSPCG_ERR_FORMAT;
  }
  lspcg_mat* L = nullptr;
  int64_t total = 0;
  if (!rc) {
    // count first, then allocate with the exact entry count
    int32_t* tmp_rp = nullptr;
    LSPCG_HIP(hipMalloc(&tmp_rp, sizeof(int32_t) * (n + 1)));
    rc = scan_to_rowptr(cnt, n, tmp_rp, &total, st);
    if (!rc) rc = mat_alloc(A->ctx, n, total, 1, A->dtype, &L);
    if (!rc) {
      LSPCG_HIP(hipMemcpyAsync(L->rowptr, tmp_rp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToDevice, st));
      if (A->dtype == LSPCG_F64)
        hipLaunchKernelGGL(k_tril_fill<double>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, A->rowptr, A->colind,
                           static_cast<const double*>(A->vals), L->rowptr, L->colind,
                           with_vals ? static_cast<double*>(L->vals) : nullptr);
      else
        hipLaunchKernelGGL(k_tril_fill<float>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, A->rowptr, A->colind,
                           static_cast<const float*>(A->vals), L->rowptr, L->colind,
                           with_vals ? static_cast<float*>(L->vals) : nullptr);
      LSPCG_HIP(hipGetLastError());
      LSPCG_HIP(hipStreamSynchronize(st));
    }
    (void)hipFree(tmp_rp);
  }
  (void)hipFree(cnt);
  (void)hipFree(flag);
  if (rc) {
    if (L) lspcg_mat_destroy(L);
    return rc;
  }
  *out = L;
  return LSPCG_OK;
}

// ---------------------------------------------------------------------------
// level sets
// ---------------------------------------------------------------------------
template <bool LOWER>
__global__ void k_level_sweep(int64_t n, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                              int32_t* lev, int* changed) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int m = 0;
    for (int p = rp[i]; p < rp[i + 1]; ++p) {
      const int64_t j = ci[p];
      if (LOWER ? j < i : j > i) {
        const int l = __hip_atomic_load(lev + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        m = l > m ? l : m;
      }
    }
    if (m > lev[i]) {
      __hip_atomic_store(lev + i, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *changed = 1;
    }
  }
}

__global__ void k_iota(int64_t n, int32_t* v) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    v[i] = int32_t(i);
}

// sorted levels -> ptr[l] = first position of level l (levels are contiguous 0..max)
__global__ void k_level_bounds(int64_t n, const int32_t* __restrict__ ls, int32_t* __restrict__ ptr) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int l = ls[i];
    const int prev = i == 0 ? -1 : ls[i - 1];
    for (int q = prev + 1; q <= l; ++q) ptr[q] = int32_t(i);
    if (i == n - 1) ptr[l + 1] = int32_t(n);
  }
}

void Levels::release() {
  (void)hipFree(ptr);
  (void)hipFree(order);
  (void)hipFree(pad);
  (void)hipFree(head);
  (void)hipFree(sv);
  (void)hipFree(inv);
  (void)hipFree(c);
  sv = inv = c = nullptr;
  ptr = order = pad = nullptr;
  head = nullptr;
  npad = 0;
  hptr.clear();
  nlev = 0;
}

// position t of the level-sorted order -> its place in the wave-padded order
__global__ void k_pad_order(int64_t n, const int32_t* __restrict__ lev_s, const int32_t* __restrict__ ptr,
                            const int32_t* __restrict__ pptr, const int32_t* __restrict__ order, int32_t* __restrict__ pad) {
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < n; t += int64_t(gridDim.x) * blockDim.x) {
    const int l = lev_s[t];
    pad[pptr[l] + (t - ptr[l])] = order[t];
  }
}

int build_levels(lspcg_ctx* ctx, int64_t n, const int32_t* rp, const int32_t* ci, bool lower, Levels* out) {
  hipStream_t st = ctx->stream;
  out->release();
  if (n == 0) {
    out->hptr = {0};
    return LSPCG_OK;
  }
  int32_t *lev = nullptr, *lev_s = nullptr, *iota = nullptr, *order = nullptr, *ptr = nullptr;
  int* changed = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  auto cleanup = [&]() {
    for (void* p : {(void*)lev, (void*)lev_s, (void*)iota, (void*)changed, tmp}) (void)hipFree(p);
  };
  LSPCG_HIP(hipMalloc(&lev, sizeof(int32_t) * n));
  LSPCG_HIP(hipMalloc(&lev_s, sizeof(int32_t) * n));
  LSPCG_HIP(hipMalloc(&iota, sizeof(int32_t) * n));
  LSPCG_HIP(hipMalloc(&order, sizeof(int32_t) * n));
  LSPCG_HIP(hipMalloc(&changed, sizeof(int)));
  LSPCG_HIP(hipMemsetAsync(lev, 0, sizeof(int32_t) * n, st));
  // relaxation sweeps until a round of sweeps changes nothing (<= longest dependency chain + 1
  // sweeps); kSweepRound sweeps per host check of the flag (extra sweeps change nothing)
  constexpr int kSweepRound = 8;
  int h = 1;
  for (int64_t sweep = 0; h && sweep <= n; sweep += kSweepRound) {
    LSPCG_HIP(hipMemsetAsync(changed, 0, sizeof(int), st));
    for (int r = 0; r < kSweepRound; ++r) {
      if (lower)
        hipLaunchKernelGGL(k_level_sweep<true>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, rp, ci, lev, changed);
      else
        hipLaunchKernelGGL(k_level_sweep<false>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, rp, ci, lev, changed);
    }
    LSPCG_HIP(hipMemcpyAsync(&h, changed, sizeof(int), hipMemcpyDeviceToHost, st));
    LSPCG_HIP(hipStreamSynchronize(st));
  }
  hipLaunchKernelGGL(k_iota, dim3(fgrid(n)), dim3(kThreads), 0, st, n, iota);
  LSPCG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, lev, lev_s, iota, order, int(n), 0, 32, st));
  LSPCG_HIP(hipMalloc(&tmp, tmp_bytes));
  LSPCG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, lev, lev_s, iota, order, int(n), 0, 32, st));
  int32_t maxl = 0;
  LSPCG_HIP(hipMemcpyAsync(&maxl, lev_s + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  LSPCG_HIP(hipMalloc(&ptr, sizeof(int32_t) * (maxl + 2)));
  hipLaunchKernelGGL(k_level_bounds, dim3(fgrid(n)), dim3(kThreads), 0, st, n, lev_s, ptr);
  out->hptr.resize(maxl + 2);
  LSPCG_HIP(hipMemcpyAsync(out->hptr.data(), ptr, sizeof(int32_t) * (maxl + 2), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  // wave-padded order for the sync-free solve
  std::vector<int32_t> pptr(maxl + 2, 0);
  for (int l = 0; l <= maxl; ++l) pptr[l + 1] = pptr[l] + (out->hptr[l + 1] - out->hptr[l] + 63) / 64 * 64;
  int32_t* dpptr = nullptr;
  LSPCG_HIP(hipMalloc(&dpptr, sizeof(int32_t) * (maxl + 2)));
  LSPCG_HIP(hipMemcpy(dpptr, pptr.data(), sizeof(int32_t) * (maxl + 2), hipMemcpyHostToDevice));
  LSPCG_HIP(hipMalloc(&out->pad, sizeof(int32_t) * pptr[maxl + 1]));
  LSPCG_HIP(hipMemsetAsync(out->pad, 0xFF, sizeof(int32_t) * pptr[maxl + 1], st));
  hipLaunchKernelGGL(k_pad_order, dim3(fgrid(n)), dim3(kThreads), 0, st, n, lev_s, ptr, dpptr, order, out->pad);
  LSPCG_HIP(hipMalloc(&out->head, 2 * sizeof(unsigned)));  // [dequeue counter | timeout flag]
  LSPCG_HIP(hipMemsetAsync(out->head, 0, 2 * sizeof(unsigned), st));
  LSPCG_HIP(hipStreamSynchronize(st));
  (void)hipFree(dpptr);
  out->npad = pptr[maxl + 1];
  cleanup();
  out->nlev = maxl + 1;
  out->ptr = ptr;
  out->order = order;
  return LSPCG_OK;
}

// ---------------------------------------------------------------------------
// IC(0): one thread per row of the level; oracle/precond.py ic0 operation order
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_ic0_level(const int32_t* __restrict__ order, int32_t beg, int32_t cnt,
                            const int32_t* __restrict__ rp, const int32_t* __restrict__ ci, T* __restrict__ L,
                            int* flag) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const int i = order[beg + t];
  const int pb = rp[i], pd = rp[i + 1] - 1;  // diagonal is the last entry of a tril row
  for (int p = pb; p < pd; ++p) {
    const int k = ci[p];
    T s = L[p];
    // merge the already computed part of row i (columns < k) with row k (off-diagonal part)
    int a = pb, b = rp[k];
    const int be = rp[k + 1] - 1;
    while (a < p && b < be) {
      const int ca = ci[a], cb = ci[b];
      if (ca == cb) {
        s = s - L[a] * L[b];
        ++a;
        ++b;
      } else if (ca < cb) {
        ++a;
      } else {
        ++b;
      }
    }
    L[p] = s / L[be];
  }
  T s = L[pd];
  for (int a = pb; a < pd; ++a) s = s - L[a] * L[a];
  if (!(s > T(0))) {
    atomicOr(flag, 1);
    s = T(1);
  }
  L[pd] = sqrt(s);
}

// ---------------------------------------------------------------------------
// triangular solves (LOWER: diagonal stored last in each row, UPPER: first)
// ---------------------------------------------------------------------------
// Sync-free solve: ONE launch for the whole triangular solve instead of one per level.  A
// resident grid (1 workgroup per CU: few polling waves per CU, short hand-offs) takes 256-position
// blocks of the wave-padded level order from a dequeue counter, in order, so a block only ever
// waits for blocks that running workgroups hold; thread t of block B owns position B*256 + t,
// waits for its dependencies' values (all still-missing ones re-read together per poll round,
// the row's values loaded beforehand) and runs scipy spsolve_triangular's arithmetic (the
// reference's IC apply, validate.py:359-365; oracle/precond.py restates it): a unit solve on the
// column-scaled factor, the row's updates in SuperLU's column order, then k_trsv_post.  The
// hand-off is the value itself: x is first filled with a NaN pattern no arithmetic produces, each
// row publishes its result with one 4- / 8-byte sc1 store (a self-validating granule,
// MI355X_MICROARCH.md R2) and waiters poll with sc1 loads.  A wave never holds rows of two
// levels, so no lane waits for a lane of its own wave.  Forward progress: a block waits only for
// blocks dequeued before it, which resident workgroups hold.  Every wave still has an exit: a row
// whose wait exceeds 2 s (a finished solve's chain is ~2 us per level) raises the levels' error
// word (head[1]) and takes NaN; lspcg_solver_solve / lspcg_trsv then fail with LSPCG_ERR_HIP
// instead of returning a result.
template <typename T>
struct TrsvBits;
template <>
struct TrsvBits<double> {
  using U = unsigned long long;
  static constexpr U kWait = 0x7FF4C0DEDEADBEEFull;  // signalling-NaN payload: never an arithmetic result
};
template <>
struct TrsvBits<float> {
  using U = unsigned;
  static constexpr U kWait = 0x7FA5C0DEu;
};

constexpr int kTrsvBatch = 8;

// read of a dependency's value: an sc1 load (an atomic RMW poll measured the same)
template <typename U>
__device__ __forceinline__ U trsv_poll(const U* p) {
  return __hip_atomic_load(const_cast<U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__global__ void k_trsv_wait_fill(int64_t n, T* __restrict__ x, const int32_t* done) {
  if (done && *done) return;
  using U = typename TrsvBits<T>::U;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    reinterpret_cast<U*>(x)[i] = TrsvBits<T>::kWait;
}

template <typename T, bool LOWER>
__global__ void __launch_bounds__(256) k_trsv_syncfree(int64_t npad, const int32_t* __restrict__ pad,
                                                       const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                       const T* __restrict__ sv, const T* __restrict__ b, T* x,
                                                       const int32_t* done, unsigned* head) {
  using U = typename TrsvBits<T>::U;
  __shared__ unsigned s_blk;
  if (done && *done) return;
  U* xu = reinterpret_cast<U*>(x);
  const unsigned nblk = unsigned((npad + 255) / 256);
  for (;;) {
    // the workgroup takes the next 256-position block (per-wave 64-position blocks measured slower:
    // 4x the dequeues on one counter)
    if (threadIdx.x == 0) s_blk = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned blk = s_blk;
    __syncthreads();
    if (blk >= nblk) return;  // every workgroup leaves through here once the blocks are taken
    const uint64_t t0 = wall_clock64();  // the block's waits are bounded from here
    const int64_t t = int64_t(blk) * 256 + threadIdx.x;
    const int i = t < npad ? pad[t] : -1;
    if (i >= 0) {
      T s = b[i];
      // the off-diagonal entries of row i, visited in spsolve_triangular's update order:
      // increasing column (lower, diagonal last) / decreasing column (upper, diagonal first)
      const int cnt = rp[i + 1] - rp[i] - 1;
      auto entry = [&](int k) { return LOWER ? rp[i] + k : rp[i + 1] - 1 - k; };
      // the dependencies' values are loaded kTrsvBatch at a time, and every poll round re-reads ALL
      // still-waiting ones together: one memory latency per round, not one per entry; the sum
      // then runs in update order
      for (int kb = 0; kb < cnt; kb += kTrsvBatch) {
        U u[kTrsvBatch];
        T w[kTrsvBatch];  // the row's scaled values, loaded before the wait (not after the last hand-off)
        const U* src[kTrsvBatch];
#pragma unroll
        for (int k = 0; k < kTrsvBatch; ++k) {
          const int q = entry(kb + k < cnt ? kb + k : 0);
          src[k] = xu + ci[q];
          w[k] = sv[q];
        }
#pragma unroll
        for (int k = 0; k < kTrsvBatch; ++k) u[k] = trsv_poll(src[k]);
        for (;;) {
          bool wait = false;
#pragma unroll
          for (int k = 0; k < kTrsvBatch; ++k) wait |= (kb + k < cnt) && u[k] == TrsvBits<T>::kWait;
          if (!wait) break;
          if (wall_clock64() - t0 > 200000000ull) {  // 2 s at the 100 MHz constant clock
            __hip_atomic_store(head + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int k = 0; k < kTrsvBatch; ++k)
              if (u[k] == TrsvBits<T>::kWait) u[k] = __builtin_bit_cast(U, T(NAN));
            break;
          }
          __builtin_amdgcn_s_sleep(2);
#pragma unroll
          for (int k = 0; k < kTrsvBatch; ++k)
            if (u[k] == TrsvBits<T>::kWait) u[k] = trsv_poll(src[k]);
        }
#pragma unroll
        for (int k = 0; k < kTrsvBatch; ++k)
          if (kb + k < cnt) s = s - __builtin_bit_cast(T, u[k]) * w[k];
      }
      // unit triangular solve: the published value is y_i itself (k_trsv_post scales it)
      __hip_atomic_store(xu + i, __builtin_bit_cast(U, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// spsolve_triangular's column scaling: inv_i = 1 / d_i, c_i = d_i inv_i (the scaled diagonal the
// lower solve's U phase divides by), then sv_p = v_p inv_{col p}
template <typename T, bool LOWER>
__global__ void k_trsv_inv(int64_t n, const int32_t* __restrict__ rp, const T* __restrict__ v, T* __restrict__ inv,
                           T* __restrict__ c) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const T d = v[LOWER ? rp[i + 1] - 1 : rp[i]];
    const T iv = T(1) / d;
    inv[i] = iv;
    c[i] = d * iv;
  }
}

template <typename T>
__global__ void k_trsv_scale(int64_t nnz, const int32_t* __restrict__ ci, const T* __restrict__ v,
                             const T* __restrict__ inv, T* __restrict__ sv) {
  for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < nnz; p += int64_t(gridDim.x) * blockDim.x)
    sv[p] = v[p] * inv[ci[p]];
}

// x_i = (y_i / c_i) inv_i (lower: SuperLU's U phase divides by the scaled diagonal) or y_i inv_i
// (upper: its L phase divides by the identity's 1)
template <typename T, bool LOWER>
__global__ void k_trsv_post(int64_t n, T* __restrict__ x, const T* __restrict__ c, const T* __restrict__ inv,
                            const int32_t* done) {
  if (done && *done) return;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    if constexpr (LOWER) x[i] = (x[i] / c[i]) * inv[i];
    else x[i] = x[i] * inv[i];
  }
}

int trsv_prepare(const lspcg_mat* T_, bool lower, Levels* lv) {
  LSPCG_CHECK(T_->block_size == 1 && T_->storage_dtype() == T_->dtype, LSPCG_ERR_UNSUPPORTED,
              "trsv: scalar CSR with plain storage required");
  hipStream_t st = T_->ctx->stream;
  const int64_t n = T_->n, nnz = T_->nnzb;
  const size_t es = T_->dtype == LSPCG_F64 ? 8 : 4;
  (void)hipFree(lv->sv);
  (void)hipFree(lv->inv);
  (void)hipFree(lv->c);
  lv->sv = lv->inv = lv->c = nullptr;
  LSPCG_HIP(hipMalloc(&lv->sv, es * std::max<int64_t>(nnz, 1)));
  LSPCG_HIP(hipMalloc(&lv->inv, es * std::max<int64_t>(n, 1)));
  LSPCG_HIP(hipMalloc(&lv->c, es * std::max<int64_t>(n, 1)));
  if (n == 0) return LSPCG_OK;
  auto go = [&](auto tag) {
    using T = decltype(tag);
    auto v = static_cast<const T*>(T_->vals);
    if (lower)
      hipLaunchKernelGGL((k_trsv_inv<T, true>), dim3(fgrid(n)), dim3(kThreads), 0, st, n, T_->rowptr, v,
                         static_cast<T*>(lv->inv), static_cast<T*>(lv->c));
    else
      hipLaunchKernelGGL((k_trsv_inv<T, false>), dim3(fgrid(n)), dim3(kThreads), 0, st, n, T_->rowptr, v,
                         static_cast<T*>(lv->inv), static_cast<T*>(lv->c));
    if (nnz)
      hipLaunchKernelGGL(k_trsv_scale<T>, dim3(fgrid(nnz)), dim3(kThreads), 0, st, nnz, T_->colind, v,
                         static_cast<const T*>(lv->inv), static_cast<T*>(lv->sv));
  };
  if (T_->dtype == LSPCG_F64) go(double{});
  else go(float{});
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int enqueue_trsv(const lspcg_mat* T_, const Levels& lv, bool lower, const void* b, void* x, const int32_t* done,
                 hipStream_t st) {
  if (lv.npad <= 0) return LSPCG_OK;
  LSPCG_CHECK(lv.sv && lv.inv && lv.c, LSPCG_ERR_ARG, "trsv: levels not prepared (trsv_prepare)");
  const int64_t n = T_->n;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  // 1 workgroup per CU (2 or 4 measured slower: more polling waves)
  const dim3 g(unsigned(std::min<int64_t>((lv.npad + 255) / 256, int64_t(cus)))), blk(256);
  LSPCG_HIP(hipMemsetAsync(lv.head, 0, sizeof(unsigned), st));
  auto go = [&](auto tag) {
    using T = decltype(tag);
    auto vx = static_cast<T*>(x);
    auto sv = static_cast<const T*>(lv.sv);
    auto vb = static_cast<const T*>(b);
    hipLaunchKernelGGL(k_trsv_wait_fill<T>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, vx, done);
    if (lower) {
      hipLaunchKernelGGL((k_trsv_syncfree<T, true>), g, blk, 0, st, lv.npad, lv.pad, T_->rowptr, T_->colind, sv, vb,
                         vx, done, lv.head);
      hipLaunchKernelGGL((k_trsv_post<T, true>), dim3(fgrid(n)), dim3(kThreads), 0, st, n, vx,
                         static_cast<const T*>(lv.c), static_cast<const T*>(lv.inv), done);
    } else {
      hipLaunchKernelGGL((k_trsv_syncfree<T, false>), g, blk, 0, st, lv.npad, lv.pad, T_->rowptr, T_->colind, sv, vb,
                         vx, done, lv.head);
      hipLaunchKernelGGL((k_trsv_post<T, false>), dim3(fgrid(n)), dim3(kThreads), 0, st, n, vx,
                         static_cast<const T*>(lv.c), static_cast<const T*>(lv.inv), done);
    }
  };
  if (T_->dtype == LSPCG_F64) go(double{});
  else go(float{});
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int trsv_check_timeout(const Levels& lv, hipStream_t st) {
  if (!lv.head) return LSPCG_OK;
  unsigned h = 0;
  LSPCG_HIP(hipMemcpyAsync(&h, lv.head + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  if (h) {
    LSPCG_HIP(hipMemsetAsync(lv.head + 1, 0, sizeof(unsigned), st));
    LSPCG_HIP(hipStreamSynchronize(st));
    set_error("triangular solve: a row waited more than 2 s for a dependency (sync-free hand-off timed out); "
              "the result is invalid");
    return LSPCG_ERR_HIP;
  }
  return LSPCG_OK;
}

int ic0_factor(const lspcg_mat* A, lspcg_mat** out) {
  LSPCG_CHECK(A && out, LSPCG_ERR_ARG, "ic0: NULL");
  hipStream_t st = A->ctx->stream;
  lspcg_mat* L = nullptr;
  int rc = tril_of(A, true, &L);
  if (rc) return rc;
  Levels lv;
  rc = build_levels(A->ctx, L->n, L->rowptr, L->colind, true, &lv);
  int* flag = nullptr;
  if (!rc && hipMalloc(&flag, sizeof(int)) != hipSuccess) rc = LSPCG_ERR_HIP;
  if (!rc) {
    (void)hipMemsetAsync(flag, 0, sizeof(int), st);
    for (int l = 0; l < lv.nlev; ++l) {
      const int beg = lv.hptr[l], cnt = lv.hptr[l + 1] - lv.hptr[l];
      const dim3 g((cnt + 127) / 128), blk(128);
      if (L->dtype == LSPCG_F64)
        hipLaunchKernelGGL(k_ic0_level<double>, g, blk, 0, st, lv.order, beg, cnt, L->rowptr, L->colind,
                           static_cast<double*>(L->vals), flag);
      else
        hipLaunchKernelGGL(k_ic0_level<float>, g, blk, 0, st, lv.order, beg, cnt, L->rowptr, L->colind,
                           static_cast<float*>(L->vals), flag);
    }
    int f = 0;
    if (hipGetLastError() != hipSuccess) rc = LSPCG_ERR_HIP;
    if (!rc) rc = flag_value(flag, st, &f);
    if (!rc && f) {
      set_error("IC(0) breakdown: a non-positive pivot (the matrix is not an M-matrix / not SPD)");
      rc = LSPCG_ERR_BREAKDOWN;
    }
  }
  (void)hipFree(flag);
  lv.release();
  if (rc) {
    lspcg_mat_destroy(L);
    return rc;
  }
  *out = L;
  return LSPCG_OK;
}

// ---------------------------------------------------------------------------
// AINV(0)
// ---------------------------------------------------------------------------
constexpr int kAinvMaxP = 64;  // |P_j| = entries of tril row j supported by the k-way merge

// candidates C_j = sorted unique {i < j : row i of A meets P_j} = U_{k in P_j} {i in row k of A, i < j}
// (symmetric pattern).  COUNT pass writes cnt[j]; FILL pass writes the list at cp[j].
template <bool FILL>
__global__ void k_ainv_cand(int64_t n, const int32_t* __restrict__ arp, const int32_t* __restrict__ aci,
                            const int32_t* __restrict__ trp, const int32_t* __restrict__ tci, int32_t* cnt,
                            const int32_t* __restrict__ cp, int32_t* __restrict__ cidx, int* flag) {
  for (int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += int64_t(gridDim.x) * blockDim.x) {
    const int pb = trp[j], pe = trp[j + 1];
    const int np = pe - pb;
    if (np > kAinvMaxP) {
      atomicOr(flag, 2);
      if (!FILL) cnt[j] = 0;
      continue;
    }
    int cur[kAinvMaxP], end[kAinvMaxP];
    for (int u = 0; u < np; ++u) {
      const int k = tci[pb + u];
      cur[u] = arp[k];
      end[u] = arp[k + 1];
    }
    int c = 0;
    int last = -1;
    int o = FILL ? cp[j] : 0;
    for (;;) {
      int mn = 0x7fffffff;
      for (int u = 0; u < np; ++u)
        if (cur[u] < end[u]) {
          const int v = aci[cur[u]];
          mn = v < mn ? v : mn;
        }
      if (mn >= j) break;  // every remaining head is >= j (rows are sorted)
      for (int u = 0; u < np; ++u)
        if (cur[u] < end[u] && aci[cur[u]] == mn) ++cur[u];
      if (mn != last) {
        if (FILL) cidx[o++] = mn;
        ++c;
        last = mn;
      }
    }
    if (!FILL) cnt[j] = c;
  }
}

// column j of Z (values z[trp[j]..trp[j+1]), pattern tci) and d_j; oracle/precond.py ainv0 order
template <typename T>
__global__ void k_ainv_level(const int32_t* __restrict__ order, int32_t beg, int32_t cnt,
                             const int32_t* __restrict__ arp, const int32_t* __restrict__ aci,
                             const T* __restrict__ av, const int32_t* __restrict__ trp,
                             const int32_t* __restrict__ tci, const int32_t* __restrict__ cp,
                             const int32_t* __restrict__ cidx, T* __restrict__ z, T* __restrict__ d, int* flag) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const int j = order[beg + t];
  const int pb = trp[j], pe = trp[j + 1];
  for (int c = cp[j]; c < cp[j + 1]; ++c) {
    const int i = cidx[c];
    // p = a_i . z_j over P_j (increasing k)
    T p = T(0);
    {
      int a = arp[i], q = pb;
      const int ae = arp[i + 1];
      while (a < ae && q < pe) {
        const int ca = aci[a], cq = tci[q];
        if (ca == cq) {
          p = p + av[a] * z[q];
          ++a;
          ++q;
        } else if (ca < cq) {
          ++a;
        } else {
          ++q;
        }
      }
    }
    if (p != T(0)) {
      const T f = p / d[i];
      int a = trp[i], q = pb;
      const int ae = trp[i + 1];
      while (a < ae && q < pe) {
        const int ca = tci[a], cq = tci[q];
        if (ca == cq) {
          z[q] = z[q] - f * z[a];
          ++a;
          ++q;
        } else if (ca < cq) {
          ++a;
        } else {
          ++q;
        }
      }
    }
  }
  T dj = T(0);
  {
    int a = arp[j], q = pb;
    const int ae = arp[j + 1];
    while (a < ae && q < pe) {
      const int ca = aci[a], cq = tci[q];
      if (ca == cq) {
        dj = dj + av[a] * z[q];
        ++a;
        ++q;
      } else if (ca < cq) {
        ++a;
      } else {
        ++q;
      }
    }
  }
  if (!(dj > T(0))) {
    atomicOr(flag, 1);
    dj = T(1);
  }
  d[j] = dj;
}

template <typename T>
__global__ void k_ainv_init(int64_t n, const int32_t* __restrict__ trp, T* __restrict__ z) {
  for (int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += int64_t(gridDim.x) * blockDim.x) {
    for (int p = trp[j]; p < trp[j + 1] - 1; ++p) z[p] = T(0);
    z[trp[j + 1] - 1] = T(1);  // diagonal (last entry of the tril row)
  }
}

template <typename T>
__global__ void k_ainv_scale(int64_t n, const int32_t* __restrict__ trp, const T* __restrict__ d, T* __restrict__ z) {
  for (int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += int64_t(gridDim.x) * blockDim.x) {
    const T s = sqrt(d[j]);
    for (int p = trp[j]; p < trp[j + 1]; ++p) z[p] = z[p] / s;
  }
}

template <typename T>
static int ainv0_run(const lspcg_mat* A, lspcg_mat* Zt, const int32_t* cp, const int32_t* cidx, const Levels& lv,
                     T* d, int* flag, hipStream_t st) {
  const int64_t n = A->n;
  T* z = static_cast<T*>(Zt->vals);
  hipLaunchKernelGGL(k_ainv_init<T>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, Zt->rowptr, z);
  for (int l = 0; l < lv.nlev; ++l) {
    const int beg = lv.hptr[l], cnt = lv.hptr[l + 1] - lv.hptr[l];
    hipLaunchKernelGGL(k_ainv_level<T>, dim3((cnt + 127) / 128), dim3(128), 0, st, lv.order, beg, cnt, A->rowptr,
                       A->colind, static_cast<const T*>(A->vals), Zt->rowptr, Zt->colind, cp, cidx, z, d, flag);
  }
  hipLaunchKernelGGL(k_ainv_scale<T>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, Zt->rowptr, d, z);
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

int ainv0_factor(const lspcg_mat* A, lspcg_mat** out) {
  LSPCG_CHECK(A && out, LSPCG_ERR_ARG, "ainv0: NULL");
  LSPCG_CHECK(A->storage_dtype() == A->dtype, LSPCG_ERR_ARG, "ainv0: compact-storage views are not accepted");
  hipStream_t st = A->ctx->stream;
  const int64_t n = A->n;
  lspcg_mat* Zt = nullptr;  // rows = columns of Z (pattern tril(A)), scaled by d^{-1/2} at the end
  int rc = tril_of(A, false, &Zt);
  if (rc) return rc;
  int32_t *cnt = nullptr, *cp = nullptr, *cidx = nullptr;
  int* flag = nullptr;
  void* d = nullptr;
  Levels lv;
  int64_t total = 0;
  auto cleanup = [&]() {
    for (void* p : {(void*)cnt, (void*)cp, (void*)cidx, (void*)flag, d}) (void)hipFree(p);
    lv.release();
  };
  auto fail = [&](int code) {
    cleanup();
    lspcg_mat_destroy(Zt);
    return code;
  };
  if (hipMalloc(&cnt, sizeof(int32_t) * std::max<int64_t>(n, 1)) != hipSuccess ||
      hipMalloc(&cp, sizeof(int32_t) * (n + 1)) != hipSuccess || hipMalloc(&flag, sizeof(int)) != hipSuccess ||
      hipMalloc(&d, (A->dtype == LSPCG_F64 ? 8 : 4) * std::max<int64_t>(n, 1)) != hipSuccess) {
    set_error("ainv0: out of device memory");
    return fail(LSPCG_ERR_HIP);
  }
  (void)hipMemsetAsync(flag, 0, sizeof(int), st);
  hipLaunchKernelGGL(k_ainv_cand<false>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, A->rowptr, A->colind,
                     Zt->rowptr, Zt->colind, cnt, static_cast<const int32_t*>(nullptr), static_cast<int32_t*>(nullptr),
                     flag);
  if ((rc = scan_to_rowptr(cnt, n, cp, &total, st))) return fail(rc);
  if (hipMalloc(&cidx, sizeof(int32_t) * std::max<int64_t>(total, 1)) != hipSuccess) {
    set_error("ainv0: out of device memory (candidate lists)");
    return fail(LSPCG_ERR_HIP);
  }
  hipLaunchKernelGGL(k_ainv_cand<true>, dim3(fgrid(n)), dim3(kThreads), 0, st, n, A->rowptr, A->colind, Zt->rowptr,
                     Zt->colind, cnt, cp, cidx, flag);
  int f = 0;
  if ((rc = flag_value(flag, st, &f))) return fail(rc);
  if (f & 2) {
    set_error("ainv0: a row of tril(A) has more than 64 entries (unsupported)");
    return fail(LSPCG_ERR_UNSUPPORTED);
  }
  if ((rc = build_levels(A->ctx, n, cp, cidx, true, &lv))) return fail(rc);
  rc = A->dtype == LSPCG_F64
           ? ainv0_run<double>(A, Zt, cp, cidx, lv, static_cast<double*>(d), flag, st)
           : ainv0_run<float>(A, Zt, cp, cidx, lv, static_cast<float*>(d), flag, st);
  if (rc) return fail(rc);
  if ((rc = flag_value(flag, st, &f))) return fail(rc);
  if (f & 1) {
    set_error("AINV(0) breakdown: a non-positive pivot");
    return fail(LSPCG_ERR_BREAKDOWN);
  }
  lspcg_mat* L = nullptr;  // L = (D^{-1/2} Zᵀ)ᵀ = Z D^{-1/2}
  rc = lspcg_mat_transpose(Zt, &L);
  cleanup();
  lspcg_mat_destroy(Zt);
  if (rc) return rc;
  *out = L;
  return LSPCG_OK;
}

}  // namespace lspcg

using namespace lspcg;

extern "C" {

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int lspcg_ic0(const lspcg_mat* A, lspcg_mat** L, double* t_ms) {
  LSPCG_CHECK(A && L, LSPCG_ERR_ARG, "ic0: NULL");
  LSPCG_HIP(hipSetDevice(A->ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = ic0_factor(A, L);
  if (t_ms) *t_ms = ms_since(t0);
  return rc;
}

int lspcg_ainv0(const lspcg_mat* A, lspcg_mat** L, double* t_ms) {
  LSPCG_CHECK(A && L, LSPCG_ERR_ARG, "ainv0: NULL");
  LSPCG_HIP(hipSetDevice(A->ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = ainv0_factor(A, L);
  if (t_ms) *t_ms = ms_since(t0);
  return rc;
}

int lspcg_trsv(const lspcg_mat* T, int lower, const void* b, void* x) {
  LSPCG_CHECK(T && (T->n == 0 || (b && x)), LSPCG_ERR_ARG, "trsv: NULL");
  LSPCG_CHECK(T->block_size == 1 && T->storage_dtype() == T->dtype, LSPCG_ERR_UNSUPPORTED,
              "trsv: scalar CSR with plain storage required");
  LSPCG_HIP(hipSetDevice(T->ctx->device));
  Levels lv;
  int rc = build_levels(T->ctx, T->n, T->rowptr, T->colind, lower != 0, &lv);
  if (!rc) rc = trsv_prepare(T, lower != 0, &lv);
  if (!rc) rc = enqueue_trsv(T, lv, lower != 0, b, x, nullptr, T->ctx->stream);
  if (!rc && hipStreamSynchronize(T->ctx->stream) != hipSuccess) {
    set_error("trsv: stream synchronize failed");
    rc = LSPCG_ERR_HIP;
  }
  if (!rc) rc = trsv_check_timeout(lv, T->ctx->stream);
  lv.release();
  return rc;
}

}  // extern "C"
