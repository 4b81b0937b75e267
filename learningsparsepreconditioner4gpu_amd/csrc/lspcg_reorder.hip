// Bandwidth-reducing row placement for the PCG solver (DESIGN.md §2 "Reordering").
//
// The SpMV kernels gather x by column; on a structured or mesh-ordered matrix a 64-row slice touches
// a few cache lines of x per slot, on a randomly numbered one every gathered entry is its own line
// (kuhn101rand: 424.8 us per PCG iteration vs 69.9 structured, VERDICT r4 missing #4).  Like a sparse
// library's analysis step, the solver may therefore run on P A P^T with P a reverse Cuthill-McKee
// permutation of A's graph -- WITHOUT changing any row's summation order: row i' of the permuted
// matrix is row perm[i'] of the original with its entries in their ORIGINAL order (only the column
// indices are renamed, col' = iperm[col]), so every row sum, and with it every SpMV result, has
// scipy's csr_matvec bits; L and L^T are permuted after L^T is formed in the original numbering, so
// L^T's rows keep the order scipy's L.T.tocsr() has.  The solver's vectors live in the permuted
// numbering (b, x0 gathered in, x scattered out); the compensated dots are order-insensitive to
// ~1 ulp.  The parity dot order (numpy's ddot order over the ORIGINAL numbering) turns it off.
//
// The permutation is computed on the device, one BFS level per step (a pseudo-peripheral start per
// connected component, then Cuthill-McKee with neighbours by increasing degree, reversed --
// scipy.sparse.csgraph.reverse_cuthill_mckee's algorithm, see rcm_device), and only for matrices
// whose numbering is far from banded: mean |col - row| > 4 nb^(2/3) (a 3-D mesh in
// any locality-preserving order sits well below; a random numbering at ~nb / 3), measured by one
// device reduction first.  The matrices are permuted on the device.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <climits>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "lspcg_internal.hpp"

namespace lspcg {

__global__ void k_abs_offset_sum(int64_t nb, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                 unsigned long long* __restrict__ sum) {
  unsigned long long acc = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nb; i += int64_t(gridDim.x) * blockDim.x) {
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      const int64_t d = int64_t(colind[k]) - i;
      acc += static_cast<unsigned long long>(d < 0 ? -d : d);
    }
  }
  // wave sum, then one atomic per wave (order-independent: integer)
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sum, acc);
}

__global__ void k_perm_len(int64_t nb, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm,
                           int32_t* __restrict__ len) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i <= nb; i += int64_t(gridDim.x) * blockDim.x) {
    if (i < nb) {
      const int32_t o = perm[i];
      len[i] = rowptr[o + 1] - rowptr[o];
    } else {
      len[i] = 0;
    }
  }
}

// one wave per new row: entries copied in their original order, columns renamed; V = one block's
// values as a word type (4 or 8 B), BB = words per block (bs * bs)
template <typename V>
__global__ void __launch_bounds__(256) k_perm_fill(int64_t nb, int bb, const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ colind, const V* __restrict__ vals,
                                                   const int32_t* __restrict__ perm, const int32_t* __restrict__ iperm,
                                                   const int32_t* __restrict__ nrowptr, int32_t* __restrict__ ncolind,
                                                   V* __restrict__ nvals) {
  const int lane = threadIdx.x & 63;
  for (int64_t i = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; i < nb;
       i += (int64_t(gridDim.x) * blockDim.x) >> 6) {
    const int32_t o = perm[i];
    const int32_t s0 = rowptr[o], len = rowptr[o + 1] - s0, d0 = nrowptr[i];
    for (int32_t j = lane; j < len; j += 64) ncolind[d0 + j] = iperm[colind[s0 + j]];
    for (int64_t j = lane; j < int64_t(len) * bb; j += 64) nvals[int64_t(d0) * bb + j] = vals[int64_t(s0) * bb + j];
  }
}

// dst[i'] = src[perm[i']] (gather into the permuted numbering) or dst[perm[i']] = src[i'] (scatter
// back); bs consecutive scalars per block row
template <typename V>
__global__ void k_vec_perm(int64_t nb, int bs, const int32_t* __restrict__ perm, const V* __restrict__ src,
                           V* __restrict__ dst, int scatter) {
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < nb * bs; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = e / bs, c = e - i * bs;
    const int64_t o = int64_t(perm[i]) * bs + c;
    if (scatter) dst[o] = src[e];
    else dst[e] = src[o];
  }
}

static size_t word_size(int dtype) { return dtype == LSPCG_F32 ? 4 : 8; }

static int grid_for(int64_t items, int per_block = kThreads) {
  const int64_t g = (items + per_block - 1) / per_block;
  return int(std::max<int64_t>(1, std::min<int64_t>(g, 16384)));
}

void Reorder::release() {
  (void)hipFree(perm);
  (void)hipFree(iperm);
  perm = iperm = nullptr;
  nb = 0;
}

int mean_abs_offset(const lspcg_mat* A, double* out) {
  hipStream_t st = A->ctx->stream;
  unsigned long long* d = nullptr;
  LSPCG_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  std::unique_ptr<unsigned long long, void (*)(unsigned long long*)> guard(d, [](unsigned long long* p) { (void)hipFree(p); });
  LSPCG_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), st));
  if (A->nb > 0)
    hipLaunchKernelGGL(k_abs_offset_sum, dim3(grid_for(A->nb)), dim3(kThreads), 0, st, A->nb, A->rowptr, A->colind, d);
  unsigned long long h = 0;
  LSPCG_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st));
  LSPCG_HIP(hipStreamSynchronize(st));
  *out = A->nnzb ? double(h) / double(A->nnzb) : 0.0;
  return LSPCG_OK;
}

// ---- reverse Cuthill-McKee on the device (level-synchronous) ---------------------------------
// Sequential Cuthill-McKee appends, while it walks its queue, each node's unvisited neighbours by
// increasing (degree, index); a node of BFS level L+1 is therefore appended by the FIRST node of
// level L (in queue order) adjacent to it, and level L+1 in order is: for each level-L node f in
// order, the children it owns (those whose first parent is f) by (degree, index).  Computed one
// level at a time with no sort and no host round trip: k_rcm_expand records every unvisited
// neighbour's smallest parent position (atomicMin) and stamps it, k_rcm_count counts each parent's
// owned children, k_rcm_emit scans those counts (each parent's output range) and emits each
// parent's children there by (degree, index) -- level sizes and bases stay on the device (the
// kernels size their work from them), and the host reads them back once per kRcmBatch levels.  Nodes whose only neighbour is themselves
// (Dirichlet rows) are placed first, by index; every other component starts from its (degree,
// index)-smallest node, moved once to the (degree, index)-smallest node of its last BFS level (one
// pseudo-peripheral step).  The whole order is reversed at the end.
__global__ void k_rcm_init(int64_t n, const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                           int32_t* __restrict__ deg, uint8_t* __restrict__ iso, int32_t* __restrict__ pos,
                           int32_t* __restrict__ pkey, int32_t* __restrict__ mark, int32_t* __restrict__ maxdeg) {
  int32_t md = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t b = rp[i], e = rp[i + 1];
    bool only_self = true, sorted = true;
    for (int32_t k = b; k < e; ++k) {
      only_self = only_self && ci[k] == i;
      sorted = sorted && (k == b || ci[k] > ci[k - 1]);
    }
    deg[i] = e - b;
    // a row with an unsorted or repeated column would count a child twice: report it as an
    // over-long row, which leaves the matrix in its order
    md = max(md, sorted ? e - b : INT_MAX);
    iso[i] = only_self ? uint8_t(e - b == 0 ? 1 : 2) : uint8_t(0);  // 1: empty row, 2: self loop only
    pos[i] = -1;
    pkey[i] = INT_MAX;
    mark[i] = -1;
  }
  for (int o = 32; o > 0; o >>= 1) md = max(md, __shfl_xor(md, o));
  if ((threadIdx.x & 63) == 0) atomicMax(maxdeg, md);
}

// the (degree, index)-smallest node with pos == -1 (list == nullptr), or among list[0..m)
__global__ void k_rcm_argmin(int64_t m, const int32_t* __restrict__ list, const int32_t* __restrict__ deg,
                             const int32_t* __restrict__ pos, unsigned long long* __restrict__ best) {
  unsigned long long b = ~0ull;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += int64_t(gridDim.x) * blockDim.x) {
    const int32_t v = list ? list[k] : int32_t(k);
    if (list || pos[v] == -1) {
      const unsigned long long key = (static_cast<unsigned long long>(deg[v]) << 32) | unsigned(v);
      b = key < b ? key : b;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(b, o);
    b = t < b ? t : b;
  }
  if ((threadIdx.x & 63) == 0 && b != ~0ull) atomicMin(best, b);
}

// A row's neighbours are visited kRcmChunk at a time with every load of a chunk issued before its
// first use (a node's neighbour loop otherwise makes one dependent memory round trip per neighbour,
// and a BFS level takes as long as its slowest row).
constexpr int kRcmChunk = 16;
struct RowChunk {
  int32_t v[kRcmChunk];
  int cnt;
  __device__ __forceinline__ void load(const int32_t* __restrict__ ci, int32_t k0, int32_t e) {
    cnt = min(kRcmChunk, e - k0);
#pragma unroll
    for (int j = 0; j < kRcmChunk; ++j) v[j] = j < cnt ? ci[k0 + j] : 0;
  }
  __device__ __forceinline__ void gather(const int32_t* __restrict__ a, int32_t (&out)[kRcmChunk]) const {
#pragma unroll
    for (int j = 0; j < kRcmChunk; ++j) out[j] = j < cnt ? a[v[j]] : 0;
  }
};

// pseudo-peripheral BFS level l (marks only, no lists): every node marked base + l marks its
// unplaced neighbours not yet reached by this pass (mark < base) base + l + 1 -- plain stores, all
// of one value, so no atomics -- and raises flag[l + 1].  (Placed nodes are skipped: a directed
// pattern can reach rows an earlier component placed.)
__global__ void k_rcm_pp_mark(int64_t n, int32_t base, int l, int32_t* __restrict__ mark,
                              const int32_t* __restrict__ pos, const int32_t* __restrict__ rp,
                              const int32_t* __restrict__ ci, int32_t* __restrict__ flag) {
  for (int64_t u = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; u < n; u += int64_t(gridDim.x) * blockDim.x) {
    if (mark[u] != base + l) continue;
    bool any = false;
    const int32_t e = rp[u + 1];
    for (int32_t k0 = rp[u]; k0 < e; k0 += kRcmChunk) {
      RowChunk r;
      r.load(ci, k0, e);
      int32_t mk[kRcmChunk], ps[kRcmChunk];
      r.gather(mark, mk);
      r.gather(pos, ps);
#pragma unroll
      for (int j = 0; j < kRcmChunk; ++j)
        if (j < r.cnt && mk[j] < base && ps[j] == -1) {
          mark[r.v[j]] = base + l + 1;
          any = true;
        }
    }
    if (any) flag[l + 1] = 1;
  }
}

// the (degree, index)-smallest node marked `value`
__global__ void k_rcm_argmin_mark(int64_t n, const int32_t* __restrict__ mark, int32_t value,
                                  const int32_t* __restrict__ deg, unsigned long long* __restrict__ best) {
  unsigned long long b = ~0ull;
  for (int64_t v = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; v < n; v += int64_t(gridDim.x) * blockDim.x)
    if (mark[v] == value) {
      const unsigned long long key = (static_cast<unsigned long long>(deg[v]) << 32) | unsigned(v);
      b = key < b ? key : b;
    }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(b, o);
    b = t < b ? t : b;
  }
  if ((threadIdx.x & 63) == 0 && b != ~0ull) atomicMin(best, b);
}

// Cuthill-McKee level lv, step 1: every unplaced neighbour v of frontier[f] gets pkey[v] = the
// smallest such f and mark[v] = stamp (the level's stamp)
__global__ void k_rcm_expand(int lv, const int32_t* __restrict__ lvm, const int32_t* __restrict__ frontier,
                             const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                             const int32_t* __restrict__ pos, int32_t* __restrict__ pkey, int32_t* __restrict__ mark,
                             int32_t stamp) {
  const int64_t m = lvm[lv];
  for (int64_t f = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; f < m; f += int64_t(gridDim.x) * blockDim.x) {
    const int32_t u = frontier[f];
    const int32_t e = rp[u + 1];
    for (int32_t k0 = rp[u]; k0 < e; k0 += kRcmChunk) {
      RowChunk r;
      r.load(ci, k0, e);
      int32_t ps[kRcmChunk];
      r.gather(pos, ps);
#pragma unroll
      for (int j = 0; j < kRcmChunk; ++j)
        if (j < r.cnt && ps[j] == -1) {
          atomicMin(&pkey[r.v[j]], int32_t(f));
          mark[r.v[j]] = stamp;
        }
    }
  }
}

// Steps 2-4 run on kRcmParts workgroups, part b taking parents [b c, (b+1) c), c = ceil(m / parts),
// so their cost follows the level's size (read on the device), not n.
constexpr int kRcmParts = 256;

__device__ __forceinline__ void rcm_part(int64_t m, int64_t* lo, int64_t* hi) {
  const int64_t c = (m + kRcmParts - 1) / kRcmParts;
  *lo = std::min<int64_t>(m, int64_t(blockIdx.x) * c);
  *hi = std::min<int64_t>(m, *lo + c);
}

__device__ __forceinline__ int32_t rcm_owned(int32_t u, int64_t f, const int32_t* __restrict__ rp,
                                             const int32_t* __restrict__ ci, const int32_t* __restrict__ pkey,
                                             const int32_t* __restrict__ mark, int32_t stamp) {
  int32_t c = 0;
  const int32_t e = rp[u + 1];
  for (int32_t k0 = rp[u]; k0 < e; k0 += kRcmChunk) {
    RowChunk r;
    r.load(ci, k0, e);
    int32_t mk[kRcmChunk], pk[kRcmChunk];
    r.gather(mark, mk);
    r.gather(pkey, pk);
#pragma unroll
    for (int j = 0; j < kRcmChunk; ++j) c += (j < r.cnt && mk[j] == stamp && pk[j] == int32_t(f)) ? 1 : 0;
  }
  return c;
}

// 256-thread workgroup sum / exclusive scan through LDS (sh: 256 ints)
__device__ __forceinline__ int32_t block_excl_scan(int32_t x, int32_t* sh, int32_t* total) {
  const int t = threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int32_t y = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += y;
    __syncthreads();
  }
  const int32_t incl = sh[t];
  *total = sh[255];
  __syncthreads();
  return incl - x;
}

// step 2: cnt[f] = the children frontier[f] owns (stamped this level, first parent f); psum[b] =
// the part's total
__global__ void __launch_bounds__(256) k_rcm_count(int lv, const int32_t* __restrict__ lvm,
                                                   const int32_t* __restrict__ frontier, const int32_t* __restrict__ rp,
                                                   const int32_t* __restrict__ ci, const int32_t* __restrict__ pkey,
                                                   const int32_t* __restrict__ mark, int32_t stamp,
                                                   int32_t* __restrict__ cnt, int32_t* __restrict__ psum) {
  __shared__ int32_t sh[256];
  int64_t lo, hi;
  rcm_part(lvm[lv], &lo, &hi);
  int32_t acc = 0;
  for (int64_t f = lo + threadIdx.x; f < hi; f += 256) {
    const int32_t c = rcm_owned(frontier[f], f, rp, ci, pkey, mark, stamp);
    cnt[f] = c;
    acc += c;
  }
  int32_t total;
  block_excl_scan(acc, sh, &total);
  if (threadIdx.x == 0) psum[blockIdx.x] = total;
}

// the next level's step 1 for one of its nodes, v = next[fn], run by the thread that emits v: its
// neighbours neither placed nor in v's own level (stamped `stamp` by this level's step 1; some of
// them may still be unplaced while this kernel runs) get pkey = min(pkey, fn), mark = stamp_next --
// the same sets and keys as k_rcm_expand over the finished level (round 5: one launch per level
// fewer)
__device__ __forceinline__ void rcm_expand_one(int32_t v, int32_t fn, const int32_t* __restrict__ rp,
                                               const int32_t* __restrict__ ci, const int32_t* __restrict__ pos,
                                               int32_t* __restrict__ pkey, int32_t* __restrict__ mark, int32_t stamp,
                                               int32_t stamp_next) {
  const int32_t e = rp[v + 1];
  for (int32_t k0 = rp[v]; k0 < e; k0 += kRcmChunk) {
    RowChunk r;
    r.load(ci, k0, e);
    int32_t ps[kRcmChunk], mk[kRcmChunk];
    r.gather(pos, ps);
    r.gather(mark, mk);
#pragma unroll
    for (int j = 0; j < kRcmChunk; ++j)
      if (j < r.cnt && ps[j] == -1 && mk[j] != stamp) {
        atomicMin(&pkey[r.v[j]], fn);
        mark[r.v[j]] = stamp_next;
      }
  }
}

// step 3: each parent writes its owned children by (degree, index) to next[off ..] and places them
// at lvbase[lv] + m + off + j, off = the totals of the parts before its own (summed by every
// workgroup from psum) + the prefix of cnt inside the part; workgroup 0 publishes the next level's
// size and base.  Then step 1 of the next level for each child (rcm_expand_one).
__global__ void __launch_bounds__(256) k_rcm_emit(int lv, const int32_t* __restrict__ lvm,
                                                  const int32_t* __restrict__ lvbase, const int32_t* __restrict__ frontier,
                                                  const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  const int32_t* __restrict__ deg, int32_t* __restrict__ pkey,
                                                  int32_t* __restrict__ mark, int32_t stamp,
                                                  const int32_t* __restrict__ cnt, const int32_t* __restrict__ psum,
                                                  int32_t* __restrict__ next, int32_t* __restrict__ pos,
                                                  int32_t* __restrict__ order, int32_t* __restrict__ lvm_next,
                                                  int32_t* __restrict__ lvbase_next, int fuse) {
  __shared__ int32_t sh[256];
  const int64_t m = lvm[lv];
  int64_t lo, hi;
  rcm_part(m, &lo, &hi);
  const int32_t base = lvbase[lv] + int32_t(m);
  int32_t total;
  const int32_t before = block_excl_scan(psum[threadIdx.x], sh, &total);  // kRcmParts == blockDim
  if (blockIdx.x == 0 && threadIdx.x == 0 && m > 0) {
    *lvm_next = total;
    *lvbase_next = base;
  }
  if (lo >= hi) return;  // workgroup-uniform
  if (threadIdx.x == blockIdx.x) sh[0] = before;  // this part's offset
  __syncthreads();
  int32_t carry = sh[0];
  __syncthreads();
  for (int64_t f0 = lo; f0 < hi; f0 += 256) {  // workgroup-uniform
    const int64_t f = f0 + threadIdx.x;
    const int32_t c = f < hi ? cnt[f] : 0;
    int32_t tile;
    const int32_t o = carry + block_excl_scan(c, sh, &tile);
    carry += tile;
    if (f >= hi) continue;
    const int32_t u = frontier[f];
    long long last = -1;  // (degree << 32 | index) of the child emitted last
    const int32_t k0 = rp[u], e = rp[u + 1];
    if (e - k0 <= kRcmChunk) {  // the row's owned children ordered in registers
      RowChunk r;
      r.load(ci, k0, e);
      int32_t mk[kRcmChunk], pk[kRcmChunk], dg[kRcmChunk];
      r.gather(mark, mk);
      r.gather(pkey, pk);
      r.gather(deg, dg);
      long long key[kRcmChunk];
#pragma unroll
      for (int j = 0; j < kRcmChunk; ++j)
        key[j] = (j < r.cnt && mk[j] == stamp && pk[j] == int32_t(f))
                     ? (static_cast<long long>(dg[j]) << 32) | unsigned(r.v[j]) : LLONG_MAX;
      for (int32_t j = 0; j < c; ++j) {
        long long best = LLONG_MAX;
#pragma unroll
        for (int q = 0; q < kRcmChunk; ++q)
          if (key[q] > last && key[q] < best) best = key[q];
        const int32_t v = int32_t(best & 0xffffffff);
        next[o + j] = v;
        pos[v] = base + o + j;
        order[base + o + j] = v;
        last = best;
      }
      if (fuse)
        for (int32_t j = 0; j < c; ++j) rcm_expand_one(next[o + j], o + j, rp, ci, pos, pkey, mark, stamp, stamp + 1);
      continue;
    }
    for (int32_t j = 0; j < c; ++j) {
      long long best = LLONG_MAX;
      for (int32_t k = rp[u]; k < rp[u + 1]; ++k) {
        const int32_t v = ci[k];
        if (mark[v] != stamp || pkey[v] != int32_t(f)) continue;
        const long long key = (static_cast<long long>(deg[v]) << 32) | unsigned(v);
        if (key > last && key < best) best = key;
      }
      const int32_t v = int32_t(best & 0xffffffff);
      next[o + j] = v;
      pos[v] = base + o + j;
      order[base + o + j] = v;
      last = best;
    }
    if (fuse)
      for (int32_t j = 0; j < c; ++j) rcm_expand_one(next[o + j], o + j, rp, ci, pos, pkey, mark, stamp, stamp + 1);
  }
}

__global__ void k_rcm_iota(int64_t n, int32_t* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = int32_t(i);
}

__global__ void k_rcm_place(int64_t m, const int32_t* __restrict__ ids, int32_t base, int32_t* __restrict__ pos,
                            int32_t* __restrict__ order) {
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += int64_t(gridDim.x) * blockDim.x) {
    pos[ids[k]] = base + int32_t(k);
    order[base + k] = ids[k];
  }
}

__global__ void k_rcm_flags(int64_t n, const uint8_t* __restrict__ iso, uint8_t want, uint8_t* __restrict__ flag) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    flag[i] = iso[i] == want;
}

// reversal: perm[i'] = order[n - 1 - i'], iperm[perm[i']] = i'
__global__ void k_rcm_reverse(int64_t n, const int32_t* __restrict__ order, int32_t* __restrict__ perm,
                              int32_t* __restrict__ iperm) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t o = order[n - 1 - i];
    perm[i] = o;
    iperm[o] = int32_t(i);
  }
}

__global__ void k_abs_offset_perm(int64_t nb, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                  const int32_t* __restrict__ iperm, unsigned long long* __restrict__ sum) {
  unsigned long long acc = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nb; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t ri = iperm[i];
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      const int64_t d = int64_t(iperm[colind[k]]) - ri;
      acc += static_cast<unsigned long long>(d < 0 ? -d : d);
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sum, acc);
}

namespace {
struct DevBuf {  // hipMalloc'd scratch freed on scope exit
  std::vector<void*> p;
  template <typename T>
  int get(T** out, size_t count) {
    void* v = nullptr;
    LSPCG_HIP(hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T)));
    p.push_back(v);
    *out = static_cast<T*>(v);
    return LSPCG_OK;
  }
  ~DevBuf() {
    for (void* v : p) (void)hipFree(v);
  }
};
}  // namespace

constexpr int kRcmMaxComponents = 256;
constexpr int kRcmMaxDegree = 1024;  // k_rcm_emit orders a parent's children in O(degree^2)
constexpr int kRcmBatch = 16;        // BFS levels enqueued per host read-back
constexpr int kRcmSkip = -1;

// perm / iperm (device, nb entries) of the reverse Cuthill-McKee order of A's block graph;
// kRcmSkip (left in its order) for more than kRcmMaxComponents non-trivial components, a row
// longer than kRcmMaxDegree, or a row whose columns are not strictly increasing
// LSPCG_REORDER_PROFILE=1: phase times of the analysis on stderr (host clock after each sync)
static bool reorder_profile() {
  static const bool on = [] {
    const char* e = std::getenv("LSPCG_REORDER_PROFILE");
    return e && e[0] == '1';
  }();
  return on;
}
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int rcm_device(const lspcg_mat* A, int32_t* perm, int32_t* iperm) {
  hipStream_t st = A->ctx->stream;
  const double t_start = now_ms();
  double t_pp = 0, t_cm = 0;
  int lv_pp = 0, lv_cm = 0;
  const int64_t n = A->nb;
  const int32_t *rp = A->rowptr, *ci = A->colind;
  // level slots over all components: a component's passes use its levels rounded up to whole
  // batches + 2, and the last read-back looks kRcmBatch slots further
  const int64_t nlv = n + int64_t(kRcmMaxComponents) * (kRcmBatch + 2) + 2 * kRcmBatch + 4;
  DevBuf B;
  int32_t *deg, *pos, *pkey, *mark, *order, *fa, *fb, *cnt, *parts, *lvm, *lvbase, *ppm, *misc;
  uint8_t *iso, *flag;
  unsigned long long* best;
  if (int rc = B.get(&deg, n) | B.get(&pos, n) | B.get(&pkey, n) | B.get(&mark, n) | B.get(&order, n) |
               B.get(&fa, n) | B.get(&fb, n) | B.get(&cnt, n) | B.get(&parts, 2 * kRcmParts) | B.get(&lvm, nlv) |
               B.get(&lvbase, nlv) | B.get(&ppm, nlv) | B.get(&misc, 2) | B.get(&iso, n) | B.get(&flag, n) |
               B.get(&best, 1))
    return rc;
  size_t tb = 0;
  LSPCG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, fa, flag, fb, misc, int(n), st));
  void* tmp = nullptr;
  if (int rc = B.get(reinterpret_cast<uint8_t**>(&tmp), tb)) return rc;
  LSPCG_HIP(hipMemsetAsync(lvm, 0, sizeof(int32_t) * nlv, st));
  LSPCG_HIP(hipMemsetAsync(ppm, 0, sizeof(int32_t) * nlv, st));
  LSPCG_HIP(hipMemsetAsync(misc, 0, sizeof(int32_t) * 2, st));
  const int g = grid_for(n);
  hipLaunchKernelGGL(k_rcm_init, dim3(g), dim3(kThreads), 0, st, n, rp, ci, deg, iso, pos, pkey, mark, misc + 1);
  int32_t placed = 0;
  // nodes without neighbours other than themselves: empty rows, then self-loop-only rows, by index
  hipLaunchKernelGGL(k_rcm_iota, dim3(g), dim3(kThreads), 0, st, n, fa);
  for (uint8_t want : {uint8_t(1), uint8_t(2)}) {
    hipLaunchKernelGGL(k_rcm_flags, dim3(g), dim3(kThreads), 0, st, n, iso, want, flag);
    size_t t = tb;
    LSPCG_HIP(hipcub::DeviceSelect::Flagged(tmp, t, fa, flag, fb, misc, int(n), st));
    int32_t h[2] = {0, 0};
    LSPCG_HIP(hipMemcpyAsync(h, misc, sizeof(h), hipMemcpyDeviceToHost, st));
    LSPCG_HIP(hipStreamSynchronize(st));
    if (h[1] > kRcmMaxDegree) return kRcmSkip;
    if (h[0]) hipLaunchKernelGGL(k_rcm_place, dim3(grid_for(h[0])), dim3(kThreads), 0, st, int64_t(h[0]), fb, placed, pos, order);
    placed += h[0];
  }
  // level-parallel kernels: a resident-sized grid striding over the level (its size is on the device)
  const int lg = int(std::min<int64_t>(grid_for(n), 1024));
  int32_t stamp = 0;
  int components = 0;
  int lv = 0, pl = 0;  // next free slots of lvm / lvbase and of ppm
  std::vector<int32_t> hb(kRcmBatch + 1);
  while (placed < n) {
    if (++components > kRcmMaxComponents) return kRcmSkip;
    // component start: the (degree, index)-smallest unplaced node
    const unsigned long long inf = ~0ull;
    unsigned long long hbest = 0;
    LSPCG_HIP(hipMemcpyAsync(best, &inf, sizeof(inf), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_rcm_argmin, dim3(g), dim3(kThreads), 0, st, n, static_cast<const int32_t*>(nullptr), deg, pos, best);
    LSPCG_HIP(hipMemcpyAsync(&hbest, best, sizeof(hbest), hipMemcpyDeviceToHost, st));
    LSPCG_HIP(hipStreamSynchronize(st));
    int32_t start = int32_t(hbest & 0xffffffffu);
    const double t0 = now_ms();
    // one pseudo-peripheral step: BFS from start by marks (level l = mark base + l), then the
    // smallest node of its last level
    {
      const int32_t base = stamp + 1;
      const int32_t one = 1;
      LSPCG_HIP(hipMemcpyAsync(mark + start, &base, sizeof(int32_t), hipMemcpyHostToDevice, st));
      LSPCG_HIP(hipMemcpyAsync(ppm + pl, &one, sizeof(int32_t), hipMemcpyHostToDevice, st));
      int l0 = 0, last = -1;
      while (last < 0) {
        for (int l = l0; l < l0 + kRcmBatch; ++l)
          hipLaunchKernelGGL(k_rcm_pp_mark, dim3(g), dim3(kThreads), 0, st, n, base, l, mark, pos, rp, ci, ppm + pl);
        LSPCG_HIP(hipMemcpyAsync(hb.data(), ppm + pl + l0, sizeof(int32_t) * (kRcmBatch + 1), hipMemcpyDeviceToHost, st));
        LSPCG_HIP(hipStreamSynchronize(st));
        for (int k = 1; k <= kRcmBatch && last < 0; ++k)
          if (hb[k] == 0) last = l0 + k - 1;
        l0 += kRcmBatch;
      }
      LSPCG_HIP(hipMemcpyAsync(best, &inf, sizeof(inf), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_rcm_argmin_mark, dim3(lg), dim3(kThreads), 0, st, n, mark, base + last, deg, best);
      LSPCG_HIP(hipMemcpyAsync(&hbest, best, sizeof(hbest), hipMemcpyDeviceToHost, st));
      LSPCG_HIP(hipStreamSynchronize(st));
      start = int32_t(hbest & 0xffffffffu);
      stamp = base + last + kRcmBatch + 1;  // past every mark this pass (and its trailing batch) wrote
      pl += l0 + 2;
      lv_pp += last + 1;
    }
    const double t1 = now_ms();
    // Cuthill-McKee from start: level 0 = {start} at position `placed`
    {
      const int32_t h0[2] = {1, placed};
      LSPCG_HIP(hipMemcpyAsync(fa, &start, sizeof(int32_t), hipMemcpyHostToDevice, st));
      LSPCG_HIP(hipMemcpyAsync(lvm + lv, &h0[0], sizeof(int32_t), hipMemcpyHostToDevice, st));
      LSPCG_HIP(hipMemcpyAsync(lvbase + lv, &h0[1], sizeof(int32_t), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_rcm_place, dim3(1), dim3(64), 0, st, int64_t(1), fa, placed, pos, order);
      // step 1 of level 0; every later level's runs inside the previous level's emit, stamped one
      // past that level's stamp (round 5's fold; the separate per-level k_rcm_expand launch it
      // replaced measured no faster and was removed in round 6)
      constexpr int fuse = 1;
      hipLaunchKernelGGL(k_rcm_expand, dim3(lg), dim3(kThreads), 0, st, lv, lvm, fa, rp, ci, pos, pkey, mark, ++stamp);
      int l0 = 0, last = -1;
      while (last < 0) {
        for (int l = l0; l < l0 + kRcmBatch; ++l) {
          const int32_t sl = stamp++;  // level l's stamp; the emit stamps level l + 2's nodes sl + 1
          const int32_t* cur = (l & 1) ? fb : fa;
          int32_t* nxt = (l & 1) ? fa : fb;
          hipLaunchKernelGGL(k_rcm_count, dim3(kRcmParts), dim3(256), 0, st, lv + l, lvm, cur, rp, ci, pkey, mark, sl,
                             cnt, parts);
          hipLaunchKernelGGL(k_rcm_emit, dim3(kRcmParts), dim3(256), 0, st, lv + l, lvm, lvbase, cur, rp, ci, deg, pkey,
                             mark, sl, cnt, parts, nxt, pos, order, lvm + lv + l + 1, lvbase + lv + l + 1, fuse);
        }
        LSPCG_HIP(hipMemcpyAsync(hb.data(), lvm + lv + l0, sizeof(int32_t) * (kRcmBatch + 1), hipMemcpyDeviceToHost, st));
        LSPCG_HIP(hipStreamSynchronize(st));
        for (int k = 1; k <= kRcmBatch && last < 0; ++k)
          if (hb[k] == 0) last = l0 + k - 1;
        l0 += kRcmBatch;
      }
      // nodes placed by this component: the sum of its level sizes
      std::vector<int32_t> sizes(last + 1);
      LSPCG_HIP(hipMemcpyAsync(sizes.data(), lvm + lv, sizeof(int32_t) * (last + 1), hipMemcpyDeviceToHost, st));
      LSPCG_HIP(hipStreamSynchronize(st));
      for (int32_t m : sizes) placed += m;
      lv += last + 2;
      lv_cm += last + 1;
    }
    t_pp += t1 - t0;
    t_cm += now_ms() - t1;
  }
  hipLaunchKernelGGL(k_rcm_reverse, dim3(g), dim3(kThreads), 0, st, n, order, perm, iperm);
  LSPCG_HIP(hipGetLastError());
  LSPCG_HIP(hipStreamSynchronize(st));  // the scratch is freed on return
  if (reorder_profile())
    std::fprintf(stderr, "[lspcg reorder] rcm n=%lld components=%d: %.2f ms (pseudo-peripheral %.2f ms / %d levels, "
                 "Cuthill-McKee %.2f ms / %d levels)\n", static_cast<long long>(n), components, now_ms() - t_start,
                 t_pp, lv_pp, t_cm, lv_cm);
  return LSPCG_OK;
}

int rcm_reorder(const lspcg_mat* A, int mode, Reorder* out, bool* applied) {
  *applied = false;
  out->release();
  const int64_t nb = A->nb;
  if (mode == 0 || nb < 2 || A->nnzb == 0) return LSPCG_OK;
  double before = 0;
  if (int rc = mean_abs_offset(A, &before)) return rc;
  out->off_before = before;
  out->off_after = before;
  // auto: only numberings far from banded (a 3-D mesh in a locality-preserving order has mean
  // |col - row| of order nb^(2/3) / 4; a random one ~ nb / 3); never small systems
  if (mode < 0 && (nb < 16384 || before <= 4.0 * std::cbrt(double(nb) * double(nb)))) return LSPCG_OK;
  hipStream_t st = A->ctx->stream;
  LSPCG_HIP(hipMalloc(&out->perm, sizeof(int32_t) * nb));
  LSPCG_HIP(hipMalloc(&out->iperm, sizeof(int32_t) * nb));
  out->nb = nb;
  if (int rc = rcm_device(A, out->perm, out->iperm)) {
    out->release();
    out->off_before = before;
    out->off_after = before;
    return rc == kRcmSkip ? LSPCG_OK : rc;
  }
  {
    unsigned long long* d = nullptr;
    LSPCG_HIP(hipMalloc(&d, sizeof(unsigned long long)));
    LSPCG_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_abs_offset_perm, dim3(grid_for(nb)), dim3(kThreads), 0, st, nb, A->rowptr, A->colind,
                       out->iperm, d);
    unsigned long long h = 0;
    const hipError_t e1 = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st);
    const hipError_t e2 = hipStreamSynchronize(st);
    (void)hipFree(d);
    LSPCG_HIP(e1);
    LSPCG_HIP(e2);
    out->off_after = double(h) / double(A->nnzb);
  }
  if (mode < 0 && !(out->off_after < 0.5 * before)) {  // RCM would not help this pattern
    const double b = out->off_before, a = out->off_after;
    out->release();
    out->off_before = b;
    out->off_after = a;
    return LSPCG_OK;
  }
  *applied = true;
  return LSPCG_OK;
}

int mat_permute(const lspcg_mat* M, const Reorder& R, lspcg_mat** out, lspcg_mat* reuse) {
  LSPCG_CHECK(R.perm && M->nb == R.nb, LSPCG_ERR_ARG, "mat_permute: permutation size differs from the matrix");
  hipStream_t st = M->ctx->stream;
  lspcg_mat* P = nullptr;
  if (mat_reusable(reuse, M)) {  // overwrite a previous P M Pᵀ of the same shape (caller keeps it on failure)
    P = reuse;
  } else {
    reuse = nullptr;
    if (int rc = mat_alloc(M->ctx, M->nb, M->nnzb, M->block_size, M->dtype, &P)) return rc;
  }
  std::unique_ptr<lspcg_mat, int (*)(lspcg_mat*)> guard(reuse ? nullptr : P, lspcg_mat_destroy);
  P->val_dtype = M->val_dtype;
  const int64_t nb = M->nb;
  int32_t* len = nullptr;
  LSPCG_HIP(hipMalloc(&len, sizeof(int32_t) * (nb + 1)));
  std::unique_ptr<int32_t, void (*)(int32_t*)> lguard(len, [](int32_t* p) { (void)hipFree(p); });
  hipLaunchKernelGGL(k_perm_len, dim3(grid_for(nb + 1)), dim3(kThreads), 0, st, nb, M->rowptr, R.perm, len);
  size_t tb = 0;
  LSPCG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, len, P->rowptr, int(nb + 1), st));
  void* tmp = nullptr;
  LSPCG_HIP(hipMalloc(&tmp, tb ? tb : 1));
  std::unique_ptr<void, void (*)(void*)> tguard(tmp, [](void* p) { (void)hipFree(p); });
  LSPCG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, len, P->rowptr, int(nb + 1), st));
  const int bb = M->block_size * M->block_size;
  const int g = grid_for(nb * 64);
  if (word_size(M->storage_dtype()) == 8)
    hipLaunchKernelGGL(k_perm_fill<uint64_t>, dim3(g), dim3(kThreads), 0, st, nb, bb, M->rowptr, M->colind,
                       static_cast<const uint64_t*>(M->vals), R.perm, R.iperm, P->rowptr, P->colind,
                       static_cast<uint64_t*>(P->vals));
  else
    hipLaunchKernelGGL(k_perm_fill<uint32_t>, dim3(g), dim3(kThreads), 0, st, nb, bb, M->rowptr, M->colind,
                       static_cast<const uint32_t*>(M->vals), R.perm, R.iperm, P->rowptr, P->colind,
                       static_cast<uint32_t*>(P->vals));
  LSPCG_HIP(hipGetLastError());
  LSPCG_HIP(hipStreamSynchronize(st));  // len / tmp are freed on return
  guard.release();
  *out = P;
  return LSPCG_OK;
}

int vec_permute(int dtype, int64_t nb, int bs, const int32_t* perm, const void* src, void* dst, bool scatter,
                hipStream_t st) {
  if (nb == 0) return LSPCG_OK;
  const int g = grid_for(nb * bs);
  if (word_size(dtype) == 8)
    hipLaunchKernelGGL(k_vec_perm<uint64_t>, dim3(g), dim3(kThreads), 0, st, nb, bs, perm,
                       static_cast<const uint64_t*>(src), static_cast<uint64_t*>(dst), int(scatter));
  else
    hipLaunchKernelGGL(k_vec_perm<uint32_t>, dim3(g), dim3(kThreads), 0, st, nb, bs, perm,
                       static_cast<const uint32_t*>(src), static_cast<uint32_t*>(dst), int(scatter));
  LSPCG_HIP(hipGetLastError());
  return LSPCG_OK;
}

}  // namespace lspcg

using namespace lspcg;

int lspcg_mat_rcm(const lspcg_mat* A, int32_t* perm, int* applied, double* mean_offset_before,
                  double* mean_offset_after) {
  LSPCG_CHECK(A && perm && applied, LSPCG_ERR_ARG, "mat_rcm: NULL argument");
  Reorder R;
  bool ap = false;
  if (int rc = rcm_reorder(A, 1, &R, &ap)) return rc;
  *applied = ap ? 1 : 0;
  if (mean_offset_before) *mean_offset_before = R.off_before;
  if (mean_offset_after) *mean_offset_after = R.off_after;
  hipError_t e = hipSuccess;
  if (ap) e = hipMemcpyAsync(perm, R.perm, sizeof(int32_t) * A->nb, hipMemcpyDeviceToDevice, A->ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(A->ctx->stream);
  R.release();
  LSPCG_HIP(e);
  return LSPCG_OK;
}
