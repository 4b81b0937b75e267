// SELL-64 view construction (layout and rationale: lspcg_sell.hpp).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <memory>

#include "lspcg_sell.hpp"

namespace lspcg {

// ---- construction kernels --------------------------------------------------
// groups-per-row of each slice = ceil(max row length / 4)
__global__ void k_sell_len(int64_t n, int64_t ns, const int32_t* __restrict__ rowptr, int32_t* __restrict__ cnt) {
  const int64_t s = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= ns) return;
  const int64_t i = s * kSellC + lane;
  int len = i < n ? rowptr[i + 1] - rowptr[i] : 0;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) len = max(len, __shfl_xor(len, m, 64));
  if (lane == 0) cnt[s] = (len + 3) >> 2;
}

// Slot-parallel fill: one workgroup per slice, threads over the slice's 256·G destination slots
// in storage order (coalesced writes; the 4 slots of a row group read 4 consecutive entries of
// that row).  Slot p -> row 64s + (p % 256) / 4, entry 4 (p / 256) + p % 4.  Writes column
// indices (col32 / col16, whichever is non-null) and, if dst != nullptr, values; slots past a
// row's end (or of rows >= n) get value 0 and the padding column (-1 / kSellPad16), so every
// slot of the view is written.
template <typename VS, typename VD>
__global__ void __launch_bounds__(256) k_sell_fill(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                   const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ colind, const VS* __restrict__ src,
                                                   int32_t* __restrict__ col32, int16_t* __restrict__ col16,
                                                   VD* __restrict__ dst) {
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const int64_t base = 256 * int64_t(gp[s]);
    const int32_t slots = 256 * (gp[s + 1] - gp[s]);
    for (int32_t p = threadIdx.x; p < slots; p += blockDim.x) {
      const int64_t i = s * kSellC + ((p & 255) >> 2);
      const int32_t k = 4 * (p >> 8) + (p & 3);
      int32_t b = 0, len = 0;
      if (i < n) {
        b = rowptr[i];
        len = rowptr[i + 1] - b;
      }
      const bool real = k < len;
      if (col32) col32[base + p] = real ? colind[b + k] : int32_t(-1);
      if (col16) col16[base + p] = real ? int16_t(colind[b + k] - int32_t(s * kSellC)) : kSellPad16;
      if (dst) dst[base + p] = real ? VD(src[b + k]) : VD(0);
    }
  }
}

// flag |= bit when some column is more than 32767 away from its slice's first row
__global__ void k_sell_fit16(int64_t n, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                             int* __restrict__ flag, int bit) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t base = int32_t((i / kSellC) * kSellC);
    const int32_t b = rowptr[i], e = rowptr[i + 1];
    // every entry (rows need not be sorted: dist_pcg's extended matrices keep the global order)
    bool far = false;
    for (int32_t k = b; k < e; ++k) {
      const int32_t o = colind[k] - base;
      far |= o < -32767 || o > 32767;
    }
    if (far) atomicOr(flag, bit);
  }
}

// ---- SELL-DIA (layout: lspcg_sell.hpp kSdiaMax) ----------------------------------------------
// Dictionary of slice s: one wave merges its 64 rows' row-relative offsets col - row: every round
// takes the wave minimum m of the lanes' current heads, appends it and advances the lanes whose head
// equals m, so with sorted rows the dictionary comes out ascending and duplicate-free.  cnt[s] =
// D_s.  flag bit 0: some slice has more than 16 offsets, or some row is not sorted (a lane's next
// head not above the value it just consumed) -- no SELL-DIA.
__global__ void k_sdia_dict(int64_t n, int64_t ns, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                            int32_t* __restrict__ dict, int32_t* __restrict__ cnt, int* __restrict__ flag) {
  const int64_t s = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= ns) return;  // wave-uniform
  const int64_t i = s * kSellC + lane;
  int32_t k = 0, e = 0;
  if (i < n) {
    k = rowptr[i];
    e = rowptr[i + 1];
  }
  int nd = 0, mine = 0;
  bool bad = false;
  int prev = INT_MIN;
  for (;;) {
    const int h = k < e ? int(int64_t(colind[k]) - i) : INT_MAX;
    bad |= k < e && h <= prev;  // unsorted (or duplicate) column in this row
    int m = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) m = min(m, __shfl_xor(m, d, 64));
    if (m == INT_MAX) break;
    if (nd == kSdiaMax) {
      bad = true;
      break;
    }
    if (lane == nd) mine = m;
    ++nd;
    if (h == m) {
      prev = h;
      ++k;
    }
  }
  if (__any(bad)) {
    if (lane == 0) atomicOr(flag, 1);
    return;
  }
  if (lane < kSdiaMax) dict[kSdiaMax * s + lane] = lane < nd ? mine : 0;
  if (lane == 0) cnt[s] = nd;
}

// row masks: bit j of row i <=> the row has the offset dict[16 s + j]
__global__ void k_sdia_mask(int64_t n, int64_t ns, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                            const int32_t* __restrict__ dict, const int32_t* __restrict__ gp, uint16_t* __restrict__ mask) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < ns * kSellC; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t s = i / kSellC;
    unsigned m = 0;
    if (i < n) {
      const int nd = gp[s + 1] - gp[s];
      int j = 0;
      for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int off = int(int64_t(colind[k]) - i);
        while (j < nd && dict[kSdiaMax * s + j] != off) ++j;  // both ascending
        m |= 1u << j;
        ++j;
      }
    }
    mask[i] = uint16_t(m);
  }
}

// values: slot j of row i holds the row's entry number popcount(mask & (2^j - 1)) when bit j is set
template <typename VS, typename VD>
__global__ void k_sdia_fill(int64_t n, int64_t ns, const int32_t* __restrict__ gp, const uint16_t* __restrict__ mask,
                            const int32_t* __restrict__ rowptr, const VS* __restrict__ src, VD* __restrict__ dst) {
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const int64_t g0 = gp[s];
    const int32_t slots = kSellC * (gp[s + 1] - gp[s]);
    for (int32_t p = threadIdx.x; p < slots; p += blockDim.x) {
      const int lane = p & 63;
      const int j = p >> 6;
      const int64_t i = s * kSellC + lane;
      const unsigned m = mask[i];
      VD v = VD(0);
      if (i < n && ((m >> j) & 1u)) v = VD(src[rowptr[i] + __builtin_popcount(m & ((1u << j) - 1u))]);
      dst[kSellC * g0 + p] = v;
    }
  }
}

// ---- SELL-64C (layout: lspcg_sell.hpp kSellCodeMax) ------------------------------------------
// Dictionary of slice s: the distinct row-relative offsets col - row of its 64 rows, gathered in a
// per-wave LDS hash set (linear probing, 256 slots), so rows need not be sorted (a reordered solver's
// permuted rows keep their original entry order).  Entries are numbered in slot order: the order is
// immaterial -- a code only names its offset, and slot k stays entry k of its row, so the sum order
// is the CSR's.  dict[64 s + j] (0 past the count); raw[s] = the slice's groups when it has more
// than kSellCodeMax offsets (kept as 16-bit offsets), else 0.
constexpr int kSellcHash = 256;
constexpr int kSellcEmpty = INT_MIN;  // never an offset: |col - row| < 2^31 - 1
__global__ void __launch_bounds__(256) k_sellc_dict(int64_t n, int64_t ns, const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ colind, const int32_t* __restrict__ gp,
                                                    int32_t* __restrict__ dict, int32_t* __restrict__ raw) {
  __shared__ int tab[4][kSellcHash];
  __shared__ int dd[4][kSellCodeMax];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t s = int64_t(blockIdx.x) * 4 + w;
  if (s >= ns) return;  // wave-uniform; only this wave's tables are used below
  for (int j = lane; j < kSellcHash; j += 64) tab[w][j] = kSellcEmpty;
  dd[w][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  const int64_t i = s * kSellC + lane;
  int32_t k = 0, e = 0;
  if (i < n) {
    k = rowptr[i];
    e = rowptr[i + 1];
  }
  bool over = false;
  for (; k < e && !over; ++k) {
    const int off = int(int64_t(colind[k]) - i);
    unsigned h = (unsigned(off) * 0x9E3779B1u) >> 24;  // 8 bits: kSellcHash slots
    int probe = 0;
    for (; probe < kSellcHash; ++probe) {
      const int prev = atomicCAS(&tab[w][h], kSellcEmpty, off);
      if (prev == kSellcEmpty || prev == off) break;
      h = (h + 1) & (kSellcHash - 1);
    }
    over = probe == kSellcHash;  // > 256 distinct offsets
  }
  __builtin_amdgcn_wave_barrier();
  int total = 0;
  for (int c = 0; c < kSellcHash / 64; ++c) {
    const int v = tab[w][64 * c + lane];
    const bool used = v != kSellcEmpty;
    const unsigned long long bal = __ballot(used);
    const int pos = total + __popcll(bal & ((1ull << lane) - 1ull));
    if (used && pos < kSellCodeMax) dd[w][pos] = v;
    total += __popcll(bal);
  }
  __builtin_amdgcn_wave_barrier();
  const bool raw_slice = __any(over) || total > kSellCodeMax;
  dict[kSellCodeMax * s + lane] = raw_slice ? 0 : dd[w][lane];
  if (lane == 0) raw[s] = raw_slice ? gp[s + 1] - gp[s] : 0;
}

// rgp[s] = the first col2 group of an uncoded slice (exclusive prefix of raw), -1 for a coded one
__global__ void k_sellc_rgp(int64_t ns, const int32_t* __restrict__ raw, const int32_t* __restrict__ rscan,
                            int32_t* __restrict__ rgp) {
  for (int64_t s = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; s < ns; s += int64_t(gridDim.x) * blockDim.x)
    rgp[s] = raw[s] ? rscan[s] : -1;
}

// codes (coded slices) or 16-bit offsets (the others), every slot written, in k_sell_fill's order
__global__ void __launch_bounds__(256) k_sellc_fill(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                    const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ colind, const int32_t* __restrict__ dict,
                                                    const int32_t* __restrict__ rgp, uint8_t* __restrict__ col8,
                                                    int16_t* __restrict__ col2) {
  __shared__ int32_t sd[kSellCodeMax];
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    __syncthreads();  // the previous slice's lookups are done
    if (threadIdx.x < kSellCodeMax) sd[threadIdx.x] = dict[kSellCodeMax * s + threadIdx.x];
    __syncthreads();
    const int32_t r0 = rgp[s];
    const int64_t base = 256 * int64_t(gp[s]);
    const int32_t slots = 256 * (gp[s + 1] - gp[s]);
    for (int32_t p = threadIdx.x; p < slots; p += blockDim.x) {
      const int64_t i = s * kSellC + ((p & 255) >> 2);
      const int32_t k = 4 * (p >> 8) + (p & 3);
      int32_t b = 0, len = 0;
      if (i < n) {
        b = rowptr[i];
        len = rowptr[i + 1] - b;
      }
      const bool real = k < len;
      if (r0 < 0) {
        uint8_t code = kSellCodePad;
        if (real) {
          const int off = int(int64_t(colind[b + k]) - i);
          int j = 0;
          while (j < kSellCodeMax - 1 && sd[j] != off) ++j;  // present, once: the dictionary is the slice's set
          code = uint8_t(j);
        }
        col8[base + p] = code;
      } else {
        col8[base + p] = kSellCodePad;
        col2[256 * int64_t(r0) + p] = real ? int16_t(colind[b + k] - int32_t(s * kSellC)) : kSellPad16;
      }
    }
  }
}

// ---- SELL-64J (layout: lspcg_sell.hpp kSellJag) ---------------------------------------------
// One wave per slice: the lanes' ranks by (row length descending, row ascending) -> lmap, the
// per-group lane counts -> jc, the slice's stored entries -> etot.  flag |= 1 when a row has more
// than 16 groups (64 entries): no jagged layout.
__global__ void k_jag_meta(int64_t n, int64_t ns, const int32_t* __restrict__ rowptr, uint8_t* __restrict__ lmap,
                           uint8_t* __restrict__ jc, int32_t* __restrict__ etot, int* __restrict__ flag) {
  const int64_t s = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= ns) return;  // wave-uniform
  const int64_t i = s * kSellC + lane;
  const int len = i < n ? rowptr[i + 1] - rowptr[i] : 0;
  const int g = (len + 3) >> 2;
  if (__any(g > kSellJagMaxG)) {
    if (lane == 0) atomicOr(flag, 1);
    return;
  }
  int rank = 0;
  for (int j = 0; j < 64; ++j) {
    const int lj = __shfl(len, j, 64);
    rank += (lj > len) || (lj == len && j < lane);
  }
  lmap[kSellC * s + rank] = uint8_t(lane);
  int total = 0;
#pragma unroll
  for (int q = 0; q < kSellJagMaxG; ++q) {
    const int c = __popcll(__ballot(g > q));
    if (lane == q) jc[kSellJagMaxG * s + q] = uint8_t(c);
    total += c;
  }
  if (lane == 0) etot[s] = 4 * total;
}

// Element-parallel fill: one workgroup per slice, threads over its stored entries in storage order
// (coalesced writes): element p of the slice -> group q (the counts' prefix in LDS), lane (p - start_q)
// / 4, entry 4 q + p % 4 of that lane's row.  16-bit offsets (col16) and / or values (dst); entries
// past the row's end get kSellPad16 / 0.
template <typename VS, typename VD>
__global__ void __launch_bounds__(256) k_jag_fill(int64_t n, int64_t ns, const int32_t* __restrict__ gp,
                                                  const uint8_t* __restrict__ jc, const uint8_t* __restrict__ lmap,
                                                  const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                                  const VS* __restrict__ src, int16_t* __restrict__ col16,
                                                  VD* __restrict__ dst) {
  __shared__ int32_t start[kSellJagMaxG + 1];
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    __syncthreads();  // the previous slice's lookups are done
    if (threadIdx.x == 0) {
      int32_t e = 0;
      for (int q = 0; q < kSellJagMaxG; ++q) {
        start[q] = e;
        e += 4 * jc[kSellJagMaxG * s + q];
      }
      start[kSellJagMaxG] = e;
    }
    __syncthreads();
    const int64_t e0 = gp[s];
    const int32_t total = start[kSellJagMaxG];
    for (int32_t p = threadIdx.x; p < total; p += blockDim.x) {
      int q = 0;
      while (q + 1 < kSellJagMaxG && start[q + 1] <= p) ++q;
      const int l = (p - start[q]) >> 2;
      const int64_t i = s * kSellC + lmap[kSellC * s + l];
      const int32_t k = 4 * q + (p & 3);
      int32_t b = 0, len = 0;
      if (i < n) {
        b = rowptr[i];
        len = rowptr[i + 1] - b;
      }
      const bool real = k < len;
      if (col16) col16[e0 + p] = real ? int16_t(colind[b + k] - int32_t(s * kSellC)) : kSellPad16;
      if (dst) dst[e0 + p] = real ? VD(src[b + k]) : VD(0);
    }
  }
}

// ---- SELL-64X (layout: lspcg_sell.hpp kSellJagX) --------------------------------------------
// The distinct x blocks (col / 16) of one 256-row tile in an LDS hash set (one workgroup per tile,
// one row per thread); returns the count, or kSellXMax + 1 once the set outgrows the limit.
constexpr int kXsHash = 1024;
__device__ int xs_tile_set(int64_t n, int64_t tile, const int32_t* __restrict__ rowptr,
                           const int32_t* __restrict__ colind, int* tab, int* count, int* maxcol = nullptr) {
  for (int j = threadIdx.x; j < kXsHash; j += blockDim.x) tab[j] = -1;
  if (threadIdx.x == 0) *count = 0;
  __syncthreads();
  const int64_t i = tile * kSellWG + threadIdx.x;
  if (i < n) {
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      const int b = colind[k] / kSellXBlk;
      if (maxcol) atomicMax(maxcol, colind[k]);
      unsigned h = (unsigned(b) * 0x9E3779B1u) >> 22;  // 10 bits
      for (int probe = 0; probe < kXsHash; ++probe, h = (h + 1) & (kXsHash - 1)) {
        const int prev = atomicCAS(&tab[h], -1, b);
        if (prev == -1) {
          atomicAdd(count, 1);
          break;
        }
        if (prev == b) break;
      }
      if (*count > kSellXMax) break;  // (racy read: only ends the insertion early, the flag follows)
    }
  }
  __syncthreads();
  return *count;
}

__global__ void __launch_bounds__(256) k_xs_count(int64_t n, int64_t ntiles, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ colind, int32_t* __restrict__ cnt,
                                                  int* __restrict__ flag) {
  __shared__ int tab[kXsHash];
  __shared__ int count;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int c = xs_tile_set(n, t, rowptr, colind, tab, &count, flag + 3);
    if (threadIdx.x == 0) {
      cnt[t] = c;
      if (c > kSellXMax) atomicOr(flag, 1);
      atomicMax(flag + 1, c);
    }
    __syncthreads();
  }
}

// The tile's ascending block list (xl at xlp[t]) and every stored entry's word: slot * 16 + col % 16
// (the jagged storage order of k_jag_fill; padding keeps kSellPad16).
__global__ void __launch_bounds__(256) k_xs_fill(int64_t n, int64_t ns, int64_t ntiles, const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ colind, const int32_t* __restrict__ xlp,
                                                 const int32_t* __restrict__ gp, const uint8_t* __restrict__ jc,
                                                 const uint8_t* __restrict__ lmap, int32_t* __restrict__ xl,
                                                 int16_t* __restrict__ code) {
  __shared__ int tab[kXsHash];
  __shared__ int sorted[kSellXMax];
  __shared__ int count;
  __shared__ int32_t start[kSellJagMaxG + 1];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int c = xs_tile_set(n, t, rowptr, colind, tab, &count);
    for (int j = threadIdx.x; j < kXsHash; j += blockDim.x) {  // rank = number of smaller keys
      const int b = tab[j];
      if (b < 0) continue;
      int r = 0;
      for (int k = 0; k < kXsHash; ++k) r += (tab[k] >= 0 && tab[k] < b);
      sorted[r] = b;
      xl[xlp[t] + r] = b;
    }
    __syncthreads();
    for (int w = 0; w < kSellWG / kSellC; ++w) {
      const int64_t s = t * (kSellWG / kSellC) + w;
      if (s >= ns) break;  // uniform
      if (threadIdx.x == 0) {
        int32_t e = 0;
        for (int q = 0; q < kSellJagMaxG; ++q) {
          start[q] = e;
          e += 4 * jc[kSellJagMaxG * s + q];
        }
        start[kSellJagMaxG] = e;
      }
      __syncthreads();
      const int64_t e0 = gp[s];
      for (int32_t p = threadIdx.x; p < start[kSellJagMaxG]; p += blockDim.x) {
        int q = 0;
        while (q + 1 < kSellJagMaxG && start[q + 1] <= p) ++q;
        const int64_t i = s * kSellC + lmap[kSellC * s + ((p - start[q]) >> 2)];
        const int32_t k = 4 * q + (p & 3);
        int16_t word = kSellPad16;
        if (i < n && k < rowptr[i + 1] - rowptr[i]) {
          const int col = colind[rowptr[i] + k];
          const int b = col / kSellXBlk;
          int lo = 0, hi = c - 1;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sorted[mid] < b) lo = mid + 1;
            else hi = mid;
          }
          word = int16_t(lo * kSellXBlk + col % kSellXBlk);
        }
        code[e0 + p] = word;
      }
      __syncthreads();  // start[] is rewritten for the next slice
    }
  }
}

static int slice_grid(int64_t ns) { return int(std::max<int64_t>(1, std::min<int64_t>(ns, 16384))); }

// SELL-64X from a SELL-64J pattern (*taken = true when every tile touches <= kSellXMax blocks): the
// column words are rewritten as LDS positions, the block lists added.
static int xs_try(int64_t n, const int32_t* rowptr, const int32_t* colind, hipStream_t st, SellPattern* P,
                  bool* taken) {
  *taken = false;
  const int64_t ntiles = (n + kSellWG - 1) / kSellWG;
  int32_t *cnt = nullptr, *xlp = nullptr, *xl = nullptr;
  int* flag = nullptr;
  void* tmp = nullptr;
  auto done = [&](hipError_t e) {
    (void)hipFree(cnt);
    (void)hipFree(xlp);
    (void)hipFree(xl);
    (void)hipFree(flag);
    (void)hipFree(tmp);
    if (e != hipSuccess) {
      set_error(std::string("sell_build_pattern (x-staged): ") + hipGetErrorString(e));
      return LSPCG_ERR_HIP;
    }
    return LSPCG_OK;
  };
  int flag_h[4] = {1, 0, 0, 0};  // [over the limit, longest list, total, largest column]
  hipError_t e = hipMalloc(&flag, 4 * sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(flag, 0, 4 * sizeof(int), st);
  if (e == hipSuccess) e = hipMalloc(&cnt, sizeof(int32_t) * (ntiles + 1));
  if (e == hipSuccess) e = hipMalloc(&xlp, sizeof(int32_t) * (ntiles + 1));
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (ntiles + 1), st);
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>(ntiles, 8192)));
  if (e == hipSuccess) hipLaunchKernelGGL(k_xs_count, dim3(grid), dim3(256), 0, st, n, ntiles, rowptr, colind, cnt, flag);
  size_t tb = 0;
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, xlp, int(ntiles + 1), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, xlp, int(ntiles + 1), st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag + 2, xlp + ntiles, sizeof(int), hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag_h, flag, 4 * sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess || (flag_h[0] & 1)) return done(e);
  e = hipMalloc(&xl, sizeof(int32_t) * std::max(flag_h[2], 1));
  if (e == hipSuccess)
    hipLaunchKernelGGL(k_xs_fill, dim3(grid), dim3(256), 0, st, n, P->ns, ntiles, rowptr, colind, xlp, P->gp, P->jc,
                       P->lmap, xl, static_cast<int16_t*>(P->col));
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return done(e);
  P->xlp = xlp;
  P->xl = xl;
  P->kx = flag_h[1];
  P->xn = int64_t(flag_h[3]) + 1;
  P->col_bits = kSellJagX;
  xlp = nullptr;
  xl = nullptr;
  *taken = true;
  return done(hipSuccess);
}

// SELL-64J pattern (P: the SELL-64 pattern with 16-bit offsets, already sized): *taken = true when
// every row has <= 64 entries; P's gp becomes the element prefix, col the jagged 16-bit offsets.
static int jag_try(int64_t n, const int32_t* rowptr, const int32_t* colind, hipStream_t st, SellPattern* P,
                   bool* taken) {
  *taken = false;
  int32_t *etot = nullptr, *egp = nullptr;
  uint8_t *lmap = nullptr, *jc = nullptr;
  int16_t* col = nullptr;
  int* flag = nullptr;
  void* tmp = nullptr;
  auto done = [&](hipError_t e) {
    (void)hipFree(etot);
    (void)hipFree(egp);
    (void)hipFree(lmap);
    (void)hipFree(jc);
    (void)hipFree(col);
    (void)hipFree(flag);
    (void)hipFree(tmp);
    if (e != hipSuccess) {
      set_error(std::string("sell_build_pattern (jagged): ") + hipGetErrorString(e));
      return LSPCG_ERR_HIP;
    }
    return LSPCG_OK;
  };
  const int64_t ns = P->ns;
  int flag_h[2] = {1, 0};
  hipError_t e = hipMalloc(&flag, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(flag, 0, 2 * sizeof(int), st);
  if (e == hipSuccess) e = hipMalloc(&etot, sizeof(int32_t) * (ns + 1));
  if (e == hipSuccess) e = hipMalloc(&egp, sizeof(int32_t) * (ns + 1));
  if (e == hipSuccess) e = hipMalloc(&lmap, size_t(kSellC) * ns);
  if (e == hipSuccess) e = hipMalloc(&jc, size_t(kSellJagMaxG) * ns);
  if (e == hipSuccess) e = hipMemsetAsync(etot, 0, sizeof(int32_t) * (ns + 1), st);
  if (e == hipSuccess)
    hipLaunchKernelGGL(k_jag_meta, dim3(unsigned((ns + 3) / 4)), dim3(256), 0, st, n, ns, rowptr, lmap, jc, etot, flag);
  size_t tb = 0;
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, etot, egp, int(ns + 1), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb ? tb : 1);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, etot, egp, int(ns + 1), st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag + 1, egp + ns, sizeof(int), hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag_h, flag, 2 * sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess || (flag_h[0] & 1)) return done(e);
  const int64_t elems = flag_h[1];
  e = hipMalloc(&col, sizeof(int16_t) * std::max<int64_t>(elems, 1));
  if (e == hipSuccess)
    hipLaunchKernelGGL((k_jag_fill<float, float>), dim3(slice_grid(ns)), dim3(256), 0, st, n, ns, egp, jc, lmap, rowptr,
                       colind, static_cast<const float*>(nullptr), col, static_cast<float*>(nullptr));
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return done(e);
  (void)hipFree(P->gp);
  (void)hipFree(P->col);
  P->gp = egp;
  P->col = col;
  P->lmap = lmap;
  P->jc = jc;
  P->elems = elems;
  P->col_bits = kSellJag;
  egp = nullptr;
  col = nullptr;
  lmap = nullptr;
  jc = nullptr;
  *taken = true;
  return done(hipSuccess);
}

static int fill_grid(int64_t n) {
  return int(std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, kElemBlocksMax)));
}

// ---- BSELL-64 (BSR 3x3) ----------------------------------------------------------
// block slots per row of each slice = its longest block row
__global__ void k_bsell_len(int64_t nb, int64_t ns, const int32_t* __restrict__ rowptr, int32_t* __restrict__ cnt) {
  const int64_t s = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s >= ns) return;
  const int64_t I = s * kSellC + lane;
  int len = I < nb ? rowptr[I + 1] - rowptr[I] : 0;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) len = max(len, __shfl_xor(len, m, 64));
  if (lane == 0) cnt[s] = len;
}

// one workgroup per slice, threads over its 64 x G slots in storage order: slot p -> block row
// 64 s + p % 64, block q = p / 64; columns and/or the 9 values in 16-B lane chunks (padding: value 0,
// padding column)
template <typename VS, typename VD>
__global__ void __launch_bounds__(256) k_bsell_fill(int64_t nb, int64_t ns, const int32_t* __restrict__ gp,
                                                    const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ colind, const VS* __restrict__ src,
                                                    int32_t* __restrict__ col32, int16_t* __restrict__ col16,
                                                    VD* __restrict__ dst) {
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const int64_t g0 = gp[s];
    const int32_t slots = 64 * (gp[s + 1] - gp[s]);
    for (int32_t p = threadIdx.x; p < slots; p += blockDim.x) {
      const int lane = p & 63;
      const int32_t q = p >> 6;
      const int64_t I = s * kSellC + lane;
      int32_t b = 0, len = 0;
      if (I < nb) {
        b = rowptr[I];
        len = rowptr[I + 1] - b;
      }
      const bool real = q < len;
      if (col32) col32[64 * g0 + p] = real ? colind[b + q] : int32_t(-1);
      if (col16) col16[64 * g0 + p] = real ? int16_t(colind[b + q] - int32_t(s * kSellC)) : kSellPad16;
      if (dst) {
#pragma unroll
        for (int v = 0; v < 9; ++v)
          dst[576 * (g0 + q) + bsell_pos<VD>(v, lane)] = real ? VD(src[9 * (int64_t(b) + q) + v]) : VD(0);
      }
    }
  }
}

// BSELL-DIA values: slot j of block row I holds the row's block number popcount(mask & (2^j - 1))
// when bit j is set (9 values in the BSELL-64 16-B lane chunks), zeros otherwise
template <typename VS, typename VD>
__global__ void __launch_bounds__(256) k_bsdia_fill(int64_t nb, int64_t ns, const int32_t* __restrict__ gp,
                                                    const uint16_t* __restrict__ mask, const int32_t* __restrict__ rowptr,
                                                    const VS* __restrict__ src, VD* __restrict__ dst) {
  for (int64_t s = blockIdx.x; s < ns; s += gridDim.x) {
    const int64_t g0 = gp[s];
    const int32_t slots = kSellC * (gp[s + 1] - gp[s]);
    for (int32_t p = threadIdx.x; p < slots; p += blockDim.x) {
      const int lane = p & 63;
      const int j = p >> 6;
      const int64_t I = s * kSellC + lane;
      const unsigned m = mask[I];
      const bool real = I < nb && ((m >> j) & 1u);
      const int64_t b = real ? int64_t(rowptr[I]) + __builtin_popcount(m & ((1u << j) - 1u)) : 0;
#pragma unroll
      for (int v = 0; v < 9; ++v) dst[576 * (g0 + j) + bsell_pos<VD>(v, lane)] = real ? VD(src[9 * b + v]) : VD(0);
    }
  }
}

int sell_build_pattern(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, double max_pad,
                       int cols, hipStream_t st, SellPattern* out);

// BSELL-DIA (allow_dia): the SELL-DIA dictionary / masks of the BLOCK graph (k_sdia_dict and
// k_sdia_mask over the block rowptr / colind: offsets in block columns), taken when every slice has
// <= 16 distinct block offsets and it stores at most 1/16 more block slots than BSELL-64
static int bsdia_try(int64_t nb, const int32_t* rowptr, const int32_t* colind, hipStream_t st, SellPattern* P,
                     bool* taken) {
  *taken = false;
  int32_t *cnt = nullptr, *dgp = nullptr, *dict = nullptr;
  int* flag = nullptr;
  void* tmp = nullptr;
  uint16_t* mask = nullptr;
  auto done = [&](hipError_t e) {
    (void)hipFree(cnt);
    (void)hipFree(tmp);
    (void)hipFree(flag);
    (void)hipFree(dgp);
    (void)hipFree(dict);
    (void)hipFree(mask);
    if (e != hipSuccess) {
      set_error(std::string("bsell_build_pattern (DIA): ") + hipGetErrorString(e));
      return LSPCG_ERR_HIP;
    }
    return LSPCG_OK;
  };
  const int64_t ns = P->ns;
  int flag_h[2] = {1, 0};
  hipError_t e = hipMalloc(&flag, 2 * sizeof(int));
  if (e == hipSuccess) e = hipMemsetAsync(flag, 0, 2 * sizeof(int), st);
  if (e == hipSuccess) e = hipMalloc(&dict, sizeof(int32_t) * kSdiaMax * ns);
  if (e == hipSuccess) e = hipMalloc(&cnt, sizeof(int32_t) * (ns + 1));
  if (e == hipSuccess) e = hipMalloc(&dgp, sizeof(int32_t) * (ns + 1));
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (ns + 1), st);
  if (e == hipSuccess)
    hipLaunchKernelGGL(k_sdia_dict, dim3(unsigned((ns + 3) / 4)), dim3(256), 0, st, nb, ns, rowptr, colind, dict, cnt,
                       flag);
  size_t tb = 0;
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, dgp, int(ns + 1), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, dgp, int(ns + 1), st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag + 1, dgp + ns, sizeof(int), hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(flag_h, flag, 2 * sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return done(e);
  // a slice whose distinct offsets outnumber its longest row pads a little more than BSELL-64
  // (C4: 24,574 vs 24,572 slots); the column loads it drops are worth up to 1/16 more slots
  if ((flag_h[0] & 1) || int64_t(flag_h[1]) > P->groups + P->groups / 16) return done(hipSuccess);
  e = hipMalloc(&mask, sizeof(uint16_t) * kSellC * std::max<int64_t>(ns, 1));
  if (e != hipSuccess) return done(e);
  hipLaunchKernelGGL(k_sdia_mask, dim3(fill_grid(ns * kSellC)), dim3(kThreads), 0, st, nb, ns, rowptr, colind, dict, dgp,
                     mask);
  e = hipGetLastError();
  if (e != hipSuccess) return done(e);
  (void)hipFree(P->gp);
  P->gp = dgp;
  P->dict = dict;
  P->col = mask;
  P->groups = flag_h[1];
  P->col_bits = 1;
  dgp = nullptr;
  dict = nullptr;
  mask = nullptr;
  *taken = true;
  return done(hipSuccess);
}

int bsell_build_pattern(int64_t nb, int64_t nnzb, const int32_t* rowptr, const int32_t* colind, double max_pad,
                        bool allow16, bool allow_dia, hipStream_t st, SellPattern* out) {
  SellPattern P;
  P.n = 3 * nb;
  P.nb = nb;
  P.bs = 3;
  P.ns = (nb + kSellC - 1) / kSellC;
  P.rowptr = rowptr;
  int32_t* cnt = nullptr;
  void* tmp = nullptr;
  auto fail = [&](hipError_t e) {
    set_error(std::string("bsell_build_pattern: ") + hipGetErrorString(e));
    (void)hipFree(cnt);
    (void)hipFree(tmp);
    P.release();
    return LSPCG_ERR_HIP;
  };
  hipError_t e = hipMalloc(&cnt, sizeof(int32_t) * (P.ns + 1));
  if (e == hipSuccess) e = hipMalloc(&P.gp, sizeof(int32_t) * (P.ns + 1));
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (P.ns + 1), st);
  if (e != hipSuccess) return fail(e);
  if (P.ns) hipLaunchKernelGGL(k_bsell_len, dim3(unsigned((P.ns + 3) / 4)), dim3(256), 0, st, nb, P.ns, rowptr, cnt);
  size_t tb = 0;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, P.gp, int(P.ns + 1), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, P.gp, int(P.ns + 1), st);
  int32_t groups = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&groups, P.gp + P.ns, sizeof(int32_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return fail(e);
  (void)hipFree(cnt);
  (void)hipFree(tmp);
  cnt = nullptr;
  tmp = nullptr;
  P.groups = groups;
  if (double(64) * double(groups) > max_pad * double(std::max<int64_t>(nnzb, 1))) {
    P.release();
    set_error("bsell: padding exceeds the limit (irregular block-row lengths)");
    return LSPCG_ERR_UNSUPPORTED;
  }
  if (allow_dia && nb) {
    bool taken = false;
    if (int rc = bsdia_try(nb, rowptr, colind, st, &P, &taken)) {
      P.release();
      return rc;
    }
    if (taken) {
      *out = P;
      return LSPCG_OK;
    }
  }
  int fit = 1;
  if (allow16 && nb) {
    int* flag = nullptr;
    e = hipMalloc(&flag, sizeof(int));
    if (e == hipSuccess) e = hipMemsetAsync(flag, 0, sizeof(int), st);
    if (e == hipSuccess)
      hipLaunchKernelGGL(k_sell_fit16, dim3(fill_grid(nb)), dim3(kThreads), 0, st, nb, rowptr, colind, flag, 1);
    if (e == hipSuccess) e = hipMemcpyAsync(&fit, flag, sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(flag);
    if (e != hipSuccess) return fail(e);
  }
  P.col_bits = fit == 0 ? 16 : 32;
  e = hipMalloc(&P.col, size_t(P.col_bits / 8) * size_t(std::max<int64_t>(64 * P.groups, 1)));
  if (e != hipSuccess) return fail(e);
  if (P.ns)
    hipLaunchKernelGGL((k_bsell_fill<float, float>), dim3(slice_grid(P.ns)), dim3(256), 0, st, nb, P.ns, P.gp, rowptr,
                       colind, static_cast<const float*>(nullptr),
                       P.col_bits == 32 ? static_cast<int32_t*>(P.col) : nullptr,
                       P.col_bits == 16 ? static_cast<int16_t*>(P.col) : nullptr, static_cast<float*>(nullptr));
  e = hipGetLastError();
  if (e != hipSuccess) return fail(e);
  *out = P;
  return LSPCG_OK;
}

int bsell_fill_values(const SellPattern& P, const void* src, int src_dtype, int dst_dtype, hipStream_t st, void** out) {
  const size_t es = dst_dtype == LSPCG_F32 ? 4 : 8;
  void* v = *out;  // an existing array of this pattern and dtype is refilled in place
  const bool mine = v == nullptr;
  if (!v) LSPCG_HIP(hipMalloc(&v, es * std::max<int64_t>(576 * P.groups, 1)));
  const dim3 g(slice_grid(P.ns)), b(256);
  const int32_t* nocol = nullptr;
  if (P.ns && P.col_bits == 1) {
    const auto* m = static_cast<const uint16_t*>(P.col);
    if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F64)
      hipLaunchKernelGGL((k_bsdia_fill<double, double>), g, b, 0, st, P.nb, P.ns, P.gp, m, P.rowptr,
                         static_cast<const double*>(src), static_cast<double*>(v));
    else if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_bsdia_fill<double, float>), g, b, 0, st, P.nb, P.ns, P.gp, m, P.rowptr,
                         static_cast<const double*>(src), static_cast<float*>(v));
    else if (src_dtype == LSPCG_F32 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_bsdia_fill<float, float>), g, b, 0, st, P.nb, P.ns, P.gp, m, P.rowptr,
                         static_cast<const float*>(src), static_cast<float*>(v));
    else
      hipLaunchKernelGGL((k_bsdia_fill<float, double>), g, b, 0, st, P.nb, P.ns, P.gp, m, P.rowptr,
                         static_cast<const float*>(src), static_cast<double*>(v));
  } else if (P.ns) {
    if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F64)
      hipLaunchKernelGGL((k_bsell_fill<double, double>), g, b, 0, st, P.nb, P.ns, P.gp, P.rowptr, nocol,
                         static_cast<const double*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr),
                         static_cast<double*>(v));
    else if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_bsell_fill<double, float>), g, b, 0, st, P.nb, P.ns, P.gp, P.rowptr, nocol,
                         static_cast<const double*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr),
                         static_cast<float*>(v));
    else if (src_dtype == LSPCG_F32 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_bsell_fill<float, float>), g, b, 0, st, P.nb, P.ns, P.gp, P.rowptr, nocol,
                         static_cast<const float*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr),
                         static_cast<float*>(v));
    else
      hipLaunchKernelGGL((k_bsell_fill<float, double>), g, b, 0, st, P.nb, P.ns, P.gp, P.rowptr, nocol,
                         static_cast<const float*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr),
                         static_cast<double*>(v));
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    if (mine) (void)hipFree(v);
    set_error(std::string("bsell_fill_values: ") + hipGetErrorString(e));
    return LSPCG_ERR_HIP;
  }
  *out = v;
  return LSPCG_OK;
}

int sell_build_pattern(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, double max_pad,
                       int cols, hipStream_t st, SellPattern* out) {
  SellPattern P;
  P.n = n;
  P.nb = n;
  P.ns = (n + kSellC - 1) / kSellC;
  P.rowptr = rowptr;
  int32_t* cnt = nullptr;
  void* tmp = nullptr;
  auto fail = [&](hipError_t e) {
    set_error(std::string("sell_build_pattern: ") + hipGetErrorString(e));
    (void)hipFree(cnt);
    (void)hipFree(tmp);
    P.release();
    return LSPCG_ERR_HIP;
  };
  hipError_t e = hipMalloc(&cnt, sizeof(int32_t) * (P.ns + 1));
  if (e == hipSuccess) e = hipMalloc(&P.gp, sizeof(int32_t) * (P.ns + 1));
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (P.ns + 1), st);
  if (e != hipSuccess) return fail(e);
  if (P.ns) hipLaunchKernelGGL(k_sell_len, dim3(unsigned((P.ns + 3) / 4)), dim3(256), 0, st, n, P.ns, rowptr, cnt);
  size_t tb = 0;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, P.gp, int(P.ns + 1), st);
  if (e == hipSuccess) e = hipMalloc(&tmp, tb);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, P.gp, int(P.ns + 1), st);
  int32_t groups = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&groups, P.gp + P.ns, sizeof(int32_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return fail(e);
  (void)hipFree(cnt);
  (void)hipFree(tmp);
  cnt = nullptr;
  tmp = nullptr;
  P.groups = groups;
  // padding past max_pad: only the jagged layout (which pads just each row's last group) may remain
  const bool overpad = double(256) * double(groups) > max_pad * double(std::max<int64_t>(nnz, 1));
  auto reject = [&]() {
    P.release();
    set_error("sell: padding exceeds the limit (irregular row lengths)");
    return LSPCG_ERR_UNSUPPORTED;
  };
  if (overpad && !(cols & kSellColJag)) return reject();
  if (overpad) cols &= ~(kSellColDia | kSellColCode);
  // SELL-DIA: dictionaries and slot counts first; one host read of (flag, DIA slot total) decides
  int fit16 = 0;  // 1 = some column out of 16-bit offset range
  int flag_h[2] = {1, 0};  // [flags (bit 0: no SELL-DIA, bit 1: no 16-bit offsets), SELL-DIA slots]
  int32_t* dgp = nullptr;  // DIA slot prefix
  int* flag = nullptr;
  if (n) {
    e = hipMalloc(&flag, 2 * sizeof(int));
    if (e == hipSuccess) e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flag), (cols & kSellColDia) ? 0 : 1, 1, st);
    if (e == hipSuccess) e = hipMemsetAsync(flag + 1, 0, sizeof(int), st);
    if (e == hipSuccess && (cols & kSellColDia)) {
      e = hipMalloc(&P.dict, sizeof(int32_t) * kSdiaMax * P.ns);
      if (e == hipSuccess) e = hipMalloc(&cnt, sizeof(int32_t) * (P.ns + 1));
      if (e == hipSuccess) e = hipMalloc(&dgp, sizeof(int32_t) * (P.ns + 1));
      if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(int32_t) * (P.ns + 1), st);
      if (e == hipSuccess)
        hipLaunchKernelGGL(k_sdia_dict, dim3(unsigned((P.ns + 3) / 4)), dim3(256), 0, st, n, P.ns, rowptr, colind, P.dict,
                           cnt, flag);
      size_t tb2 = 0;
      if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, cnt, dgp, int(P.ns + 1), st);
      if (e == hipSuccess) e = hipMalloc(&tmp, tb2);
      if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb2, cnt, dgp, int(P.ns + 1), st);
      if (e == hipSuccess) e = hipMemcpyAsync(flag + 1, dgp + P.ns, sizeof(int), hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess && (cols & kSellCol16))
      hipLaunchKernelGGL(k_sell_fit16, dim3(fill_grid(n)), dim3(kThreads), 0, st, n, rowptr, colind, flag, 2);
    if (e == hipSuccess) e = hipMemcpyAsync(flag_h, flag, 2 * sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(cnt);
    (void)hipFree(tmp);
    cnt = nullptr;
    tmp = nullptr;
    if (e != hipSuccess) {
      (void)hipFree(flag);
      (void)hipFree(dgp);
      return fail(e);
    }
    fit16 = (!(cols & kSellCol16) || (flag_h[0] & 2)) ? 1 : 0;
  } else {
    fit16 = (cols & kSellCol16) ? 0 : 1;
  }
  // SELL-DIA when it fits and stores no more slots than the 4-entry groups
  const bool dia = n && !(flag_h[0] & 1) && int64_t(flag_h[1]) <= 4 * P.groups;
  if (dia) {
    (void)hipFree(P.gp);
    P.gp = dgp;
    dgp = nullptr;
    P.groups = flag_h[1];
    P.col_bits = 1;
    e = hipMalloc(&P.col, sizeof(uint16_t) * kSellC * std::max<int64_t>(P.ns, 1));
    (void)hipFree(flag);
    if (e != hipSuccess) return fail(e);
    hipLaunchKernelGGL(k_sdia_mask, dim3(fill_grid(P.ns * kSellC)), dim3(kThreads), 0, st, n, P.ns, rowptr, colind, P.dict,
                       P.gp, static_cast<uint16_t*>(P.col));
    e = hipGetLastError();
    if (e != hipSuccess) return fail(e);
    *out = P;
    return LSPCG_OK;
  }
  (void)hipFree(flag);
  (void)hipFree(dgp);
  (void)hipFree(P.dict);
  P.dict = nullptr;
  if ((cols & kSellColCode) && !fit16 && n && P.groups > 0) {
    // SELL-64C when at least half of the slots lie in slices of <= 64 distinct offsets
    int32_t* raw = nullptr;
    int32_t* rscan = nullptr;
    int32_t rawg = 0;
    e = hipMalloc(&P.dict, sizeof(int32_t) * kSellCodeMax * P.ns);
    if (e == hipSuccess) e = hipMalloc(&raw, sizeof(int32_t) * (P.ns + 1));
    if (e == hipSuccess) e = hipMalloc(&rscan, sizeof(int32_t) * (P.ns + 1));
    if (e == hipSuccess) e = hipMemsetAsync(raw, 0, sizeof(int32_t) * (P.ns + 1), st);
    if (e == hipSuccess)
      hipLaunchKernelGGL(k_sellc_dict, dim3(unsigned((P.ns + 3) / 4)), dim3(256), 0, st, n, P.ns, rowptr, colind, P.gp,
                         P.dict, raw);
    size_t tb3 = 0;
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, raw, rscan, int(P.ns + 1), st);
    if (e == hipSuccess) e = hipMalloc(&tmp, tb3 ? tb3 : 1);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb3, raw, rscan, int(P.ns + 1), st);
    if (e == hipSuccess) e = hipMemcpyAsync(&rawg, rscan + P.ns, sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(tmp);
    tmp = nullptr;
    if (e == hipSuccess && int64_t(rawg) * 2 <= P.groups) {
      e = hipMalloc(&P.rgp, sizeof(int32_t) * P.ns);
      if (e == hipSuccess) e = hipMalloc(&P.col, std::max<size_t>(size_t(256) * size_t(P.groups), 1));
      if (e == hipSuccess) e = hipMalloc(&P.col2, sizeof(int16_t) * std::max<size_t>(size_t(256) * size_t(rawg), 1));
      if (e == hipSuccess) {
        hipLaunchKernelGGL(k_sellc_rgp, dim3(fill_grid(P.ns)), dim3(kThreads), 0, st, P.ns, raw, rscan, P.rgp);
        hipLaunchKernelGGL(k_sellc_fill, dim3(slice_grid(P.ns)), dim3(256), 0, st, n, P.ns, P.gp, rowptr, colind, P.dict,
                           P.rgp, static_cast<uint8_t*>(P.col), P.col2);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipStreamSynchronize(st);  // raw / rscan are freed below
      (void)hipFree(raw);
      (void)hipFree(rscan);
      if (e != hipSuccess) return fail(e);
      P.col_bits = 8;
      *out = P;
      return LSPCG_OK;
    }
    (void)hipFree(raw);
    (void)hipFree(rscan);
    (void)hipFree(P.dict);
    P.dict = nullptr;
    if (e != hipSuccess) return fail(e);
  }
  if ((cols & kSellColJag) && !fit16 && n && double(256) * double(P.groups) > kSellJagPad * double(nnz)) {
    bool taken = false;  // irregular row lengths: the jagged layout stores ~1.1 x nnz instead
    if (int rc = jag_try(n, rowptr, colind, st, &P, &taken)) {
      P.release();
      return rc;
    }
    if (taken && (cols & kSellColXs) && n >= kSellXMinN) {  // stage each tile's x blocks in LDS where they fit
      bool xs = false;
      if (int rc = xs_try(n, rowptr, colind, st, &P, &xs)) {
        P.release();
        return rc;
      }
    }
    if (taken) {
      *out = P;
      return LSPCG_OK;
    }
  }
  if (overpad) return reject();
  P.col_bits = fit16 ? 32 : 16;
  // the fill writes every slot (padding included)
  const size_t cbytes = size_t(P.col_bits / 8) * size_t(std::max<int64_t>(256 * P.groups, 1));
  e = hipMalloc(&P.col, cbytes);
  if (e != hipSuccess) return fail(e);
  if (P.ns)
    hipLaunchKernelGGL((k_sell_fill<float, float>), dim3(slice_grid(P.ns)), dim3(256), 0, st, n, P.ns, P.gp, rowptr, colind,
                       static_cast<const float*>(nullptr), P.col_bits == 32 ? static_cast<int32_t*>(P.col) : nullptr,
                       P.col_bits == 16 ? static_cast<int16_t*>(P.col) : nullptr, static_cast<float*>(nullptr));
  e = hipGetLastError();
  if (e != hipSuccess) return fail(e);
  *out = P;
  return LSPCG_OK;
}

int sell_fill_values(const SellPattern& P, const int32_t* colind, const void* src, int src_dtype, int dst_dtype,
                     hipStream_t st, void** out) {
  const size_t es = dst_dtype == LSPCG_F32 ? 4 : 8;
  void* v = *out;  // an existing array of this pattern and dtype is refilled in place
  const bool mine = v == nullptr;
  if (!v) LSPCG_HIP(hipMalloc(&v, es * std::max<int64_t>(P.slots(), 1)));
  const dim3 g(slice_grid(P.ns)), b(256);
  if (P.ns && P.jagged()) {
    int16_t* nc = nullptr;
    if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F64)
      hipLaunchKernelGGL((k_jag_fill<double, double>), g, b, 0, st, P.n, P.ns, P.gp, P.jc, P.lmap, P.rowptr, colind,
                         static_cast<const double*>(src), nc, static_cast<double*>(v));
    else if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_jag_fill<double, float>), g, b, 0, st, P.n, P.ns, P.gp, P.jc, P.lmap, P.rowptr, colind,
                         static_cast<const double*>(src), nc, static_cast<float*>(v));
    else if (src_dtype == LSPCG_F32 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_jag_fill<float, float>), g, b, 0, st, P.n, P.ns, P.gp, P.jc, P.lmap, P.rowptr, colind,
                         static_cast<const float*>(src), nc, static_cast<float*>(v));
    else
      hipLaunchKernelGGL((k_jag_fill<float, double>), g, b, 0, st, P.n, P.ns, P.gp, P.jc, P.lmap, P.rowptr, colind,
                         static_cast<const float*>(src), nc, static_cast<double*>(v));
  } else if (P.ns && P.col_bits == 1) {
    const auto* m = static_cast<const uint16_t*>(P.col);
    if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F64)
      hipLaunchKernelGGL((k_sdia_fill<double, double>), g, b, 0, st, P.n, P.ns, P.gp, m, P.rowptr,
                         static_cast<const double*>(src), static_cast<double*>(v));
    else if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_sdia_fill<double, float>), g, b, 0, st, P.n, P.ns, P.gp, m, P.rowptr,
                         static_cast<const double*>(src), static_cast<float*>(v));
    else if (src_dtype == LSPCG_F32 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_sdia_fill<float, float>), g, b, 0, st, P.n, P.ns, P.gp, m, P.rowptr,
                         static_cast<const float*>(src), static_cast<float*>(v));
    else
      hipLaunchKernelGGL((k_sdia_fill<float, double>), g, b, 0, st, P.n, P.ns, P.gp, m, P.rowptr,
                         static_cast<const float*>(src), static_cast<double*>(v));
  } else if (P.ns) {
    if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F64)
      hipLaunchKernelGGL((k_sell_fill<double, double>), g, b, 0, st, P.n, P.ns, P.gp, P.rowptr, colind,
                         static_cast<const double*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr), static_cast<double*>(v));
    else if (src_dtype == LSPCG_F64 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_sell_fill<double, float>), g, b, 0, st, P.n, P.ns, P.gp, P.rowptr, colind,
                         static_cast<const double*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr), static_cast<float*>(v));
    else if (src_dtype == LSPCG_F32 && dst_dtype == LSPCG_F32)
      hipLaunchKernelGGL((k_sell_fill<float, float>), g, b, 0, st, P.n, P.ns, P.gp, P.rowptr, colind,
                         static_cast<const float*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr), static_cast<float*>(v));
    else
      hipLaunchKernelGGL((k_sell_fill<float, double>), g, b, 0, st, P.n, P.ns, P.gp, P.rowptr, colind,
                         static_cast<const float*>(src), static_cast<int32_t*>(nullptr), static_cast<int16_t*>(nullptr), static_cast<double*>(v));
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    if (mine) (void)hipFree(v);
    set_error(std::string("sell_fill_values: ") + hipGetErrorString(e));
    return LSPCG_ERR_HIP;
  }
  *out = v;
  return LSPCG_OK;
}


}  // namespace lspcg
