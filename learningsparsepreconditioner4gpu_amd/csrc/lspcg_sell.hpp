// Sliced-ELL (SELL-64) iteration view of a scalar CSR matrix, for the PCG loop.
//
// Why (DESIGN.md "SpMV formats"): in the staged CSR kernel one gather instruction covers the
// entries of ~17 consecutive rows at ~4 different stencil positions (~30 distinct cache lines),
// and every row tile pays a dependent rowptr load, an LDS round trip and two barriers.  In
// SELL-64 a wave owns a slice of 64 consecutive rows; entry k of row r is stored at
//     256*(gp[slice] + k/4) + 4*r + k%4
// so lane r loads 4 consecutive entries of ITS row with one 16-B load (values) and one 16-B
// load (columns), and one gather instruction reads x at the same in-row position of 64
// consecutive rows (~4 cache lines on banded FEM matrices).  The row sum stays in a register
// and is accumulated in the row's index order -- scipy's csr_matvec order, so results are
// bit-identical to the CSR kernels.  Padding slots (k >= row length) are skipped by a
// predicate, never added (0*inf and -0.0 + 0.0 must not leak into the sum).
#pragma once

#include "lspcg_internal.hpp"
#include "lspcg_spmv.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace lspcg {

constexpr int kSellC = 64;  // rows per slice = one wave64

// Column storage: 16-bit offsets from the slice's first row when every |col - 64*slice| <=
// 32767 (banded FEM orderings: 6 instead of 8 B per fp32-valued entry), padding marked by the
// sentinel kSellPad16; otherwise int32 columns with padding sentinel -1.  Either way the kernel
// needs no row lengths (no dependent rowptr load before the entry loads).
constexpr int16_t kSellPad16 = -32768;

// Slice-diagonal layout ("SELL-DIA", col_bits == 1; structured-grid orderings: the Kuhn-tet
// stencil has 15 distinct row-relative offsets col - row per 64-row slice, the 2-D 5-point stencil
// 5, boundary rows use subsets).  Each slice s keeps its D_s <= 16 distinct offsets, ascending, in
// dict[16 s + j] and stores its rows' values slot-major, ONE slot per dictionary entry:
//     vals[64 (gp[s] + j) + lane]   (row 64 s + lane, column row + dict[16 s + j]),
// with bit j of mask[64 s + lane] set where the row has that entry (absent entries: value 0, bit
// clear, never added).  Rows are sorted, so slot order = the row's column order = scipy's sum
// order.  No column storage at all: the offset of slot j is wave-uniform (a scalar register), the
// x / r / t / p "gather" of slot j is one contiguous 64-entry load, and a row costs D_s values +
// 2 bytes of mask (Kuhn: 15 slots per row where SELL-64's 4-entry groups store 16).
constexpr int kSdiaMax = 16;       // slots (distinct offsets) per slice
// column-storage choices for sell_build_pattern (bit mask); int32 columns are always possible
constexpr int kSellCol16 = 1;
constexpr int kSellColDia = 2;
constexpr int kSellColCode = 4;
// Coded SELL-64 ("SELL-64C", col_bits == 8; unstructured orderings after a bandwidth-reducing
// permutation, where a slice's rows share few row-relative offsets col - row but more than SELL-DIA's
// 16): SELL-64's slot layout and values, with ONE byte per slot -- the rank of the slot's offset in
// its slice's ascending dictionary dict[64 s + j] (<= 64 entries, kSellCodePad for padding) --
// instead of a 16-bit column offset.  The lane's dictionary entry sits in one register and a code
// is decoded with one ds_bpermute (no LDS allocation).  Slices with more than 64 distinct offsets
// keep 16-bit offsets in a second array: rgp[s] = their first group there (-1: coded slice).
constexpr int kSellCodeMax = 64;
constexpr uint8_t kSellCodePad = 0xff;
// Jagged SELL-64 ("SELL-64J", col_bits == kSellJag: 16-bit offsets; unstructured meshes, whose rows
// in one 64-row slice range from 4 to ~35 entries, so SELL-64's 64 x longest-row slots pad 1.6x).
// Inside each slice the LANES are sorted by descending row length (ties by row): lane l owns row
// 64 s + lmap[64 s + l], and group q (entries 4q .. 4q+3) holds only the cnt_q = jc[16 s + q] lanes
// whose rows reach it, a prefix of the lanes -- stored densely:
//     entry k of lane l at  gp[s] + 4 (cnt_0 + ... + cnt_{q-1}) + 4 l + k % 4,   q = k / 4, l < cnt_q,
// with gp[s] the slice's first ELEMENT.  Padding is only the row's last group (16.1 -> 17.6 entries
// per row on the 1 M Delaunay mesh, vs 26.1 for SELL-64).  Rows move only inside their slice, so x
// gathers and y / r / p accesses hit the same cache lines as before, and slot k is still entry k of
// its row: scipy's sum order, the same bits.  Rows of more than 64 entries (16 groups) keep SELL-64.
constexpr int kSellJag = 17;
constexpr int kSellJagMaxG = 16;   // groups per slice (jc bytes per slice)
constexpr int kSellColJag = 8;     // sell_build_pattern: jagged 16-bit layout allowed
constexpr double kSellJagPad = 1.15;  // taken when SELL-64 stores more than this x nnz slots
// x-staged SELL-64J ("SELL-64X", col_bits == kSellJagX): the jagged layout whose 16-bit column words
// are positions in an LDS copy of the vector blocks the row tile (4 slices, 256 rows) touches.  An
// unstructured mesh's 64-row slice gathers ~14 distinct 128-B lines per 64-lane gather (Kuhn grid: 4),
// mostly L1 misses (a slice's x footprint is ~11 KB, 24 resident slices per CU), and those gathers
// cost 40 % of the jagged SpMV (tools/jag_probe.py: 43.8 vs 26.8 us with contiguous gathers, delaunay1m).
// Here a tile's distinct 16-element x blocks (xl[xlp[t] .. xlp[t+1]), ascending; ~170 on delaunay1m)
// are loaded ONCE per tile with 16-B loads into LDS (barrier), and entry k's word is
// slot * 16 + col % 16 with slot the block's rank in the list: the gathers become LDS reads of the
// same values, so the bits are unchanged.  kx = the largest list (LDS: kx * 16 * sizeof(x) per
// workgroup); patterns whose tiles touch more than kSellXMax blocks keep SELL-64J.
constexpr int kSellJagX = 18;
constexpr int kSellColXs = 16;  // sell_build_pattern: the x-staged layout allowed (GatherVec only)
constexpr int kSellXMax = 256;  // blocks per tile (32 KB of fp64)
constexpr int kSellXBlk = 16;   // vector entries per staged block
// smallest pattern staged: below it the per-tile staging latency and barriers cost more than the
// gathers they replace (us per iteration, SELL-64X vs SELL-64J: delaunay1m 127.0 vs 134.9, delaunay64k
// 31.5 vs 28.6, bunny 18.8 vs 16.9; profiles/r6_sellx_probe.jsonl)
constexpr int64_t kSellXMinN = 262144;

// Pattern shared by every matrix with the same CSR (rowptr, colind).
//
// Block variant (bs == 3, "BSELL-64"; BSR 3x3 matrices): a wave owns 64
// consecutive BLOCK rows; slot q of block row I = 64 s + lane holds ONE column index (int32 block
// column or 16-bit offset from 64 s) and the block's 9 values (v = 3 a + c) in 16-byte lane
// chunks: planes 0-7 in groups of W = 16 / sizeof(value) (fp64 pairs, fp32 quads), plane 8 alone,
//     col[64 (gp[s] + q) + lane],
//     vals[576 (gp[s] + q) + 64 W (v / W) + W lane + v % W]   (v < 8),  vals[576 (gp[s] + q) + 512 + lane]
// so a slot is 8 / W + 1 value loads (16-B per lane, 1 KiB per wave instruction) + 1 column load
// and a block costs 9 values + 1 column instead of 9 scalar (value, column) pairs; x is gathered
// once per block (3 consecutive entries) for the lane's 3 scalar rows.  Row 3I + a sums its blocks in column
// order and inside a block c = 0, 1, 2: the order of the reference's expanded scalar CSR
// (validate.py:51), in-block zeros kept (adding an exact 0*x changes no finite sum).
struct SellPattern {
  int64_t n = 0;                   // scalar rows
  int64_t nb = 0;                  // rows of the pattern: scalar rows (bs 1) or block rows (bs 3)
  int bs = 1;
  int64_t ns = 0;                  // slices
  int64_t groups = 0;              // gp[ns]: 4-entry groups (bs 1) / block slots (bs 3) / DIA slots per lane, summed
  int32_t* gp = nullptr;           // [ns+1] exclusive prefix of per-slice groups (slots) per row
  void* col = nullptr;             // [256*groups] (bs 1) / [64*groups] (bs 3) int32 columns or int16 offsets;
                                   // SELL-DIA (col_bits 1): [64*ns] uint16 row masks
  int col_bits = 32;
  int32_t* dict = nullptr;         // SELL-DIA: [16*ns] ascending row-relative offsets per slice;
                                   // SELL-64C (col_bits 8): [64*ns], col = [256*groups] uint8 codes
  int32_t* rgp = nullptr;          // SELL-64C: [ns] group start in col2 of a slice kept uncoded, or -1
  int16_t* col2 = nullptr;         // SELL-64C: 16-bit offsets of the uncoded slices
  uint8_t* lmap = nullptr;         // SELL-64J: [64*ns] row (within the slice) of each lane
  uint8_t* jc = nullptr;           // SELL-64J: [16*ns] lanes per group (non-increasing, 0 past the last)
  int64_t elems = 0;               // SELL-64J: stored entries (gp is an element prefix, not a group prefix)
  int32_t* xlp = nullptr;          // SELL-64X: [ntiles+1] block-list prefix per 256-row tile
  int32_t* xl = nullptr;           // SELL-64X: the tiles' ascending x-block lists
  int kx = 0;                      // SELL-64X: the longest list
  int64_t xn = 0;                  // SELL-64X: vector entries read (largest column + 1; > n for dist_pcg's halo)
  const int32_t* rowptr = nullptr; // CSR row pointer (row lengths), not owned
  // the jagged element layout (SELL-64J / SELL-64X): gp is an element prefix
  bool jagged() const { return col_bits == kSellJag || col_bits == kSellJagX; }
  // entries of a value array of this pattern (sell_fill_values allocates this many)
  int64_t slots() const {
    if (bs == 3) return int64_t(576) * groups;  // BSELL-64 / BSELL-DIA: 9 values per block slot
    return jagged() ? elems : (col_bits == 1 ? int64_t(64) : int64_t(256)) * groups;
  }
  void release() {
    (void)hipFree(gp);
    (void)hipFree(col);
    (void)hipFree(dict);
    (void)hipFree(rgp);
    (void)hipFree(col2);
    (void)hipFree(lmap);
    (void)hipFree(jc);
    (void)hipFree(xlp);
    (void)hipFree(xl);
    xlp = nullptr;
    xl = nullptr;
    gp = nullptr;
    col = nullptr;
    dict = nullptr;
    rgp = nullptr;
    col2 = nullptr;
    lmap = nullptr;
    jc = nullptr;
  }
};

template <typename VT, typename CT>
struct SellArgs {
  int64_t n;
  int64_t ns;
  const int32_t* gp;
  const CT* col;
  const int32_t* rowptr;
  const VT* vals;
  const int32_t* dict = nullptr;  // SELL-64C (CT = uint8_t): see kSellCodeMax
  const int32_t* rgp = nullptr;
  const int16_t* col2 = nullptr;
  const uint8_t* lmap = nullptr;  // SELL-64J: see kSellJag
  const uint8_t* jc = nullptr;
  const int32_t* xlp = nullptr;   // SELL-64X: see kSellJagX
  const int32_t* xl = nullptr;
  int64_t xn = 0;
};

template <typename VT>
struct SdiaArgs {
  int64_t n;
  int64_t ns;
  const int32_t* gp;
  const uint16_t* mask;
  const int32_t* dict;
  const VT* vals;
};

// ---- the SpMV ----------------------------------------------------------------
template <typename VT>
struct Vec4Ld;
template <>
struct Vec4Ld<float> {
  __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
    const f32x4 a = *(const __attribute__((address_space(1))) f32x4*)(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};
template <>
struct Vec4Ld<double> {
  __device__ static __forceinline__ void load(const double* p, double (&v)[4]) {
    const auto* q = (const __attribute__((address_space(1))) f64x2*)(p);
    const f64x2 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
};

using i16x4 = short __attribute__((ext_vector_type(4)));
using xs_u4 = unsigned __attribute__((ext_vector_type(4)));  // 16-B staging part (SELL-64X)

// Epilogues with a PREFETCH member (a device pointer) read one own-row value in row(); the SELL
// kernel loads it before the row's slot loop so it does not add a memory latency after the
// gathers, and passes it to row_pf() (latency-bound mid-size systems).
template <class E, class = void>
struct epi_prefetch : std::false_type {};
template <class E>
struct epi_prefetch<E, std::void_t<decltype(E::PREFETCH)>> : std::bool_constant<E::PREFETCH> {};

// 256-thread workgroups = 4 slices = one 256-row tile (the same row tiles as k_spmv, so the
// prologue / epilogue functors and the dot-product reduction are shared).  QB groups of 4
// entries are loaded per lane before the first gather (branch-free: the group index is
// clamped, the surplus is masked at the add).
// MINW: minimum workgroups per CU the register allocation must allow (6 x 256 threads for the
// compact-value PCG kernels, whose reducing launches use a resident 6-per-CU grid; 1 for fp64
// values and the double-gather fused epilogues, which need more registers than 6/CU leaves).
template <typename T, typename VT, typename CT, int QB, int TH, int MINW, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(TH, MINW) k_spmv_sell(SellArgs<VT, CT> a, Pro pro, Gx gx, Epi epi) {
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  constexpr bool C16 = std::is_same<CT, int16_t>::value;
  constexpr bool C8 = std::is_same<CT, uint8_t>::value;  // SELL-64C
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t ntiles = (a.n + TH - 1) / TH;
  // the first tile's slice range is loaded before the prologue's state read, so the two
  // dependent-free loads share one memory latency (the state line was written by another CU)
  int32_t gb[2] = {0, 0};
  [[maybe_unused]] int32_t rg = -1, dl = 0;  // SELL-64C: uncoded group start, this lane's dictionary entry
  if (int64_t(blockIdx.x) * (TH / 64) + w < a.ns) {
    gb[0] = a.gp[int64_t(blockIdx.x) * (TH / 64) + w];
    gb[1] = a.gp[int64_t(blockIdx.x) * (TH / 64) + w + 1];
    if constexpr (C8) {
      rg = a.rgp[int64_t(blockIdx.x) * (TH / 64) + w];
      dl = a.dict[kSellCodeMax * (int64_t(blockIdx.x) * (TH / 64) + w) + lane];
    }
  }
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * (TH / 64) + w;
    const int64_t i = tile * TH + threadIdx.x;
    if (s < a.ns) {  // wave-uniform
      if (tile != int64_t(blockIdx.x)) {
        gb[0] = a.gp[s];
        gb[1] = a.gp[s + 1];
        if constexpr (C8) {
          rg = a.rgp[s];
          dl = a.dict[kSellCodeMax * s + lane];
        }
      }
      const int32_t g0 = gb[0];
      const int nq = gb[1] - g0;
      const int32_t base = int32_t(s * kSellC);
      const VT* vp = a.vals + 256 * int64_t(g0) + 4 * lane;
      const CT* cp = a.col + 256 * int64_t(g0) + 4 * lane;
      [[maybe_unused]] const int16_t* cp2 = C8 ? a.col2 + 256 * int64_t(rg) + 4 * lane : nullptr;
      T acc = T(0);
      T pf = T(0);
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) pf = epi.prefetch(i);
      }
      for (int q0 = 0; q0 < nq; q0 += QB) {
        VT v[QB][4];
        int c[QB][4];
        bool m[QB][4];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int q = min(q0 + u, nq - 1);
          Vec4Ld<VT>::load(vp + 256 * q, v[u]);
          if constexpr (C8) {
            if (rg < 0) {  // wave-uniform: a coded slice
              const unsigned cc = *(const __attribute__((address_space(1))) unsigned*)(cp + 256 * q);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const unsigned b = (cc >> (8 * j)) & 0xffu;
                const int off = __builtin_amdgcn_ds_bpermute(int((b & 63u) << 2), dl);
                m[u][j] = (b != kSellCodePad) && (q0 + u < nq);
                c[u][j] = b != kSellCodePad ? base + lane + off : base;  // padding gathers row base
              }
            } else {
              const i16x4 cc = *(const __attribute__((address_space(1))) i16x4*)(cp2 + 256 * q);
              const int o[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                m[u][j] = (o[j] != kSellPad16) && (q0 + u < nq);
                c[u][j] = base + (o[j] != kSellPad16 ? o[j] : 0);
              }
            }
          } else if constexpr (C16) {
            const i16x4 cc = *(const __attribute__((address_space(1))) i16x4*)(cp + 256 * q);
            const int o[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              m[u][j] = (o[j] != kSellPad16) && (q0 + u < nq);
              c[u][j] = base + (o[j] != kSellPad16 ? o[j] : 0);
            }
          } else {
            const i32x4 cc = *(const __attribute__((address_space(1))) i32x4*)(cp + 256 * q);
            const int o[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              m[u][j] = (o[j] >= 0) && (q0 + u < nq);
              c[u][j] = o[j] >= 0 ? o[j] : base;
            }
          }
        }
        T xv[QB][4];
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[u][j] = gx(c[u][j]);
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (m[u][j]) acc = acc + T(v[u][j]) * xv[u][j];
      }
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) epi.row_pf(i, acc, d, pf);
      } else {
        if (i < a.n) epi.row(i, acc, d);
      }
    }
  }
  finish_epi_dots<Epi>(d, epi);
}

// SELL-64J SpMV (layout: see kSellJag): one wave = one 64-row slice; lane l sums row 64 s + lmap[l].
// The slice's metadata is its first element gp[s], the 16 group counts (two 8-byte scalar loads)
// and the lane's row byte, loaded in one batch (the first tile's before the prologue's state read).
// Group q's loads are issued only by its cnt_q active lanes (a prefix of the wave): a shorter row's
// lane neither loads nor adds past its last group.  The counts are consumed from a 128-bit scalar
// shift register, QB groups per batch, every load of a batch before the first add.
// XS (SELL-64X, kSellJagX): the column words index the tile's LDS copy of its x blocks (dynamic
// shared memory, kx * 16 entries), staged by the whole workgroup between two barriers per tile.
template <typename T, typename VT, int QB, int TH, int MINW, bool XS, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(TH, MINW) k_spmv_sellj(SellArgs<VT, int16_t> a, Pro pro, Gx gx, Epi epi) {
  static_assert(QB >= 1 && QB <= 4, "QB groups per batch");
  static_assert(!XS || std::is_same<Gx, GatherVec<T>>::value, "SELL-64X stages a plain vector");
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  [[maybe_unused]] extern __shared__ __attribute__((aligned(16))) unsigned char sx_raw[];
  [[maybe_unused]] T* sx = reinterpret_cast<T*>(sx_raw);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t ntiles = (a.n + TH - 1) / TH;
  int32_t e0 = 0;
  uint64_t c0 = 0, c1 = 0;
  int rl = 0;
  auto meta = [&](int64_t sl) {
    e0 = a.gp[sl];
    const uint64_t* cp = reinterpret_cast<const uint64_t*>(a.jc + kSellJagMaxG * sl);
    c0 = cp[0];
    c1 = cp[1];
    rl = a.lmap[kSellC * sl + lane];
  };
  // QB groups' loads (values, column words) of the lane's row, issued for the active lanes only;
  // advances the element offset and the count shift register
  struct Batch {
    VT v[QB][4];
    i16x4 cc[QB];
  };
  auto issue = [&](Batch& B, int32_t& eo, uint64_t& lo, uint64_t& hi) {
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int cq = int((lo >> (8 * u)) & 0xffu);
      B.cc[u] = i16x4{kSellPad16, kSellPad16, kSellPad16, kSellPad16};
      B.v[u][0] = B.v[u][1] = B.v[u][2] = B.v[u][3] = VT(0);
      if (lane < cq) {
        Vec4Ld<VT>::load(a.vals + int64_t(eo) + 4 * lane, B.v[u]);
        B.cc[u] = *(const __attribute__((address_space(1))) i16x4*)(a.col + int64_t(eo) + 4 * lane);
      }
      eo += 4 * cq;
    }
    lo = (lo >> (8 * QB)) | (hi << (64 - 8 * QB));
    hi >>= 8 * QB;
  };
  uint64_t lo = 0, hi = 0;
  int32_t eo = 0;
  Batch cur;
  {  // the first tile's metadata and first batch (matrix data only) before the prologue's state read
    const int64_t s = int64_t(blockIdx.x) * (TH / 64) + w;
    if (int64_t(blockIdx.x) < ntiles && s < a.ns) {
      meta(s);
      lo = c0;
      hi = c1;
      eo = e0;
      if (lo & 0xffu) issue(cur, eo, lo, hi);
    }
  }
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * (TH / 64) + w;
    const bool live = s < a.ns;  // wave-uniform
    if (live && tile != int64_t(blockIdx.x)) {  // the first batch's loads fly during the staging
      meta(s);
      lo = c0;
      hi = c1;
      eo = e0;
      if (lo & 0xffu) issue(cur, eo, lo, hi);
    }
    if constexpr (XS) {  // the tile's x blocks -> LDS (16-B loads; a block past n element by element)
      if (tile != int64_t(blockIdx.x)) __syncthreads();  // the previous tile's LDS reads are done
      const int32_t b0 = a.xlp[tile], nbk = a.xlp[tile + 1] - b0;
      constexpr int W = 16 / int(sizeof(T));   // entries per 16-B part
      constexpr int PPB = kSellXBlk / W;       // parts per block
      const T* xg = gx.x;
      for (int p = threadIdx.x; p < nbk * PPB; p += TH) {
        const int64_t e = int64_t(a.xl[b0 + p / PPB]) * kSellXBlk + (p % PPB) * W;
        T* dst = sx + (p / PPB) * kSellXBlk + (p % PPB) * W;
        if (e + W <= a.xn) {
          *reinterpret_cast<xs_u4*>(dst) = *(const __attribute__((address_space(1))) xs_u4*)(xg + e);
        } else {
#pragma unroll
          for (int k = 0; k < W; ++k) dst[k] = e + k < a.xn ? xg[e + k] : T(0);
        }
      }
      __syncthreads();
    }
    if (live) {
      const int32_t base = int32_t(s * kSellC);
      const int64_t i = int64_t(base) + rl;
      T acc = T(0);
      T pf = T(0);
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) pf = epi.prefetch(i);
      }
      bool have = (c0 & 0xffu) != 0;
      while (have) {  // wave-uniform: software-pipelined, the next batch's loads beside this one's gathers
        const bool more = (lo & 0xffu) != 0;
        Batch nxt;
        if (more) issue(nxt, eo, lo, hi);
        bool m[QB][4];
        T xv[QB][4];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int o[4] = {cur.cc[u].x, cur.cc[u].y, cur.cc[u].z, cur.cc[u].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            m[u][j] = o[j] != kSellPad16;
            if constexpr (XS) xv[u][j] = sx[m[u][j] ? o[j] : 0];
            else xv[u][j] = gx(base + (m[u][j] ? o[j] : 0));
          }
        }
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (m[u][j]) acc = acc + T(cur.v[u][j]) * xv[u][j];
        if (more) cur = nxt;
        have = more;
      }
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) epi.row_pf(i, acc, d, pf);
      } else {
        if (i < a.n) epi.row(i, acc, d);
      }
    }
  }
  finish_epi_dots<Epi>(d, epi);
}

// SELL-DIA SpMV (layout: see kSdiaMax): one wave = one 64-row slice of a 256-row tile, SB slots
// per batch, every load of a batch issued before the first add (value loads and vector loads are
// independent: the slot's offset is a scalar).  A slice's metadata -- its slot range (gp), its
// whole 16-entry offset dictionary (one scalar block load: entries past the slice's count are
// never used, masked lanes read x[base]) and its row masks -- is loaded in one batch, and the
// first tile's batch before the prologue's state read: one memory latency before the value /
// vector loads instead of three in a row (state, gp, dictionary).
template <typename T, typename VT, int SB, int TH, int MINW, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(TH, MINW) k_spmv_sdia(SdiaArgs<VT> a, Pro pro, Gx gx, Epi epi) {
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t ntiles = (a.n + TH - 1) / TH;
  int32_t g0 = 0, g1 = 0;
  unsigned msk = 0;
  int32_t dct[kSdiaMax];
  auto meta = [&](int64_t sl) {
    g0 = a.gp[sl];
    g1 = a.gp[sl + 1];
    msk = gld(a.mask + kSellC * sl + lane);
    const int32_t* dp = a.dict + kSdiaMax * sl;
#pragma unroll
    for (int j = 0; j < kSdiaMax; ++j) dct[j] = dp[j];
  };
  {
    const int64_t s = int64_t(blockIdx.x) * (TH / 64) + w;
    if (int64_t(blockIdx.x) < ntiles && s < a.ns) meta(s);
  }
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * (TH / 64) + w;
    const int64_t i = tile * TH + threadIdx.x;
    if (s < a.ns) {  // wave-uniform
      if (tile != int64_t(blockIdx.x)) meta(s);
      const int nd = g1 - g0;
      const int32_t base = int32_t(s * kSellC);
      const int32_t row = base + lane;
      T acc = T(0);
      T pf = T(0);
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) pf = epi.prefetch(i);
      }
#pragma unroll
      for (int j0 = 0; j0 < kSdiaMax; j0 += SB) {
        if (j0 >= nd) break;  // wave-uniform
        VT v[SB];
        T xv[SB];
        bool m[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const int j = j0 + u;
          m[u] = (j < nd) && ((msk >> j) & 1u);
          const int32_t c = m[u] ? row + dct[j] : base;
          v[u] = gld(a.vals + kSellC * int64_t(g0 + min(j, nd - 1)) + lane);
          xv[u] = gx(c);
        }
#pragma unroll
        for (int u = 0; u < SB; ++u)
          if (m[u]) acc = acc + T(v[u]) * xv[u];
      }
      if constexpr (epi_prefetch<Epi>::value) {
        if (i < a.n) epi.row_pf(i, acc, d, pf);
      } else {
        if (i < a.n) epi.row(i, acc, d);
      }
    }
  }
  finish_epi_dots<Epi>(d, epi);
}

// position of plane v of lane `lane` inside a BSELL-64 slot (see SellPattern)
template <typename VT>
__host__ __device__ constexpr int bsell_pos(int v, int lane) {
  constexpr int W = 16 / int(sizeof(VT));
  return v < 8 ? 64 * W * (v / W) + W * lane + v % W : 512 + lane;
}

// the 9 values of this lane's block in slot `slot` (576 values): 16-B loads
__device__ __forceinline__ void bsell_load_block(const double* slot, double (&v)[9]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f64x2 a = *(const __attribute__((address_space(1))) f64x2*)(slot + bsell_pos<double>(2 * k, lane));
    v[2 * k] = a.x;
    v[2 * k + 1] = a.y;
  }
  v[8] = gld(slot + bsell_pos<double>(8, lane));
}
__device__ __forceinline__ void bsell_load_block(const float* slot, float (&v)[9]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const f32x4 a = *(const __attribute__((address_space(1))) f32x4*)(slot + bsell_pos<float>(4 * k, lane));
    v[4 * k] = a.x;
    v[4 * k + 1] = a.y;
    v[4 * k + 2] = a.z;
    v[4 * k + 3] = a.w;
  }
  v[8] = gld(slot + bsell_pos<float>(8, lane));
}

// BSR 3x3 over the BSELL-64 layout (see SellPattern): one lane = one block row = 3 scalar rows,
// QB block slots loaded per batch before the first gather.
template <typename T, typename VT, typename CT, int QB, int TH, int MINW, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(TH, MINW) k_spmv_bsell3(SellArgs<VT, CT> a, Pro pro, Gx gx, Epi epi) {
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  constexpr bool C16 = sizeof(CT) == 2;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t nb = a.n / 3;
  const int64_t ntiles = (nb + TH - 1) / TH;
  int32_t gb[2] = {0, 0};  // first tile's slice range, loaded beside the prologue's state read
  if (int64_t(blockIdx.x) * (TH / 64) + w < a.ns) {
    gb[0] = a.gp[int64_t(blockIdx.x) * (TH / 64) + w];
    gb[1] = a.gp[int64_t(blockIdx.x) * (TH / 64) + w + 1];
  }
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * (TH / 64) + w;
    const int64_t I = tile * TH + threadIdx.x;
    if (s < a.ns) {  // wave-uniform
      if (tile != int64_t(blockIdx.x)) {
        gb[0] = a.gp[s];
        gb[1] = a.gp[s + 1];
      }
      const int32_t g0 = gb[0];
      const int nq = gb[1] - g0;
      const int32_t base = int32_t(s * kSellC);
      const VT* vp = a.vals + 576 * int64_t(g0);
      const CT* cp = a.col + 64 * int64_t(g0) + lane;
      T acc[3] = {T(0), T(0), T(0)};
      for (int q0 = 0; q0 < nq; q0 += QB) {
        VT v[QB][9];
        int c[QB];
        bool m[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int q = min(q0 + u, nq - 1);
          bsell_load_block(vp + 576 * q, v[u]);
          const int o = int(gld(cp + 64 * q));
          if constexpr (C16) {
            m[u] = (o != kSellPad16) && (q0 + u < nq);
            c[u] = base + (o != kSellPad16 ? o : 0);
          } else {
            m[u] = (o >= 0) && (q0 + u < nq);
            c[u] = o >= 0 ? o : base;
          }
        }
        T xv[QB][3];
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
          for (int cc = 0; cc < 3; ++cc) xv[u][cc] = gx(3 * int64_t(c[u]) + cc);
#pragma unroll
        for (int u = 0; u < QB; ++u)
          if (m[u]) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
              for (int cc = 0; cc < 3; ++cc) acc[r] = acc[r] + T(v[u][3 * r + cc]) * xv[u][cc];
          }
      }
      if (I < nb) {
#pragma unroll
        for (int r = 0; r < 3; ++r) epi.row(3 * I + r, acc[r], d);
      }
    }
  }
  finish_epi_dots<Epi>(d, epi);
}

// BSR 3x3 over the BSELL-DIA layout (SELL-DIA's slot dictionary on the block graph + BSELL-64's
// 9-value lane chunks): one lane = one block row = 3 scalar rows; slot j of the slice holds the
// block at block column I + dict[j] (mask bit j), so the x entries of a slot are three contiguous
// 64-block loads at a wave-uniform offset and no column is loaded at all.  SB slots per batch, all
// value and x loads of a batch issued before the first add; the slot order is the row's block
// column order, c = 0, 1, 2 inside a block: the expanded scalar CSR's summation order.
template <typename T, typename VT, int SB, int TH, int MINW, class Pro, class Gx, class Epi>
__global__ void __launch_bounds__(TH, MINW) k_spmv_bsdia3(SdiaArgs<VT> a, Pro pro, Gx gx, Epi epi) {
  constexpr int ND = Epi::NDOT > 0 ? Epi::NDOT : 1;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int64_t nb = a.n / 3;
  const int64_t ntiles = (nb + TH - 1) / TH;
  int32_t g0 = 0, g1 = 0;
  unsigned msk = 0;
  int32_t dct[kSdiaMax];
  auto meta = [&](int64_t sl) {
    g0 = a.gp[sl];
    g1 = a.gp[sl + 1];
    msk = gld(a.mask + kSellC * sl + lane);
    const int32_t* dp = a.dict + kSdiaMax * sl;
#pragma unroll
    for (int j = 0; j < kSdiaMax; ++j) dct[j] = dp[j];
  };
  {
    const int64_t s = int64_t(blockIdx.x) * (TH / 64) + w;
    if (int64_t(blockIdx.x) < ntiles && s < a.ns) meta(s);
  }
  if (pro.exit()) return;
  gx.prepare();
  epi.prepare();
  DD d[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = dd_zero();
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t s = tile * (TH / 64) + w;
    const int64_t I = tile * TH + threadIdx.x;
    if (s < a.ns) {  // wave-uniform
      if (tile != int64_t(blockIdx.x)) meta(s);
      const int nd = g1 - g0;
      const int32_t base = int32_t(s * kSellC);
      const int32_t brow = base + lane;
      T acc[3] = {T(0), T(0), T(0)};
#pragma unroll
      for (int j0 = 0; j0 < kSdiaMax; j0 += SB) {
        if (j0 >= nd) break;  // wave-uniform
        VT v[SB][9];
        T xv[SB][3];
        bool m[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const int j = j0 + u;
          m[u] = (j < nd) && ((msk >> j) & 1u);
          const int64_t c = 3 * int64_t(m[u] ? brow + dct[j] : base);
          bsell_load_block(a.vals + 576 * int64_t(g0 + min(j, nd - 1)), v[u]);
#pragma unroll
          for (int cc = 0; cc < 3; ++cc) xv[u][cc] = gx(c + cc);
        }
#pragma unroll
        for (int u = 0; u < SB; ++u)
          if (m[u]) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
              for (int cc = 0; cc < 3; ++cc) acc[r] = acc[r] + T(v[u][3 * r + cc]) * xv[u][cc];
          }
      }
      if (I < nb) {
#pragma unroll
        for (int r = 0; r < 3; ++r) epi.row(3 * I + r, acc[r], d);
      }
    }
  }
  finish_epi_dots<Epi>(d, epi);
}

// Reducing launches use a resident grid: 6 workgroups per CU (the compact-value kernels'
// __launch_bounds__ guarantee), i.e. 1536 on MI355X -- one wave of workgroups, each walking its
// row tiles, so no straggler round delays the ticket (8 per CU / 2048 measured the same; caps of
// 1024 / 1342 / 2013 / 4025 measured no better).  Capped by the solver's 4096
// partial slots.  Non-reducing launches take one workgroup per row tile.
inline int64_t sell_cap(bool reducing) {
  static const int64_t rcap = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return std::max<int64_t>(1, std::min<int64_t>(int64_t(6) * cus, 4096));
  }();
  return reducing ? rcap : int64_t(1) << 40;
}

// largest padded-slots / nnz ratio for which a SELL view is built (LSPCG_SELL_MAXPAD, read once)
inline double sell_max_pad() {
  static const double v = [] {
    const char* e = std::getenv("LSPCG_SELL_MAXPAD");
    return e ? std::atof(e) : 2.0;  // 2-D 5-point rows (5 -> 8 slots) still run faster as SELL
  }();
  return v;
}

// grid of a SELL launch (the solver sizes the split-reduction groups from it)
constexpr int kSellWG = 256;  // 4 slices per workgroup (512 / 1024 measured slower: DESIGN.md §5)
constexpr int kSdiaSB = 8;    // SELL-DIA slots per batch

inline int64_t sell_grid(const SellPattern& P, bool reducing) {
  return std::min<int64_t>((P.nb + kSellWG - 1) / kSellWG, sell_cap(reducing));
}

template <typename T, typename VT, typename CT, int TH, class Pro, class Gx, class Epi>
inline void launch_spmv_sell_th(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st,
                                bool one_tile_per_wg = false) {
  int64_t grid = (P.nb + TH - 1) / TH;  // row tiles: TH scalar rows (bs 1) or TH block rows (bs 3)
  // one_tile_per_wg (batched solves): workgroup b owns exactly row tile b, so its dot partial is
  // that tile's and its prologue may test the tile's own system
  if (!one_tile_per_wg) grid = std::min<int64_t>(grid, sell_cap(Epi::NDOT > 0));
  if (grid <= 0) return;
  SellArgs<VT, CT> a{P.n,      P.ns,  P.gp,  static_cast<const CT*>(P.col), P.rowptr, static_cast<const VT*>(vals),
                     P.dict, P.rgp, P.col2};
  // compact-value kernels: registers for 6 workgroups per CU (the resident reducing grid)
  constexpr int MINW = (sizeof(VT) == 4 && std::is_same<Gx, GatherVec<T>>::value) ? (TH <= 1536 ? 1536 / TH : 1) : 1;
  if constexpr (!std::is_same<CT, uint16_t>::value && !std::is_same<CT, uint8_t>::value) {  // BSELL-64: int16 / int32 columns
    if (P.bs == 3) {
      // 2 block slots (18 values, 6 gathers) per batch
      LSPCG_LAUNCH_SPMV((k_spmv_bsell3<T, VT, CT, 2, TH, MINW, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(TH), 0, st,
                         a, pro, gx, epi);
      return;
    }
  }
  // 2 groups of 4 entries per batch (tools/sell_sweep.py on kuhn101, dictionary columns, cold:
  // fp64 values 32.2 us vs 33.8 with 4 groups and 46.0 with 8; fp32 values 22.7 vs 24.1 / 37.0)
  constexpr int QB = 2;
  LSPCG_LAUNCH_SPMV((k_spmv_sell<T, VT, CT, QB, TH, MINW, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(TH), 0, st, a,
                     pro, gx, epi);
}

// SELL-DIA launch
template <typename T, typename VT, class Pro, class Gx, class Epi>
inline void launch_spmv_sdia(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st,
                             bool one_tile_per_wg = false) {
  int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  if (!one_tile_per_wg) grid = std::min<int64_t>(grid, sell_cap(Epi::NDOT > 0));
  if (grid <= 0) return;
  SdiaArgs<VT> a{P.n, P.ns, P.gp, static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals)};
  constexpr int MINW = (sizeof(VT) <= 4 && std::is_same<Gx, GatherVec<T>>::value) ? 1536 / kSellWG : 1;
  LSPCG_LAUNCH_SPMV((k_spmv_sdia<T, VT, kSdiaSB, kSellWG, MINW, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(kSellWG),
                     0, st, a, pro, gx, epi);
}

// BSELL-DIA launch: 256 block rows (4 slices) per row tile, as BSELL-64
#ifndef LSPCG_BSDIA_SB64
#define LSPCG_BSDIA_SB64 2
#endif
#ifndef LSPCG_BSDIA_SB32
#define LSPCG_BSDIA_SB32 2
#endif
// block slots per batch (2: 18 values, 6 x loads) by value size
template <typename VT>
constexpr int bsdia_sb() { return sizeof(VT) == 8 ? LSPCG_BSDIA_SB64 : LSPCG_BSDIA_SB32; }
template <typename T, typename VT, class Pro, class Gx, class Epi>
inline void launch_spmv_bsdia3(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st,
                               bool one_tile_per_wg = false) {
  int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  if (!one_tile_per_wg) grid = std::min<int64_t>(grid, sell_cap(Epi::NDOT > 0));
  if (grid <= 0) return;
  SdiaArgs<VT> a{P.n, P.ns, P.gp, static_cast<const uint16_t*>(P.col), P.dict, static_cast<const VT*>(vals)};
  constexpr int MINW = (sizeof(VT) == 4 && std::is_same<Gx, GatherVec<T>>::value) ? 1536 / kSellWG : 1;
  LSPCG_LAUNCH_SPMV((k_spmv_bsdia3<T, VT, bsdia_sb<VT>(), kSellWG, MINW, Pro, Gx, Epi>), dim3(unsigned(grid)),
                     dim3(kSellWG), 0, st, a, pro, gx, epi);
}

// SELL-64J / SELL-64X launch: 256-row tiles (4 slices), the SELL-64 grid rules
#ifndef LSPCG_JAG_QB
#define LSPCG_JAG_QB 2  // groups of 4 entries per batch
#endif
template <typename T, typename VT, class Pro, class Gx, class Epi>
inline void launch_spmv_sellj(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st,
                              bool one_tile_per_wg = false) {
  int64_t grid = (P.nb + kSellWG - 1) / kSellWG;
  if (!one_tile_per_wg) grid = std::min<int64_t>(grid, sell_cap(Epi::NDOT > 0));
  if (grid <= 0) return;
  SellArgs<VT, int16_t> a{P.n, P.ns, P.gp, static_cast<const int16_t*>(P.col), P.rowptr, static_cast<const VT*>(vals)};
  a.lmap = P.lmap;
  a.jc = P.jc;
  a.xlp = P.xlp;
  a.xl = P.xl;
  a.xn = P.xn;
  constexpr int MINW = (sizeof(VT) == 4 && std::is_same<Gx, GatherVec<T>>::value) ? 1536 / kSellWG : 1;
  if constexpr (std::is_same<Gx, GatherVec<T>>::value) {
    if (P.col_bits == kSellJagX) {
      const size_t lds = size_t(P.kx) * kSellXBlk * sizeof(T);
      LSPCG_LAUNCH_SPMV((k_spmv_sellj<T, VT, LSPCG_JAG_QB, kSellWG, MINW, true, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(kSellWG),
                         lds, st, a, pro, gx, epi);
      return;
    }
  }
  if (P.col_bits != kSellJag) return;  // (SELL-64X needs a plain vector gather: sell_build_pattern's callers)
  LSPCG_LAUNCH_SPMV((k_spmv_sellj<T, VT, LSPCG_JAG_QB, kSellWG, MINW, false, Pro, Gx, Epi>), dim3(unsigned(grid)), dim3(kSellWG),
                     0, st, a, pro, gx, epi);
}

template <typename T, typename VT, class Pro, class Gx, class Epi>
inline void launch_spmv_sell_cfg(const SellPattern& P, const void* vals, Gx gx, Pro pro, Epi epi, hipStream_t st,
                                 bool one_tile_per_wg = false) {
  if (P.jagged()) launch_spmv_sellj<T, VT>(P, vals, gx, pro, epi, st, one_tile_per_wg);
  else if (P.col_bits == 1 && P.bs == 3) launch_spmv_bsdia3<T, VT>(P, vals, gx, pro, epi, st, one_tile_per_wg);
  else if (P.col_bits == 1) launch_spmv_sdia<T, VT>(P, vals, gx, pro, epi, st, one_tile_per_wg);
  else if (P.col_bits == 16) launch_spmv_sell_th<T, VT, int16_t, kSellWG>(P, vals, gx, pro, epi, st, one_tile_per_wg);
  else if (P.col_bits == 8) launch_spmv_sell_th<T, VT, uint8_t, kSellWG>(P, vals, gx, pro, epi, st, one_tile_per_wg);
  else launch_spmv_sell_th<T, VT, int32_t, kSellWG>(P, vals, gx, pro, epi, st, one_tile_per_wg);
}

}  // namespace lspcg

// SELL copy attached to a matrix handle for the standalone SpMV (same values, same dtype)
// (reordered: the copy is of P A Pᵀ; lspcg_spmv gathers x into xs and the SpMV stores each row at
// its original place, EpiStorePerm; ys is unused)
struct SellCopy {
  lspcg::SellPattern P;
  void* vals = nullptr;
  lspcg::Reorder ro;
  lspcg_mat* Ap = nullptr;  // P A Pᵀ (owned), its rowptr is P.rowptr
  void* xs = nullptr;
  void* ys = nullptr;
  void release() {
    P.release();
    (void)hipFree(vals);
    vals = nullptr;
    ro.release();
    if (Ap) lspcg_mat_destroy(Ap);
    Ap = nullptr;
    (void)hipFree(xs);
    (void)hipFree(ys);
    xs = ys = nullptr;
  }
};

namespace lspcg {
// Host-side construction (lspcg_sell.hip), enqueued on `st`.
// Builds the SELL-64 pattern of a scalar CSR (n rows); fails with LSPCG_ERR_UNSUPPORTED when the
// padded size exceeds max_pad x nnz (irregular row lengths: the CSR kernel is used instead).
// cols (kSellCol16 | kSellColDia | kSellColCode): the column storages allowed besides int32; SELL-DIA
// is taken when every slice has <= 16 distinct offsets, every row is sorted and it stores no more
// slots than the 4-entry groups would, else (kSellColCode, 16-bit offsets fit, rows sorted) SELL-64C
// when at least half of the slots fall in slices of <= 64 distinct offsets, else 16-bit offsets
// when they fit.
int sell_build_pattern(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* colind, double max_pad,
                       int cols, hipStream_t st, SellPattern* out);
// Allocates and fills the SELL value array of a CSR with the same pattern (*out == nullptr), or
// refills *out in place (an array of this pattern and dst_dtype).  src_dtype / dst_dtype:
// LSPCG_F32 or LSPCG_F64 (fp64 -> fp32 only for exactly representable values).
int sell_fill_values(const SellPattern& P, const int32_t* colind, const void* src, int src_dtype, int dst_dtype,
                     hipStream_t st, void** out);
// BSELL-64 pattern of a BSR 3x3 (nb block rows, nnzb blocks, sorted block columns); the same
// padding rule on block slots (64 x groups <= max_pad x nnzb) and 16-bit block-column offsets.
// allow_dia: BSELL-DIA (col_bits 1) when every slice has <= 16 distinct block offsets and it
// stores at most 1/16 more block slots than BSELL-64 (env LSPCG_BSDIA=0 turns it off: bsdia_allowed()).
int bsell_build_pattern(int64_t nb, int64_t nnzb, const int32_t* rowptr, const int32_t* colind, double max_pad,
                        bool allow16, bool allow_dia, hipStream_t st, SellPattern* out);
// SELL-64C for the solver's views of >= LSPCG_SELLC_MIN_N rows (env LSPCG_SELLC=0 turns it off): the
// byte codes pay where the loop streams matrix bytes; below, the decode's ds_bpermute in the gathers'
// dependency chain costs more than the bytes save (us per iteration, SELL-64C vs 16-bit: bunny 6.3 k
// rows 17.4 vs 16.6, kuhn41rcm 69 k 28.6 vs 27.1, kuhn64rcm 262 k 37.7 vs 37.4, kuhn80rcm 512 k 53.0 vs
// 55.5, kuhn101rcm 1 M 86.7 vs 90.2)
inline bool sellc_allowed(int64_t n) {
  const char* e = std::getenv("LSPCG_SELLC");
  if (e && e[0] == '0') return false;
  const char* m = std::getenv("LSPCG_SELLC_MIN_N");
  return n >= (m ? std::atoll(m) : int64_t(400000));
}
inline bool bsdia_allowed() {
  const char* e = std::getenv("LSPCG_BSDIA");
  return !(e && e[0] == '0');
}
// its block values (16-B lane chunks) from the BSR's [nnzb][3][3] array
int bsell_fill_values(const SellPattern& P, const void* src, int src_dtype, int dst_dtype, hipStream_t st, void** out);
}  // namespace lspcg
