// Level-scheduled sparse factorizations / triangular solves shared by lspcg_factor.hip and the
// PCG solver (lspcg_pcg.hip).  See lspcg_factor.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "lspcg.h"

namespace lspcg {

// Rows grouped by dependency level: rows order[ptr[l] .. ptr[l+1]) form level l (ascending row
// index inside a level); hptr is the host copy of ptr used to size the per-level launches.
struct Levels {
  int nlev = 0;
  int32_t* ptr = nullptr;
  int32_t* order = nullptr;
  std::vector<int32_t> hptr;
  // sync-free solve (lspcg_factor.hip k_trsv_syncfree): `order` with every level padded to whole
  // wave64s (-1 = no row), so no wave holds two rows of which one waits for the other; npad
  // positions; head[0] = the launch's block dequeue counter, head[1] = timeout flag
  int32_t* pad = nullptr;
  int64_t npad = 0;
  unsigned* head = nullptr;
  // the triangular factor's column-scaled values sv_p = v_p / d_col and per row inv = 1 / d,
  // c = d inv (trsv_prepare: spsolve_triangular's scaling)
  void* sv = nullptr;
  void* inv = nullptr;
  void* c = nullptr;
  void release();
};

// lower: row i depends on the columns j < i of its row; upper: on the columns j > i.
int build_levels(lspcg_ctx* ctx, int64_t n, const int32_t* rp, const int32_t* ci, bool lower, Levels* out);
// scaled values of T for enqueue_trsv (after build_levels), enqueued on T's context stream
int trsv_prepare(const lspcg_mat* T, bool lower, Levels* lv);
// x = T⁻¹ b in scipy spsolve_triangular's arithmetic (lower: diagonal stored last in each row,
// upper: first); `done` (nullable) is the solver's device done flag -- every launch returns at
// once when it is set.  Counter reset + fill + one sync-free launch (rows wait for their
// dependencies' values) + the diagonal scaling.
int enqueue_trsv(const lspcg_mat* T, const Levels& lv, bool lower, const void* b, void* x, const int32_t* done,
                 hipStream_t st);
constexpr int kTrsvLaunches = 4;  // graph nodes one enqueue_trsv adds
// LSPCG_ERR_HIP (and clears the flag) when a sync-free solve on these levels timed out
int trsv_check_timeout(const Levels& lv, hipStream_t st);
int ic0_factor(const lspcg_mat* A, lspcg_mat** L);
int ainv0_factor(const lspcg_mat* A, lspcg_mat** L);

}  // namespace lspcg
