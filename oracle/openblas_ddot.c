/* CPU restatement of the dot product the reference's recorded trajectories used -- TEST
 * INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline).
 *
 * The reference's PCG restatement (neural_cg/utils/validate.py:163-341) calls scipy's cg, whose
 * dots and norms (scipy 1.15 iterative.py:398-418: np.dot, np.linalg.norm -> x.dot(x)) are
 * numpy's cblas_ddot.  numpy 2.2.6 here bundles OpenBLAS 0.3.29 (libscipy_openblas64_, pthreads,
 * core "SkylakeX"; threadpoolctl reports it), a third-party dependency absent from
 * /root/reference.  Its published algorithm (kernel/x86_64/ddot.c + ddot_microk_skylakex-2.c +
 * driver/others/blas_l1_thread.c), restated:
 *
 *   ddot(n, x, y):  n <= 10000 or 1 thread -> dot_compute(n, x, y)
 *                   else split [0, n) into `threads` consecutive chunks, chunk t of width
 *                   ceil(remaining / (threads - t)); dot_compute per chunk; sum the chunk
 *                   results in chunk order starting from 0.0
 *   dot_compute(n): n1 = n & -16; kernel_8(n1) then dot = fma(x[i], y[i], dot) for i in [n1, n)
 *   kernel_8(n1):   32 accumulators (4 x 512-bit) over the n1 & -32 prefix, element i FMA'd into
 *                   accumulator i % 32; fold each 8-wide accumulator to 4 lanes (lo + hi);
 *                   one 16-element step on 4 x 4 lanes for the remaining [n32, n1); then
 *                   s = ((a0 + a1) + a2) + a3 lane-wise, h = (s0 + s2, s1 + s3), dot = h0 + h1.
 *
 * Verified bit for bit against np.dot in this container for n = 1 .. 70,000 at 1, 2, 3, 4 and
 * 8 OpenBLAS threads (tests/test_oracle_golden.py::test_openblas_ddot_restatement).  Built with
 * -ffp-contract=off: the only fused operations are the explicit fma() calls.
 */
#include <math.h>
#include <stdint.h>

static double dot_compute(int64_t n, const double* x, const double* y) {
  const int64_t n1 = n & -16;
  const int64_t n32 = n1 & ~(int64_t)31;
  double acc[32];
  for (int k = 0; k < 32; ++k) acc[k] = 0.0;
  for (int64_t i = 0; i < n32; i += 32)
    for (int k = 0; k < 32; ++k) acc[k] = fma(x[i + k], y[i + k], acc[k]);
  double a[4][4];
  for (int v = 0; v < 4; ++v)
    for (int j = 0; j < 4; ++j) a[v][j] = acc[8 * v + j] + acc[8 * v + 4 + j];
  for (int64_t i = n32; i < n1; i += 16)
    for (int v = 0; v < 4; ++v)
      for (int j = 0; j < 4; ++j) a[v][j] = fma(x[i + 4 * v + j], y[i + 4 * v + j], a[v][j]);
  double s[4];
  for (int j = 0; j < 4; ++j) s[j] = ((a[0][j] + a[1][j]) + a[2][j]) + a[3][j];
  double dot = (s[0] + s[2]) + (s[1] + s[3]);
  for (int64_t i = n1; i < n; ++i) dot = fma(y[i], x[i], dot);
  return dot;
}

double lspcg_oracle_openblas_ddot(int64_t n, const double* x, const double* y, int threads) {
  if (n <= 0) return 0.0;
  if (n <= 10000 || threads <= 1) return dot_compute(n, x, y);
  double dot = 0.0;
  int64_t m = n, start = 0;
  for (int t = 0; t < threads && m > 0; ++t) {
    int64_t w = (m + (threads - t) - 1) / (threads - t);
    m -= w;
    if (m < 0) w += m;
    dot = dot + dot_compute(w, x + start, y + start);
    start += w;
  }
  return dot;
}
