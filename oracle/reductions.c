/*
 * TEST INFRASTRUCTURE ONLY — CPU restatements of the float32 reductions the
 * reference's variant servers run, in their exact evaluation order.  Only
 * tests/ (and bench.py's cpu_baseline leg) load this, as the checker of the
 * device kernels in plato_amd/csrc/flat.hip; the product never does.
 *
 * Compiled with -ffp-contract=off: every fmaf() below is an explicit fused
 * multiply-add of the restated code, every other op is separately rounded.
 *
 * 1. FedAdp (examples/server_aggregation/fedadp/fedadp_server.py:95-99):
 *    np.inner / np.linalg.norm of float32 vectors = cblas_sdot of numpy's
 *    bundled OpenBLAS 0.3.29 (scipy-openblas64, DYNAMIC_ARCH), whose
 *    cblas_sdot jumps straight to the per-CPU kernel (no threading).  On
 *    AVX-512 hosts that is sdot_k_SKYLAKEX (read from its disassembly):
 *      - n1 = n & -32, n64 = n1 & -64;
 *      - 4 x 16-lane fp32 accumulators, acc[r][l] = fma(x[i+16r+l], y[..], acc)
 *        over the 64-element blocks below n64;
 *      - fold to 4 x 8 lanes: a[r][l] = acc[r][l] + acc[r][l+8];
 *      - the remaining 32-block (if any): a[r][l] = fma(x[i+8r+l], y, a);
 *      - s[l] = ((a[0][l] + a[1][l]) + a[2][l]) + a[3][l];
 *        h[l] = s[l] + s[l+4]; kern = (h0 + h1) + (h2 + h3)   (two hadds);
 *      - tail i in [n1, n): double t += (double)fp32(y[i] * x[i]);
 *      - result = (float)(t + (double)kern).
 *    np.linalg.norm(x) = np.sqrt(np.float32(sdot(x, x))).
 * 2. Port (examples/async/port/port_server.py:50): F.cosine_similarity(a, b,
 *    dim=0) of PyTorch 2.10 on the CPU (ATen Distance.cpp + reduce kernels):
 *      na = vector_norm(a): 8 fp32 lanes fma(v, v, acc) over n - n%8 elements
 *           (lane l takes i = l mod 8), lanes added in order, then the n%8
 *           tail: 4 separately rounded v*v added in order if 4+ remain, the
 *           rest fma'd; sqrtf — one pass, independent of the thread count;
 *      q[i] = (a[i] / max(na, eps)) * (b[i] / max(nb, eps));
 *      sum(q): TensorIterator two-pass reduction over T = torch.get_num_threads()
 *           OpenMP chunks of ceil(n / min(T, ceil(n / 32768))) elements
 *           (one pass if n < 32768 or T == 1), each chunk by SumKernel's
 *           cascade sum (Vectorized<float> width 8, 4 rows of ILP, 4 levels
 *           of 2^max(4, ceil_log2(rows)/4) rows), the T per-thread results
 *           (unused ones 0) summed by the same cascade.
 * Pinned by tests/test_reductions.py against torch / numpy on this host and
 * against the reference-generated fixtures (FedAdp adaptive weights, Port
 * similarities).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------ OpenBLAS */
float plato_oracle_sdot_skx(int64_t n, const float* x, const float* y) {
  double tail = 0.0, kern = 0.0;
  const int64_t n1 = n & -32;
  if (n1) {
    float a512[4][16];
    memset(a512, 0, sizeof a512);
    int64_t i = 0;
    const int64_t n64 = n1 & -64;
    for (; i < n64; i += 64)
      for (int r = 0; r < 4; ++r)
        for (int l = 0; l < 16; ++l) a512[r][l] = fmaf(x[i + 16 * r + l], y[i + 16 * r + l], a512[r][l]);
    float a[4][8];
    for (int r = 0; r < 4; ++r)
      for (int l = 0; l < 8; ++l) a[r][l] = a512[r][l] + a512[r][l + 8];
    for (; i < n1; i += 32)
      for (int r = 0; r < 4; ++r)
        for (int l = 0; l < 8; ++l) a[r][l] = fmaf(x[i + 8 * r + l], y[i + 8 * r + l], a[r][l]);
    float s[8], h[4];
    for (int l = 0; l < 8; ++l) s[l] = ((a[0][l] + a[1][l]) + a[2][l]) + a[3][l];
    for (int l = 0; l < 4; ++l) h[l] = s[l] + s[l + 4];
    kern = (double)((h[0] + h[1]) + (h[2] + h[3]));
  }
  for (int64_t i = n1; i < n; ++i) tail += (double)(y[i] * x[i]);
  return (float)(tail + kern);
}

/* --------------------------------------------------------------- torch */
float plato_oracle_torch_norm(const float* x, int64_t n) {
  float acc[8] = {0};
  const int64_t m = n - n % 8;
  for (int64_t d = 0; d < m; d += 8)
    for (int l = 0; l < 8; ++l) acc[l] = fmaf(x[d + l], x[d + l], acc[l]);
  float b = acc[0];
  for (int l = 1; l < 8; ++l) b = b + acc[l];
  /* the scalar tail loop `buffer[0] += v * v`, as the compiler emitted it:
   * while 4 or more remain, 4 products in one SSE multiply, then added in
   * order (separately rounded); the last 1-3 fused (vfmadd231ss) */
  int64_t d = m;
  for (; d + 4 <= n; d += 4)
    for (int j = 0; j < 4; ++j) {
      const float p = x[d + j] * x[d + j];
      b = b + p;
    }
  for (; d < n; ++d) b = fmaf(x[d], x[d], b);
  return sqrtf(b);
}

static int ceil_log2(int64_t x) {
  int r = 0;
  while (((int64_t)1 << r) < x) ++r;
  return r;
}

/* SumKernel multi_row_sum + row_sum over `rows` rows of 4 x W values
 * (W = 8 for the vectorised path, 1 for the scalar one); in[(i*4+k)*W + l]. */
static void cascade_rows(const float* in, int64_t size_ilp, int W, float ps[4][8]) {
  enum { LEVELS = 4 };
  int64_t level_power = ceil_log2(size_ilp) / LEVELS;
  if (level_power < 4) level_power = 4;
  const int64_t level_step = (int64_t)1 << level_power;
  const int64_t level_mask = level_step - 1;
  float acc[LEVELS][4][8];
  memset(acc, 0, sizeof acc);
  int64_t i = 0;
  for (; i + level_step <= size_ilp;) {
    for (int64_t j = 0; j < level_step; ++j, ++i)
      for (int k = 0; k < 4; ++k)
        for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
    for (int j = 1; j < LEVELS; ++j) {
      for (int k = 0; k < 4; ++k)
        for (int l = 0; l < W; ++l) {
          acc[j][k][l] += acc[j - 1][k][l];
          acc[j - 1][k][l] = 0;
        }
      if ((i & (level_mask << (j * level_power))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
  for (int j = 1; j < LEVELS; ++j)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < W; ++l) acc[0][k][l] += acc[j][k][l];
  for (int k = 0; k < 4; ++k)
    for (int l = 0; l < W; ++l) ps[k][l] = acc[0][k][l];
}

/* vectorized_inner_sum / scalar_inner_sum of one contiguous piece */
static float inner_sum(const float* in, int64_t n) {
  float ps[4][8];
  if (n >= 8) {
    const int64_t vec_size = n / 8;
    const int64_t size_ilp = vec_size / 4;
    cascade_rows(in, size_ilp, 8, ps);
    for (int64_t v = size_ilp * 4; v < vec_size; ++v)
      for (int l = 0; l < 8; ++l) ps[0][l] += in[v * 8 + l];
    for (int k = 1; k < 4; ++k)
      for (int l = 0; l < 8; ++l) ps[0][l] += ps[k][l];
    float final_acc = 0.f;
    for (int64_t k = vec_size * 8; k < n; ++k) final_acc += in[k];
    for (int l = 0; l < 8; ++l) final_acc += ps[0][l];
    return final_acc;
  }
  const int64_t size_ilp = n / 4;
  cascade_rows(in, size_ilp, 1, ps);
  for (int64_t v = size_ilp * 4; v < n; ++v) ps[0][0] += in[v];
  for (int k = 1; k < 4; ++k) ps[0][0] += ps[k][0];
  return ps[0][0];
}

float plato_oracle_torch_sum(const float* in, int64_t n, int threads) {
  const int64_t grain = 32768;
  if (n < grain || threads <= 1) return 0.f + inner_sum(in, n);
  int64_t nt = threads;
  const int64_t by_grain = (n + grain - 1) / grain;
  if (by_grain < nt) nt = by_grain;
  const int64_t chunk = (n + nt - 1) / nt;
  float buf[1024];
  if (threads > 1024) return NAN;
  for (int t = 0; t < threads; ++t) buf[t] = 0.f;
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t b = t * chunk;
    if (b >= n) break;
    const int64_t e = b + chunk < n ? b + chunk : n;
    buf[t] += inner_sum(in + b, e - b);
  }
  return 0.f + inner_sum(buf, threads);
}

/* F.cosine_similarity(a, b, dim=0); tmp: n floats of scratch */
float plato_oracle_torch_cosine(const float* a, const float* b, int64_t n, int threads, float eps, float* tmp) {
  float na = plato_oracle_torch_norm(a, n), nb = plato_oracle_torch_norm(b, n);
  if (na < eps) na = eps;
  if (nb < eps) nb = eps;
  for (int64_t i = 0; i < n; ++i) tmp[i] = (a[i] / na) * (b[i] / nb);
  return plato_oracle_torch_sum(tmp, n, threads);
}

/* ------------------------------------------------------------------ numpy */
/* 3. Polaris (examples/client_selection/polaris/polaris_server.py:78-81):
 *    np.sum(np.square(d)) of a float32 array = the ufunc reduction's inner
 *    loops over 8192-element buffer chunks, out += pairwise_sum(chunk) from
 *    0, with numpy's pairwise_sum (numpy/_core/src/umath/loops_utils.h). */
static float pairwise(const float* a, int64_t n) {
  if (n < 8) {
    float res = 0.f;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

float plato_oracle_np_sum(const float* a, int64_t n) {
  float out = 0.f;
  for (int64_t s = 0; s < n; s += 8192) out += pairwise(a + s, n - s < 8192 ? n - s : 8192);
  return out;
}
