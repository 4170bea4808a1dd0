// entrywise.hip — per-entry (per state_dict tensor) kernels for the FedAvg
// variants whose numbers depend on the tensor as well as the client
// (SURVEY.md §8(f) rank 2):
//   * entry_stats: per (client, entry) sums of d^2 and d*v in fp64 — FedAtt's
//     per-layer norms, FedAdp's inner products / norms, Polaris' conv norms;
//   * fedavg_entrywise: acc += fp32(d * W[entry][client]) with an fp32 post-op
//     (scale, additive noise, + baseline) — FedAtt's attentive aggregation and
//     FedAdp's global-gradient pass.
//
// Both walk a host-built chunk table (include/plato_agg.h plato_agg_chunk):
// one workgroup per chunk, so the entry — and with it every weight — is
// workgroup-uniform and read through the scalar cache, exactly like the
// client pointers.  Entries are packed back to back in the arena (not
// 4-aligned), so the first and last float4 group of a chunk are partial:
// elements outside [begin, end) are masked (no contribution, no store); the
// neighbouring chunk owns them.  Interior groups take the dwordx4 path.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>

#include "common.h"
#include "plato_agg.h"
#include "plato_agg_tune.h"

namespace {

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gf4;
typedef __attribute__((address_space(1))) f4 gf4w;

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

template <class T>
__device__ __forceinline__ T sld(const T* p, uint64_t i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

__device__ __forceinline__ f4 ld_nt(const float* p, uint64_t g) { return __builtin_nontemporal_load((gf4*)p + g); }
__device__ __forceinline__ f4 ld_c(const float* p, uint64_t g) { return *((gf4*)p + g); }
__device__ __forceinline__ void st_nt(float* p, uint64_t g, f4 v) { __builtin_nontemporal_store(v, (gf4w*)p + g); }

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

struct Chunk {
  uint32_t entry, begin, end;
};

__device__ __forceinline__ Chunk load_chunk(const plato_agg_chunk* t, uint32_t c, uint64_t n) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(t + c);
  Chunk ch{sld(p, 0), sld(p, 1), sld(p, 2)};
  // never trust the table past the arena (a bad table gives wrong sums, not a fault)
  if (ch.end > n) ch.end = uint32_t(n);
  if (ch.begin > ch.end) ch.begin = ch.end;
  return ch;
}

__device__ __forceinline__ float i64_delta(const int64_t* x, const int64_t* b, uint64_t e) {
  const int64_t xv = x[e];
  // torch's int64 subtraction wraps; the promotion to fp32 happens after
  const int64_t d = b ? (int64_t)((uint64_t)xv - (uint64_t)b[e]) : xv;
  return (float)d;
}

// ---------------------------------------------------------------------------
// entry_stats
// ---------------------------------------------------------------------------
// Workspace rows (each n_chunks doubles): [0, K) d.v, [K, 2K) d.d, 2K v.v.
constexpr int kSV = 4;  // float4 groups per lane per pass (chunk pass = 4096 floats)
constexpr int kSU = 4;  // clients per batch

struct StatArgs {
  const float* const* xf;
  const int64_t* const* xi;
  const float* base_f;
  const int64_t* base_i;
  const float* v_f;
  const float* v_if;
  const plato_agg_chunk* cf;
  const plato_agg_chunk* ci;
  double* ws;
  uint64_t n_f32, n_i64;
  uint32_t ncf, nci, nc;
  int K;
};

// Block-wide sum of NV per-lane values; thread 0..NV-1 get the totals in out.
template <int NV>
__device__ __forceinline__ void block_sums(double (&v)[NV], double (*red)[2 * kSU + 1], double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = wave_sum(v[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) red[wave][j] = v[j];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double t = 0.0;
    for (int w = 0; w < kWaves; ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// Accumulate into ws[row * nc + c]; the pass index makes the first write a store.
__device__ __forceinline__ void ws_acc(const StatArgs& a, uint64_t row, uint32_t c, double t, bool first) {
  double* p = a.ws + row * a.nc + c;
  *p = first ? t : *p + t;
}

__device__ __forceinline__ double masked_dot(f4 p, f4 q, const bool (&m)[4]) {
  double s = 0.0;
  if (m[0]) s += (double)p.x * q.x;
  if (m[1]) s += (double)p.y * q.y;
  if (m[2]) s += (double)p.z * q.z;
  if (m[3]) s += (double)p.w * q.w;
  return s;
}

// TAIL: the chunk reaches the arena's last, partial float4 group (scalar loads
// there); every other chunk loads whole groups unconditionally.
template <bool HAS_BASE, bool HAS_V, bool TAIL>
__device__ void stats_f32_chunk(const StatArgs& a, uint32_t c, const Chunk ch, double (*red)[2 * kSU + 1],
                                double* tot) {
  const uint64_t n4 = a.n_f32 / 4;  // groups with 4 in-range elements
  const uint64_t g0 = ch.begin / 4, g1 = (uint64_t(ch.end) + 3) / 4;
  const int K = a.K;
  constexpr uint64_t kPass = uint64_t(kBlock) * kSV;
  uint64_t gp = g0;
  bool first = true;
  do {
    // this lane's groups of the pass; clamp the address, mask the elements
    uint64_t g[kSV];
    bool m[kSV][4];
    bool vec[kSV];
    f4 b[kSV], v[kSV];
#pragma unroll
    for (int j = 0; j < kSV; ++j) {
      const uint64_t gg = gp + threadIdx.x + uint64_t(j) * kBlock;
      const bool in = gg < g1;
      g[j] = in ? gg : (g1 > g0 ? g1 - 1 : g0);
      vec[j] = !TAIL || g[j] < n4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t e = 4 * gg + q;
        m[j][q] = in && e >= ch.begin && e < ch.end;
      }
      b[j] = f4{0.f, 0.f, 0.f, 0.f};
      v[j] = f4{0.f, 0.f, 0.f, 0.f};
      if (vec[j]) {
        if (HAS_BASE) b[j] = ld_c(a.base_f, g[j]);
        if (HAS_V) v[j] = ld_c(a.v_f, g[j]);
      } else {
        // the arena's last, partial group: scalar loads of the in-range elements
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint64_t e = 4 * g[j] + q;
          if (e < a.n_f32) {
            if (HAS_BASE) b[j][q] = a.base_f[e];
            if (HAS_V) v[j][q] = a.v_f[e];
          }
        }
      }
    }
    if (HAS_V) {
      double s[1] = {0.0};
#pragma unroll
      for (int j = 0; j < kSV; ++j) s[0] += masked_dot(v[j], v[j], m[j]);
      block_sums<1>(s, red, tot);
      if (threadIdx.x == 0) ws_acc(a, uint64_t(2 * K), c, tot[0], first);
    }
    for (int i0 = 0; i0 < K; i0 += kSU) {
      f4 x[kSU][kSV];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const int i = i0 + u < K ? i0 + u : K - 1;
        const float* p = sld(a.xf, i);
#pragma unroll
        for (int j = 0; j < kSV; ++j) {
          if (vec[j]) {
            x[u][j] = ld_nt(p, g[j]);
          } else {
            x[u][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint64_t e = 4 * g[j] + q;
              if (e < a.n_f32) x[u][j][q] = p[e];
            }
          }
        }
      }
      double acc[2 * kSU];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        double dv = 0.0, dd = 0.0;
#pragma unroll
        for (int j = 0; j < kSV; ++j) {
          // the delta is formed in fp32, as compute_weight_deltas does
          const f4 d = HAS_BASE ? x[u][j] - b[j] : x[u][j];
          if (HAS_V) dv += masked_dot(d, v[j], m[j]);
          dd += masked_dot(d, d, m[j]);
        }
        acc[u] = dv;
        acc[kSU + u] = dd;
      }
      block_sums<2 * kSU>(acc, red, tot);
      if (threadIdx.x < 2 * kSU) {
        const int u = threadIdx.x % kSU;
        if (i0 + u < K) {
          const bool is_dd = threadIdx.x >= kSU;
          if (is_dd || HAS_V) ws_acc(a, uint64_t(is_dd ? K + i0 + u : i0 + u), c, tot[threadIdx.x], first);
        }
      }
    }
    gp += kPass;
    first = false;
  } while (gp < g1);
}

template <bool HAS_BASE, bool HAS_V>
__device__ void stats_i64_chunk(const StatArgs& a, uint32_t cc, double (*red)[2 * kSU + 1], double* tot) {
  const Chunk ch = load_chunk(a.ci, cc, a.n_i64);
  const uint32_t c = a.ncf + cc;
  const int K = a.K;
  if (HAS_V) {
    double s[1] = {0.0};
    for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += kBlock) s[0] += (double)a.v_if[e] * a.v_if[e];
    block_sums<1>(s, red, tot);
    if (threadIdx.x == 0) ws_acc(a, uint64_t(2 * K), c, tot[0], true);
  }
  for (int i0 = 0; i0 < K; i0 += kSU) {
    double acc[2 * kSU];
#pragma unroll
    for (int u = 0; u < 2 * kSU; ++u) acc[u] = 0.0;
    for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += kBlock) {
      const double vv = HAS_V ? (double)a.v_if[e] : 0.0;
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        if (i0 + u < K) {
          const float d = i64_delta(sld(a.xi, i0 + u), HAS_BASE ? a.base_i : nullptr, e);
          acc[u] += (double)d * vv;
          acc[kSU + u] += (double)d * d;
        }
      }
    }
    block_sums<2 * kSU>(acc, red, tot);
    if (threadIdx.x < 2 * kSU) {
      const int u = threadIdx.x % kSU;
      if (i0 + u < K) {
        const bool is_dd = threadIdx.x >= kSU;
        if (is_dd || HAS_V) ws_acc(a, uint64_t(is_dd ? K + i0 + u : i0 + u), c, tot[threadIdx.x], true);
      }
    }
  }
}

template <bool HAS_BASE, bool HAS_V>
__global__ __launch_bounds__(kBlock) void entry_stats_partial(StatArgs a) {
  __shared__ double red[kWaves][2 * kSU + 1];
  __shared__ double tot[2 * kSU + 1];
  const uint32_t c = blockIdx.x;
  if (c < a.ncf) {
    const Chunk ch = load_chunk(a.cf, c, a.n_f32);
    if ((uint64_t(ch.end) + 3) / 4 > a.n_f32 / 4) {
      stats_f32_chunk<HAS_BASE, HAS_V, true>(a, c, ch, red, tot);
    } else {
      stats_f32_chunk<HAS_BASE, HAS_V, false>(a, c, ch, red, tot);
    }
  } else {
    stats_i64_chunk<HAS_BASE, HAS_V>(a, c - a.ncf, red, tot);
  }
}

// first chunk of `entry` in a table sorted by entry (n if none)
__device__ uint32_t lower_bound(const plato_agg_chunk* t, uint32_t n, uint32_t entry) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (t[mid].entry < entry) {
      lo = mid + 1;
    } else {
      hi = mid;
    }
  }
  return lo;
}

// One thread per (row, entry): sum that entry's chunk partials in table order.
__global__ __launch_bounds__(kBlock) void entry_stats_final(const double* ws, uint32_t nc,
                                                           const plato_agg_chunk* cf, uint32_t ncf,
                                                           const plato_agg_chunk* ci, uint32_t nci,
                                                           uint32_t n_entries, uint64_t rows, bool has_v,
                                                           int K, double* out) {
  const uint64_t idx = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (idx >= rows * n_entries) return;
  const uint64_t row = idx / n_entries;
  const uint32_t e = uint32_t(idx % n_entries);
  double s = 0.0;
  const bool computed = has_v || (row >= uint64_t(K) && row < uint64_t(2 * K));
  if (computed) {
    const double* w = ws + row * nc;
    for (uint32_t c = lower_bound(cf, ncf, e); c < ncf && cf[c].entry == e; ++c) s += w[c];
    for (uint32_t c = lower_bound(ci, nci, e); c < nci && ci[c].entry == e; ++c) s += w[ncf + c];
  }
  out[idx] = s;
}

// ---------------------------------------------------------------------------
// fedavg_entrywise
// ---------------------------------------------------------------------------
constexpr int kEU = 8;  // clients per batch (independent dwordx4 loads per lane)

struct EwArgs {
  const float* const* xf;
  const int64_t* const* xi;
  const float* w;  // [n_entries][K]
  const float* base_f;
  const int64_t* base_i;
  const float* noise_f;
  const float* noise_if;
  float* out_f;
  float* out_if;
  const plato_agg_chunk* cf;
  const plato_agg_chunk* ci;
  uint64_t n_f32, n_i64;
  uint32_t ncf, nci;
  float scale, noise_scale;
  int K, flags;
};

template <bool HAS_BASE>
__device__ __forceinline__ f4 ew_post(const EwArgs& a, f4 acc, f4 b, f4 noise, bool has_noise) {
  f4 u = acc * a.scale;
  if (has_noise) u = u + noise * a.noise_scale;
  if (HAS_BASE && (a.flags & PLATO_AGG_ADD_BASE)) u = b + u;
  return u;
}

// One element of a chunk's partial float4 group, or of an int64 entry: its K clients walked in order
// with kEwSU independent loads per round trip (a one-load-at-a-time walk is K round trips to HBM).
constexpr int kEwSU = 16;

template <bool HAS_BASE>
__device__ __forceinline__ float ew_f32_scalar(const EwArgs& a, const float* wrow, uint64_t e) {
  const float b = HAS_BASE ? a.base_f[e] : 0.f;
  const int K = a.K;
  float acc = 0.f;
  int i = 0;
  for (; i + kEwSU <= K; i += kEwSU) {
    float x[kEwSU];
#pragma unroll
    for (int u = 0; u < kEwSU; ++u) x[u] = sld(a.xf, i + u)[e];
#pragma unroll
    for (int u = 0; u < kEwSU; ++u) acc = acc + (HAS_BASE ? x[u] - b : x[u]) * sld(wrow, i + u);
  }
  for (; i < K; ++i) {
    const float x = sld(a.xf, i)[e];
    acc = acc + (HAS_BASE ? x - b : x) * sld(wrow, i);
  }
  return acc;
}

template <bool HAS_BASE, int B>
__device__ void ew_f32_chunk(const EwArgs& a, uint32_t c) {
  const Chunk ch = load_chunk(a.cf, c, a.n_f32);
  const uint64_t n4 = a.n_f32 / 4;
  const uint64_t g0 = ch.begin / 4, g1 = (uint64_t(ch.end) + 3) / 4;
  const float* wrow = a.w + uint64_t(ch.entry) * a.K;
  const int K = a.K;
  const bool has_noise = a.noise_f != nullptr;
  for (uint64_t g = g0 + threadIdx.x; g < g1; g += B) {
    const uint64_t e0 = 4 * g;
    const bool full = e0 >= ch.begin && e0 + 4 <= ch.end;  // all 4 elements in the chunk (=> in range)
    if (full && g < n4) {
      const f4 b = HAS_BASE ? ld_c(a.base_f, g) : f4{0.f, 0.f, 0.f, 0.f};
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
      int i = 0;
      for (; i + kEU <= K; i += kEU) {
        f4 x[kEU];
#pragma unroll
        for (int u = 0; u < kEU; ++u) x[u] = ld_nt(sld(a.xf, i + u), g);
#pragma unroll
        for (int u = 0; u < kEU; ++u) {
          const f4 d = HAS_BASE ? x[u] - b : x[u];
          acc = acc + d * sld(wrow, i + u);
        }
      }
      for (; i < K; ++i) {
        const f4 x = ld_nt(sld(a.xf, i), g);
        const f4 d = HAS_BASE ? x - b : x;
        acc = acc + d * sld(wrow, i);
      }
      const f4 noise = has_noise ? ld_c(a.noise_f, g) : f4{0.f, 0.f, 0.f, 0.f};
      st_nt(a.out_f, g, ew_post<HAS_BASE>(a, acc, b, noise, has_noise));
    } else {
      // boundary group: the chunk's own elements one by one
      for (int q = 0; q < 4; ++q) {
        const uint64_t e = e0 + q;
        if (e < ch.begin || e >= ch.end) continue;
        const float acc = ew_f32_scalar<HAS_BASE>(a, wrow, e);
        float u = acc * a.scale;
        if (has_noise) u = u + a.noise_f[e] * a.noise_scale;
        if (HAS_BASE && (a.flags & PLATO_AGG_ADD_BASE)) u = a.base_f[e] + u;
        a.out_f[e] = u;
      }
    }
  }
}

template <bool HAS_BASE, int B>
__device__ void ew_i64_chunk(const EwArgs& a, uint32_t cc) {
  typedef __attribute__((address_space(1))) const int64_t gi64;
  const Chunk ch = load_chunk(a.ci, cc, a.n_i64);
  const float* wrow = a.w + uint64_t(ch.entry) * a.K;
  const int K = a.K;
  for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += B) {
    // torch's int64 subtraction wraps; the promotion to fp32 happens after (i64_delta)
    const int64_t bv = HAS_BASE ? a.base_i[e] : 0;
    float acc = 0.f;
    int i = 0;
    for (; i + kEwSU <= K; i += kEwSU) {
      int64_t x[kEwSU];
#pragma unroll
      for (int u = 0; u < kEwSU; ++u) x[u] = ((gi64*)sld(a.xi, i + u))[e];
#pragma unroll
      for (int u = 0; u < kEwSU; ++u) {
        const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x[u] - (uint64_t)bv) : x[u];
        acc = acc + (float)d * sld(wrow, i + u);
      }
    }
    for (; i < K; ++i) {
      const int64_t x = ((gi64*)sld(a.xi, i))[e];
      const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x - (uint64_t)bv) : x;
      acc = acc + (float)d * sld(wrow, i);
    }
    float u = acc * a.scale;
    if (a.noise_if) u = u + a.noise_if[e] * a.noise_scale;
    // update_weights: int64 weight + fp32 delta -> fp32(b) + u
    if (HAS_BASE && (a.flags & PLATO_AGG_ADD_BASE)) u = (float)a.base_i[e] + u;
    a.out_if[e] = u;
  }
}

// The int64 chunks are the grid's first blocks (dispatched first, their K-client walks run beside the
// stream instead of after it), the fp32 chunks follow.  B threads per chunk; the engine's chunk
// (FedAvgEngine.ENTRYWISE_CHUNK = 256 elements) is B x 1 float4 group at the default B = 64; the
// chunk loop strides by the block, so any chunk length is covered.
template <bool HAS_BASE, int B>
__global__ __launch_bounds__(B) void fedavg_entrywise_kernel(EwArgs a) {
  const uint32_t c = blockIdx.x;
  if (c < a.nci) {
    ew_i64_chunk<HAS_BASE, B>(a, c);
  } else {
    ew_f32_chunk<HAS_BASE, B>(a, c - a.nci);
  }
}

// threads per fedavg_entrywise workgroup: one wave, as the FedAvg kernel
constexpr int kEwBlock = 64;
#ifdef PLATO_AGG_TUNE
int g_ew_block = 0;  // plato_agg_tune_set_entrywise_block: 0 = kEwBlock
#endif

template <bool HAS_BASE>
void launch_entrywise(const EwArgs& a, uint32_t nc, hipStream_t stream) {
  int blk = kEwBlock;
#ifdef PLATO_AGG_TUNE
  if (g_ew_block) blk = g_ew_block;
#endif
  if (blk == 256) {
    hipLaunchKernelGGL((fedavg_entrywise_kernel<HAS_BASE, 256>), dim3(nc), dim3(256), 0, stream, a);
  } else if (blk == 128) {
    hipLaunchKernelGGL((fedavg_entrywise_kernel<HAS_BASE, 128>), dim3(nc), dim3(128), 0, stream, a);
  } else {
    hipLaunchKernelGGL((fedavg_entrywise_kernel<HAS_BASE, 64>), dim3(nc), dim3(64), 0, stream, a);
  }
}


// ---------------------------------------------------------------------------
// entry_norms_f32: torch.linalg.norm(fp32 tensor) exactly as x86-64 PyTorch
// computes it on the CPU (ATen's vectorised last-dim 2-norm reduction, the
// path a contiguous whole-tensor norm takes): 8 fp32 lanes, lane j
// accumulating fma(v, v, acc_j) over elements j, j+8, ... of the first
// m = n - n%8 elements; then acc_0 + acc_1 + ... + acc_7 in order, the tail
// elements fma'd onto that, and an fp32 sqrt.  Reproducing the order makes
// FedAtt's attention (fedatt_algorithm.py:39) bit-exact.
//
// Each chain is serial (m/8 dependent fmas), so the kernel is built for
// bytes in flight per chain: ONE wavefront per (entry, client).  All 64 lanes
// load the delta coalesced, kNR elements each per tile (lane L, register r
// holds element 64r + L), prefetching the next tile while the current one is
// consumed.  The tile is transposed through a wave-private LDS region so that
// chain j's steps are contiguous (32 ds_write_b32 per lane per tile), and
// lanes 0..7 walk their chain with 16-byte LDS reads, 4 fmas each.  Elements
// past m are fed as +0 (acc + 0*0 leaves a non-negative acc unchanged).
// ---------------------------------------------------------------------------
constexpr int kNormLanes = 8;
constexpr int kNR = 32;                 // elements per lane per tile
constexpr int kNTile = 64 * kNR;        // 2048 elements per tile

struct NormArgs {
  const float* const* xf;
  const int64_t* const* xi;
  const float* base_f;
  const int64_t* base_i;
  const plato_agg_chunk* ef;  // one piece per fp32 entry
  const plato_agg_chunk* ei;  // one piece per int64 entry
  float* out;                 // [K][n_entries]
  uint64_t n_f32, n_i64;
  uint32_t nef, nei, n_entries;
  int K;
};

// one client's delta at element e of its region (pointers hoisted by the caller)

// ATen's scalar tail of the last-dim 2-norm (`buffer[0] += v * v` after the
// 8-lane part), as x86-64 PyTorch 2.10 compiled it: while 4 or more remain,
// the four products come from one SSE multiply and are added in order
// (separately rounded); the last 1-3 are fused (vfmadd231ss).  Pinned against
// torch on ragged sizes in tests/test_reductions.py (oracle/reductions.c).
__device__ __forceinline__ float torch_norm_tail_step(float s, float v, uint64_t e, uint64_t m, uint64_t n) {
  if (n - m >= 4 && e < m + 4) return s + v * v;
  return __builtin_fmaf(v, v, s);
}

template <bool HAS_BASE, bool I64>
__device__ __forceinline__ float norm_delta(const void* x, const void* b, uint64_t e) {
  if constexpr (I64) {
    return i64_delta((const int64_t*)x, HAS_BASE ? (const int64_t*)b : nullptr, e);
  } else {
    const float xv = __builtin_nontemporal_load(((__attribute__((address_space(1))) const float*)x) + e);
    return HAS_BASE ? xv - ((__attribute__((address_space(1))) const float*)b)[e] : xv;
  }
}

// LDS transpose region of one wavefront: chain j's 256 steps of a tile in row
// j, rows padded by 8 floats so that both the 64-lane writes and the 8-lane
// 16-byte reads hit distinct banks.
constexpr int kNRow = kNTile / kNormLanes + 8;

template <bool HAS_BASE, bool I64>
__device__ void norm_pair(const NormArgs& a, const Chunk ch, int i, int lane, float (*rows)[kNRow]) {
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  const void* x = I64 ? (const void*)sld(a.xi, i) : (const void*)sld(a.xf, i);
  const void* b = I64 ? (const void*)a.base_i : (const void*)a.base_f;
  float acc = 0.f;
  float cur[kNR], nxt[kNR];
  auto load_tile = [&](uint64_t t0, float (&dst)[kNR]) {
    // clamp the address, zero the value: no branch around the loads (m > 0 here)
#pragma unroll
    for (int r = 0; r < kNR; ++r) {
      const uint64_t off = t0 + uint64_t(r) * 64 + lane;
      const float v = norm_delta<HAS_BASE, I64>(x, b, ch.begin + (off < m ? off : m - 1));
      dst[r] = off < m ? v : 0.f;
    }
  };
  if (m) load_tile(0, cur);
  for (uint64_t t0 = 0; t0 < m; t0 += kNTile) {
    // element 64r + lane of the tile is step 8r + lane/8 of chain lane%8
#pragma unroll
    for (int r = 0; r < kNR; ++r) rows[lane & 7][8 * r + (lane >> 3)] = cur[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t0 + kNTile < m) load_tile(t0 + kNTile, nxt);
    if (lane < kNormLanes) {
      const f4* row = reinterpret_cast<const f4*>(rows[lane]);
#pragma unroll 8
      for (int t = 0; t < kNTile / kNormLanes / 4; ++t) {
        const f4 v = row[t];
        acc = __builtin_fmaf(v.x, v.x, acc);
        acc = __builtin_fmaf(v.y, v.y, acc);
        acc = __builtin_fmaf(v.z, v.z, acc);
        acc = __builtin_fmaf(v.w, v.w, acc);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int r = 0; r < kNR; ++r) cur[r] = nxt[r];
  }
  // lanes added in order (ATen's buffer[0] + buffer[1] + ...), then the tail on top
  float s = __shfl(acc, 0, 64);
  for (int l = 1; l < kNormLanes; ++l) s = s + __shfl(acc, l, 64);
  if (lane != 0) return;
  for (uint64_t e = m; e < n; ++e) {
    const float v = norm_delta<HAS_BASE, I64>(x, b, ch.begin + e);
    s = torch_norm_tail_step(s, v, e, m, n);
  }
  if (ch.entry < a.n_entries) a.out[uint64_t(i) * a.n_entries + ch.entry] = sqrtf(s);
}

// kRest: only the pairs the split register-staged launch leaves out (int64 entries, and the fp32 entry
// that reaches the arena's partial last float4 group).
template <bool HAS_BASE, bool kRest = false>
__global__ __launch_bounds__(kBlock) void entry_norms_kernel(NormArgs a) {
  // one wavefront per (entry, client), entry-major
  __shared__ __attribute__((aligned(16))) float rows[kBlock / 64][kNormLanes][kNRow];
  const int wave = threadIdx.x >> 6;
  const uint64_t pair = uint64_t(blockIdx.x) * (kBlock / 64) + wave;
  const int lane = threadIdx.x & 63;
  if (pair >= uint64_t(a.nef + a.nei) * a.K) return;  // whole wavefronts exit together
  const uint32_t ent = uint32_t(pair / a.K);
  const int i = int(pair % a.K);
  if (ent < a.nef) {
    const Chunk ch = load_chunk(a.ef, ent, a.n_f32);
    if (kRest && uint64_t(ch.end) <= (a.n_f32 & ~3ull)) return;
    norm_pair<HAS_BASE, false>(a, ch, i, lane, rows[wave]);
  } else {
    norm_pair<HAS_BASE, true>(a, load_chunk(a.ei, ent - a.nef, a.n_i64), i, lane, rows[wave]);
  }
}

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

// s_waitcnt with only vmcnt bounded (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt[5:4] at [15:14]).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// ---------------------------------------------------------------------------
// entry_norms, producer / consumer version: two waves per (entry, client).
// The chain wave (wave 0) does nothing but walk its chains over ready tiles of
// d = x - b; the producer wave (wave 1) streams x and b into a kPS-deep LDS ring
// by LDS-DMA (the only reader of that ring, so reusing a slot needs no sync),
// forms d for the next tile into a double-buffered d tile, and meets the chain
// wave at one s_barrier per tile.  Same chains, same order as the kernels above.
// ---------------------------------------------------------------------------

// s_waitcnt lgkmcnt(0) alone (vmcnt left at its maximum: the glds stay in flight)
__device__ __forceinline__ void wait_lgkm0() {
  __builtin_amdgcn_s_waitcnt((63 & 15) | (7 << 4) | (0 << 8) | ((63 >> 4) << 14));
}
// s_waitcnt lgkmcnt(N) alone
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  __builtin_amdgcn_s_waitcnt((63 & 15) | (7 << 4) | (N << 8) | ((63 >> 4) << 14));
}

template <int T, bool HAS_BASE>
__device__ __forceinline__ void pc_issue(const float* x, const float* b, float (*raw)[2][T], uint32_t slot,
                                         uint64_t g0, uint64_t gmax, int lane) {
#pragma unroll
  for (int o = 0; o < (HAS_BASE ? 2 : 1); ++o) {
    const float* src = o == 0 ? x : b;
#pragma unroll
    for (int c = 0; c < T / 256; ++c) {
      uint64_t g = g0 + uint64_t(c) * 64 + lane;
      g = g < gmax ? g : gmax;
      __builtin_amdgcn_global_load_lds((gvoid*)(src + 4 * g), (lvoid*)&raw[slot][o][c * 256], 16, 0, 0);
    }
  }
}

// d tile layout: natural (element t of the tile at t), or transposed (TR): chain
// c's steps contiguous in row c, rows kTS floats apart.  kTS = T/8 + 4 keeps the
// producer's ds_write_b32 (32-lane groups, banks (a/4) mod 32) and the chain
// wave's ds_read_b128 (16-lane groups, banks (a/4) mod 64) conflict-free, and
// the chain wave reads 4 steps per instruction instead of 1.
template <int T, bool TR>
struct DTile {
  static constexpr int kTS = T / 8 + 4;
  static constexpr int kSize = TR ? 8 * kTS : T;
};

// Producer wave of the producer / consumer norms kernels: streams client x (and
// the baseline) through its kPS-deep LDS-DMA ring `raw` and writes tile tt of
// d = x - b to dtile + (tt & 1) * dstride (natural or transposed, DTile), then
// meets the chain wave at one s_barrier per tile.
template <int T, int PS, bool HAS_BASE, bool TR>
__device__ void pc_produce(const NormArgs& a, const Chunk ch, const float* x, int lane, float (*raw)[2][T],
                           float* dtile, int dstride) {
  constexpr int kRT = T, kPS = PS, kTS = DTile<T, TR>::kTS;
  constexpr int kPer = (HAS_BASE ? 2 : 1) * (kRT / 256);  // glds per stage
  static_assert((kPS - 1) * kPer < 64, "vmcnt range");
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  const uint32_t delta = ch.begin & 3u;
  const uint64_t g_first = ch.begin >> 2;
  const uint64_t ntiles = (delta + m + kRT - 1) / kRT;
  const uint64_t gmax = (a.n_f32 >> 2) - 1;
#pragma unroll
  for (int p = 0; p < kPS - 1; ++p)
    if (uint64_t(p) < ntiles) pc_issue<T, HAS_BASE>(x, a.base_f, raw, p, g_first + uint64_t(p) * (kRT / 4), gmax, lane);
  for (uint64_t tt = 0; tt < ntiles; ++tt) {
    // slot (tt - 1) % kPS was read by this wave's previous d pass
    if (tt + kPS - 1 < ntiles) {
      pc_issue<T, HAS_BASE>(x, a.base_f, raw, uint32_t((tt + kPS - 1) % kPS), g_first + (tt + kPS - 1) * (kRT / 4),
                         gmax, lane);
      wait_vmcnt<(kPS - 1) * kPer>();
    } else {
      wait_vmcnt<0>();
    }
    const uint32_t slot = uint32_t(tt % kPS);
    float* dt = dtile + (tt & 1) * dstride;
#pragma unroll
    for (int r = 0; r < kRT / 256; ++r) {
      f4 dv = *(reinterpret_cast<const f4*>(raw[slot][0]) + r * 64 + lane);
      if (HAS_BASE) dv = dv - *(reinterpret_cast<const f4*>(raw[slot][1]) + r * 64 + lane);  // fp32, as
                                                                                             // compute_weight_deltas
      if constexpr (TR) {
        // tile elements 256r + 4 lane + j: chain 4 (lane & 1) + j, step 32 r + lane / 2
        float* col = dt + 32 * r + (lane >> 1) + 4 * (lane & 1) * kTS;
        col[0] = dv.x;
        col[kTS] = dv.y;
        col[2 * kTS] = dv.z;
        col[3 * kTS] = dv.w;
      } else {
        reinterpret_cast<f4*>(dt)[r * 64 + lane] = dv;
      }
    }
    wait_lgkm0();  // d tile written (the glds of later stages stay in flight)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();  // tile tt ready; the chain wave is done with tile tt - 2
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  wait_vmcnt<0>();
}

// Chain wave of the producer / consumer norms kernels: walks the 8 chains
// (lanes 8..63 duplicating lanes 0..7) over tile tt at dtile + (tt & 1) *
// dstride, one s_barrier per tile.  Returns this lane's chain sum (torch's
// accumulator lane & 7).
// Tiles of an entry's vectorised part (tiles start on the arena's float4 grid, so the first one
// also covers the delta = begin mod 4 positions before the entry).
template <int T>
__device__ __forceinline__ uint64_t pc_ntiles(const Chunk ch) {
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  return ((ch.begin & 3u) + m + T - 1) / T;
}

// nbar >= the tile count: barriers past the last tile (a producer that runs whole trips of D
// tiles, entry_norms_rs_kernel) are met without reading a tile.
// kOW (transposed tiles): 0 = the compiler's waits (one s_waitcnt per ds_read_b128 of a 16-step block);
// 1 / 2 = one s_waitcnt per 16- / 32-step block (4 / 8 reads), the next block's reads in flight.  Each
// ds_read_b128 costs the chain wave ~5 issue cycles and each s_waitcnt ~3.7 beside the 4 of a
// dependent v_fmac_f32 (scripts/micro/chain_b128.hip, profiles/r04_micro_chain_b128.log).
template <int T, bool TR, int kOW = 0, int kLanes = kNormLanes>
__device__ float pc_chain(const Chunk ch, int lane, const float* dtile, int dstride, uint64_t nbar) {
  constexpr int kRT = T, kTS = DTile<T, TR>::kTS;
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  const uint32_t delta = ch.begin & 3u;
  const uint64_t ntiles = pc_ntiles<T>(ch);
  const int c = lane & 7;
  const int pj = int((uint32_t(c) + delta) & 7u);
  const int64_t s_shift = (uint32_t(c) + delta) >= 8u ? -1 : 0;
  const int64_t s_end = int64_t(m / kNormLanes);
  float acc = 0.f;
  for (uint64_t tt = 0; tt < nbar; ++tt) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (tt >= ntiles) continue;
    const float* tile = dtile + (tt & 1) * dstride;
    const float* p = TR ? tile + pj * kTS : tile + pj;
    constexpr int kStep = TR ? 1 : 8;  // floats between a chain's consecutive steps
    const int64_t s0 = int64_t(tt) * (kRT / kNormLanes) + s_shift;
    if (TR && kOW > 0 && tt >= 1 && int64_t(tt + 1) * (kRT / kNormLanes) <= s_end) {
      constexpr int kQ = 4 * (kOW > 0 ? kOW : 1), kNB = kRT / kNormLanes / (4 * kQ);
      const f4* q4 = reinterpret_cast<const f4*>(p);
      f4 buf[2][kQ];
#pragma unroll
      for (int q = 0; q < kQ; ++q) buf[0][q] = q4[q];
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        const int cb = blk & 1;
        if (blk + 1 < kNB) {
#pragma unroll
          for (int q = 0; q < kQ; ++q) buf[cb ^ 1][q] = q4[kQ * (blk + 1) + q];
          wait_lgkm<kQ>();  // this block's reads have landed; the next block's stay in flight
        } else {
          wait_lgkm<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
          acc = __builtin_fmaf(buf[cb][q].x, buf[cb][q].x, acc);
          acc = __builtin_fmaf(buf[cb][q].y, buf[cb][q].y, acc);
          acc = __builtin_fmaf(buf[cb][q].z, buf[cb][q].z, acc);
          acc = __builtin_fmaf(buf[cb][q].w, buf[cb][q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (TR && tt >= 1 && int64_t(tt + 1) * (kRT / kNormLanes) <= s_end) {
      // 16 steps per block as 4 ds_read_b128, the next block's in flight
      constexpr int kNB = kRT / kNormLanes / 16;
      const f4* q4 = reinterpret_cast<const f4*>(p);
      f4 cur[4], nxt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[q] = q4[q];
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        if (blk + 1 < kNB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) nxt[q] = q4[4 * (blk + 1) + q];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc = __builtin_fmaf(cur[q].x, cur[q].x, acc);
          acc = __builtin_fmaf(cur[q].y, cur[q].y, acc);
          acc = __builtin_fmaf(cur[q].z, cur[q].z, acc);
          acc = __builtin_fmaf(cur[q].w, cur[q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
      }
    } else if (!TR && tt >= 1 && int64_t(tt + 1) * (kRT / kNormLanes) <= s_end) {
      constexpr int kCB = 16, kNB = kRT / kNormLanes / kCB;
      float cur[kCB], nxt[kCB];
#pragma unroll
      for (int q = 0; q < kCB; ++q) cur[q] = p[8 * q];
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        if (blk + 1 < kNB) {
#pragma unroll
          for (int q = 0; q < kCB; ++q) nxt[q] = p[8 * (kCB * (blk + 1) + q)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < kCB; ++q) acc = __builtin_fmaf(cur[q], cur[q], acc);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < kCB; ++q) cur[q] = nxt[q];
      }
    } else if (lane < kLanes) {  // the first and the ragged last tile (kLanes: the lanes that own a chain)
      for (int u = 0; u < kRT / kNormLanes; ++u) {
        const int64_t st = s0 + u;
        if (st >= 0 && st < s_end) {
          const float v = p[kStep * u];
          acc = __builtin_fmaf(v, v, acc);
        }
      }
    }
  }
  return acc;
}

// The chain wave's epilogue: the 8 lanes added in order (ATen's buffer[0] + buffer[1] + ...),
// then the scalar tail over positions m .. n - 1, then the square root.
template <bool HAS_BASE>
__device__ __forceinline__ void pc_finish(const NormArgs& a, const Chunk ch, int i, const float* x, int lane,
                                          float acc) {
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  float s = __shfl(acc, 0, 64);
  for (int l = 1; l < kNormLanes; ++l) s = s + __shfl(acc, l, 64);
  if (lane != 0) return;
  for (uint64_t e = m; e < n; ++e) {
    const uint64_t idx = ch.begin + e;
    const float v = HAS_BASE ? x[idx] - a.base_f[idx] : x[idx];
    s = torch_norm_tail_step(s, v, e, m, n);
  }
  if (ch.entry < a.n_entries) a.out[uint64_t(i) * a.n_entries + ch.entry] = sqrtf(s);
}

// Long entries (at least half as long as the table's first: the engine passes the table longest
// first) are the launch's critical path.
__device__ __forceinline__ bool pc_long(const NormArgs& a, const Chunk ch) {
  const Chunk c0 = load_chunk(a.ef, 0, a.n_f32);
  return 2 * uint64_t(ch.end - ch.begin) >= uint64_t(c0.end - c0.begin);
}

// Chain-wave priority (PRIO): > 0 a flat s_setprio; -1 the long entries' chains at 3, the others at 1
// (the longest chains, the launch's critical path, first); -2 as -1, and the long entries' producers
// at 2 (entry_norms_rs_kernel).  The other producers stay at 0.
template <int PRIO>
__device__ __forceinline__ void pc_chain_prio(const NormArgs& a, const Chunk ch) {
  if constexpr (PRIO > 0) {
    __builtin_amdgcn_s_setprio(PRIO);
  } else if constexpr (PRIO < 0) {  // -1, -2
    if (pc_long(a, ch)) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(1);
  }
}

template <int T, int PS, bool HAS_BASE, bool TR = false, int PRIO = 0>
__device__ void norm_pc(const NormArgs& a, const Chunk ch, int i, int wave, int lane, float (*raw)[2][T],
                        float (*dbuf)[DTile<T, TR>::kSize]) {
  const float* x = sld(a.xf, i);
  if (wave == 1) {  // producer
    pc_produce<T, PS, HAS_BASE, TR>(a, ch, x, lane, raw, dbuf[0], DTile<T, TR>::kSize);
    return;
  }
  pc_chain_prio<PRIO>(a, ch);
  pc_finish<HAS_BASE>(a, ch, i, x, lane, pc_chain<T, TR>(ch, lane, dbuf[0], DTile<T, TR>::kSize, pc_ntiles<T>(ch)));
}

template <int T, int PS, bool HAS_BASE, bool TR = false, int PRIO = 0>
__global__ __launch_bounds__(128) void entry_norms_pc_kernel(NormArgs a) {
  __shared__ __attribute__((aligned(16))) float raw[PS][2][T];
  __shared__ __attribute__((aligned(16))) float dbuf[2][DTile<T, TR>::kSize];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint64_t pair = blockIdx.x;  // entry-major over the (longest-first) tables
  const uint32_t ent = uint32_t(pair / uint64_t(a.K));
  const int i = int(pair % uint64_t(a.K));
  float(*rows)[kNRow] = reinterpret_cast<float(*)[kNRow]>(&raw[0][0][0]);
  if (ent < a.nef) {
    const Chunk ch = load_chunk(a.ef, ent, a.n_f32);
    if (uint64_t(ch.end) > (a.n_f32 & ~3ull)) {  // the arena's partial last float4 group: per-wave path
      if (wave == 0) norm_pair<HAS_BASE, false>(a, ch, i, lane, rows);
      return;
    }
    norm_pc<T, PS, HAS_BASE, TR, PRIO>(a, ch, i, wave, lane, raw, dbuf);
  } else if (ent < a.nef + a.nei) {
    if (wave == 0) norm_pair<HAS_BASE, true>(a, load_chunk(a.ei, ent - a.nef, a.n_i64), i, lane, rows);
  }
}

// ---------------------------------------------------------------------------
// entry_norms, register-staged producer / consumer (round 4).  The kernel above
// stages x and b through a kPS-deep LDS ring by LDS-DMA, so the bytes a pair
// keeps in flight cost LDS (49-66 KB per workgroup, 2-3 workgroups per CU) and
// every element crosses the LDS three times (DMA in, d pass out, transposed d).
// Here P producer waves hold D tiles of x and b in VGPRs (the register file is
// 4x the LDS and otherwise idle in this kernel), form d = x - b in registers and
// write it transposed straight into the two-slot d tile ring the chain wave
// reads: LDS per workgroup is the d ring alone (8.4 / 16.6 KB at T = 1,024 /
// 2,048), a pair keeps D x T x 8 bytes in flight, and the chain wave (pc_chain,
// same tiles, same order) meets the producers at one s_barrier per tile.
// Producers run whole trips of D tiles (register slots are static); tiles past
// the last reload the last tile (valid addresses, never read) and the chain wave
// meets their barriers without reading.
// ---------------------------------------------------------------------------
template <int T, int P, int D, bool HAS_BASE>
__device__ void rs_produce(const NormArgs& a, const Chunk ch, const float* x, int w, int lane, float* dtile,
                           int dstride, uint64_t ntiles, uint64_t nbar) {
  constexpr int kTS = DTile<T, true>::kTS;
  constexpr int kIt = T / 256 / P;  // 256-element iterations (4 per lane) per producer and tile
  static_assert(kIt >= 1 && kIt * P * 256 == T, "whole iterations per producer");
  constexpr int kOps = HAS_BASE ? 2 : 1;
  static_assert((D - 1) * kIt * kOps < 64, "vmcnt range");
  const uint64_t g_first = ch.begin >> 2;
  const uint64_t gmax = (a.n_f32 >> 2) - 1;
  const gf4* xs = (const gf4*)(x);
  const gf4* bs = (const gf4*)(a.base_f);
  f4 xr[D][kIt], br[D][kIt];
  auto issue = [&](f4(&xv)[kIt], f4(&bv)[kIt], uint64_t t) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      uint64_t g = g_first + t * (T / 4) + uint64_t(it * P + w) * 64 + lane;
      g = g < gmax ? g : gmax;
      xv[it] = __builtin_nontemporal_load(xs + g);
      if (HAS_BASE) bv[it] = bs[g];
    }
  };
#pragma unroll
  for (int j = 0; j < D; ++j) issue(xr[j], br[j], uint64_t(j) < ntiles ? uint64_t(j) : ntiles - 1);
  for (uint64_t t0 = 0; t0 < nbar; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const uint64_t tt = t0 + j;
      wait_vmcnt<(D - 1) * kIt * kOps>();  // tile tt's loads (the oldest D - 1 trips stay in flight)
      float* dt = dtile + (tt & 1) * dstride;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        f4 dv = xr[j][it];
        if (HAS_BASE) dv = dv - br[j][it];  // fp32, as compute_weight_deltas
        // tile elements 256 r + 4 lane + c: chain 4 (lane & 1) + c, step 32 r + lane / 2
        float* col = dt + 32 * (it * P + w) + (lane >> 1) + 4 * (lane & 1) * kTS;
        col[0] = dv.x;
        col[kTS] = dv.y;
        col[2 * kTS] = dv.z;
        col[3 * kTS] = dv.w;
      }
      const uint64_t nt = tt + D;
      issue(xr[j], br[j], nt < ntiles ? nt : ntiles - 1);
      wait_lgkm0();  // d tile written (the loads stay in flight)
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __builtin_amdgcn_s_barrier();  // tile tt ready; the chain wave is done with tile tt - 1
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
  }
  wait_vmcnt<0>();
}

template <int T, int P, int D, bool HAS_BASE, int PRIO, bool kSplit = false, int kOW = 0>
__device__ __forceinline__ void rs_pair(const NormArgs& a, uint64_t pair, int wave, int lane, float* dbuf) {
  constexpr int kSize = DTile<T, true>::kSize;
  const uint32_t ent = uint32_t(pair / uint64_t(a.K));  // entry-major over the (longest-first) tables
  const int i = int(pair % uint64_t(a.K));
  float(*rows)[kNRow] = reinterpret_cast<float(*)[kNRow]>(dbuf);
  if (ent < a.nef) {
    const Chunk ch = load_chunk(a.ef, ent, a.n_f32);
    if (uint64_t(ch.end) > (a.n_f32 & ~3ull)) {  // the arena's partial last float4 group: per-wave path
      if (!kSplit && wave == 0) norm_pair<HAS_BASE, false>(a, ch, i, lane, rows);
      return;
    }
    const uint64_t ntiles = pc_ntiles<T>(ch), nbar = (ntiles + D - 1) / D * D;
    const float* x = sld(a.xf, i);
    if (wave > 0) {
      if (PRIO == -2 && pc_long(a, ch)) __builtin_amdgcn_s_setprio(2);  // long producers above short chains
      else __builtin_amdgcn_s_setprio(0);
      if (ntiles) rs_produce<T, P, D, HAS_BASE>(a, ch, x, wave - 1, lane, dbuf, kSize, ntiles, nbar);
      return;
    }
    pc_chain_prio<PRIO>(a, ch);
    pc_finish<HAS_BASE>(a, ch, i, x, lane, pc_chain<T, true, kOW>(ch, lane, dbuf, kSize, nbar));
  } else if (!kSplit && ent < a.nef + a.nei) {
    if (wave == 0) norm_pair<HAS_BASE, true>(a, load_chunk(a.ei, ent - a.nef, a.n_i64), i, lane, rows);
  }
}

// kSplit: the per-wave pairs (int64 entries, the partial-last-group fp32 entry) are left to a second
// launch (entry_norms_kernel<., true>), so that norm_pair's 64 registers of tile prefetch do not set
// this kernel's register count and with it how many pairs share a CU.
template <int T, int P, int D, bool HAS_BASE, int PRIO, bool kSplit = false, int kOW = 0>
__global__ __launch_bounds__(64 * (1 + P)) void entry_norms_rs_kernel(NormArgs a) {
  constexpr int kSize = DTile<T, true>::kSize;
  static_assert(2 * kSize >= kNormLanes * kNRow, "norm_pair's rows fit the d ring");
  __shared__ __attribute__((aligned(16))) float dbuf[2 * kSize];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  rs_pair<T, P, D, HAS_BASE, PRIO, kSplit, kOW>(a, blockIdx.x, wave, lane, dbuf);
}

// ---------------------------------------------------------------------------
// entry_norms, C clients of one entry per workgroup (register-staged, split launch only).  The
// one-pair kernel above streams the baseline b once per (entry, client): at K = 128 the L2-served b
// re-reads take as many of a CU's ~110 in-flight read slots as the client bytes themselves
// ("What bounds the streams").  Here C chain waves (one per client, the same chains
// and order as pc_chain) share P producer waves that load each b tile once and the C clients' x
// tiles beside it, and write C transposed d tiles; everyone meets at one s_barrier per tile (the C
// pairs of one entry have the same tile count).  A ragged last group (K mod C) recomputes client
// K - 1 in its idle chain waves and does not store it.
// ---------------------------------------------------------------------------
template <int T, int P, int D, int C, bool HAS_BASE, int kCS = 2 * DTile<T, true>::kSize>
__device__ void rsc_produce(const NormArgs& a, const Chunk ch, const gf4* const (&xs)[C], int w, int lane,
                            float* dbuf, uint64_t ntiles, uint64_t nbar) {
  constexpr int kTS = DTile<T, true>::kTS, kSize = DTile<T, true>::kSize;
  constexpr int kIt = T / 256 / P;
  static_assert(kIt >= 1 && kIt * P * 256 == T, "whole iterations per producer");
  constexpr int kOps = C + (HAS_BASE ? 1 : 0);
  static_assert((D - 1) * kIt * kOps < 64, "vmcnt range");
  const uint64_t g_first = ch.begin >> 2;
  const uint64_t gmax = (a.n_f32 >> 2) - 1;
  const gf4* bs = (const gf4*)(a.base_f);
  f4 xr[D][kIt][C], br[D][kIt];
  auto issue = [&](f4(&xv)[kIt][C], f4(&bv)[kIt], uint64_t t) {
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      uint64_t g = g_first + t * (T / 4) + uint64_t(it * P + w) * 64 + lane;
      g = g < gmax ? g : gmax;
#pragma unroll
      for (int c = 0; c < C; ++c) xv[it][c] = __builtin_nontemporal_load(xs[c] + g);
      if (HAS_BASE) bv[it] = bs[g];
    }
  };
#pragma unroll
  for (int j = 0; j < D; ++j) issue(xr[j], br[j], uint64_t(j) < ntiles ? uint64_t(j) : ntiles - 1);
  for (uint64_t t0 = 0; t0 < nbar; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const uint64_t tt = t0 + j;
      wait_vmcnt<(D - 1) * kIt * kOps>();  // tile tt's loads (the later trips stay in flight)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float* dt = dbuf + c * kCS + int(tt & 1) * kSize;  // client c's two-slot ring
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
          f4 dv = xr[j][it][c];
          if (HAS_BASE) dv = dv - br[j][it];  // fp32, as compute_weight_deltas
          // tile elements 256 r + 4 lane + k: chain 4 (lane & 1) + k, step 32 r + lane / 2
          float* col = dt + 32 * (it * P + w) + (lane >> 1) + 4 * (lane & 1) * kTS;
          col[0] = dv.x;
          col[kTS] = dv.y;
          col[2 * kTS] = dv.z;
          col[3 * kTS] = dv.w;
        }
      }
      const uint64_t nt = tt + D;
      issue(xr[j], br[j], nt < ntiles ? nt : ntiles - 1);
      wait_lgkm0();  // d tiles written (the loads stay in flight)
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __builtin_amdgcn_s_barrier();  // tile tt ready; the chain waves are done with tile tt - 1
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
  }
  wait_vmcnt<0>();
}

template <int T, int P, int D, int C, bool HAS_BASE, int PRIO, int kOW>
__global__ __launch_bounds__(64 * (C + P)) void entry_norms_rsc_kernel(NormArgs a) {
  constexpr int kSize = DTile<T, true>::kSize;
  __shared__ __attribute__((aligned(16))) float dbuf[2 * C * kSize];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint32_t groups = uint32_t((a.K + C - 1) / C);
  const uint32_t ent = blockIdx.x / groups;  // entry-major over the (longest-first) fp32 table
  const int i0 = int(blockIdx.x % groups) * C;
  const Chunk ch = load_chunk(a.ef, ent, a.n_f32);
  if (uint64_t(ch.end) > (a.n_f32 & ~3ull)) return;  // the arena's partial last float4 group: per-wave launch
  const uint64_t ntiles = pc_ntiles<T>(ch), nbar = (ntiles + D - 1) / D * D;
  if (wave >= C) {
    __builtin_amdgcn_s_setprio(0);
    if (!ntiles) return;
    const gf4* xs[C];
#pragma unroll
    for (int c = 0; c < C; ++c) xs[c] = (const gf4*)sld(a.xf, i0 + c < a.K ? i0 + c : a.K - 1);
    rsc_produce<T, P, D, C, HAS_BASE>(a, ch, xs, wave - C, lane, dbuf, ntiles, nbar);
    return;
  }
  const int i = i0 + wave;
  const float* x = sld(a.xf, i < a.K ? i : a.K - 1);
  pc_chain_prio<PRIO>(a, ch);
  const float acc = pc_chain<T, true, kOW>(ch, lane, dbuf + 2 * wave * kSize, kSize, nbar);
  if (i < a.K) pc_finish<HAS_BASE>(a, ch, i, x, lane, acc);
}

// C clients of one entry in ONE chain wave (round 6): lane l runs chain l & 7 of client (l >> 3) % C
// (lanes 8 C .. 63 duplicate lanes 0 .. 8 C - 1), over that client's tile ring, so a workgroup holds one
// chain wave instead of C: the chain waves that share a SIMD's issue halve, and no chain waits at the
// tile barrier for a second chain wave.  Client rings kCS = 32 (mod 64) floats apart: a ds_read_b128 lane
// group's rows then fall on 16 different 4-bank slots (the 8 chains of a tile on slots 4 j, the clients
// 32 banks apart).  The epilogue of client c runs on lane 8 c.
template <bool HAS_BASE, int C>
__device__ __forceinline__ void pc_finish_folded(const NormArgs& a, const Chunk ch, int i0, int lane, float acc) {
  const int cl = (lane >> 3) % C, base = 8 * cl;
  float s = __shfl(acc, base, 64);
  for (int l = 1; l < kNormLanes; ++l) s = s + __shfl(acc, base + l, 64);
  const int i = i0 + cl;
  if (lane >= 8 * C || (lane & 7) || i >= a.K) return;
  const uint64_t n = ch.end - ch.begin, m = n - n % kNormLanes;
  const float* x = sld(a.xf, i);
  for (uint64_t e = m; e < n; ++e) {
    const uint64_t idx = ch.begin + e;
    const float v = HAS_BASE ? x[idx] - a.base_f[idx] : x[idx];
    s = torch_norm_tail_step(s, v, e, m, n);
  }
  if (ch.entry < a.n_entries) a.out[uint64_t(i) * a.n_entries + ch.entry] = sqrtf(s);
}

template <int T, int P, int D, int C, bool HAS_BASE, int PRIO, int kOW>
__global__ __launch_bounds__(64 * (1 + P)) void entry_norms_rscf_kernel(NormArgs a) {
  static_assert(8 * C <= 64, "C clients' chains in one wave");
  constexpr int kSize = DTile<T, true>::kSize;
  constexpr int kCS = 2 * kSize + (96 - (2 * kSize) % 64) % 64;  // client stride, = 32 (mod 64)
  static_assert(kCS % 64 == 32 && kCS % 4 == 0, "client rings 32 banks apart, 16-byte aligned");
  __shared__ __attribute__((aligned(16))) float dbuf[C * kCS];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint32_t groups = uint32_t((a.K + C - 1) / C);
  const uint32_t ent = blockIdx.x / groups;  // entry-major over the (longest-first) fp32 table
  const int i0 = int(blockIdx.x % groups) * C;
  const Chunk ch = load_chunk(a.ef, ent, a.n_f32);
  if (uint64_t(ch.end) > (a.n_f32 & ~3ull)) return;  // the arena's partial last float4 group: per-wave launch
  const uint64_t ntiles = pc_ntiles<T>(ch), nbar = (ntiles + D - 1) / D * D;
  if (wave >= 1) {
    __builtin_amdgcn_s_setprio(0);
    if (!ntiles) return;
    const gf4* xs[C];
#pragma unroll
    for (int c = 0; c < C; ++c) xs[c] = (const gf4*)sld(a.xf, i0 + c < a.K ? i0 + c : a.K - 1);
    rsc_produce<T, P, D, C, HAS_BASE, kCS>(a, ch, xs, wave - 1, lane, dbuf, ntiles, nbar);
    return;
  }
  const int cl = (lane >> 3) % C;
  pc_chain_prio<PRIO>(a, ch);
  const float acc = pc_chain<T, true, kOW, 8 * C>(ch, lane, dbuf + cl * kCS, kSize, nbar);
  pc_finish_folded<HAS_BASE, C>(a, ch, i0, lane, acc);
}

bool misaligned(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) != 0; }

int launch_error(const char* what) {
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string(what) + ": " + hipGetErrorString(err));
  return clear_error();
}

}  // namespace

extern "C" {

size_t plato_agg_entry_stats_workspace(int K, uint32_t n_chunks) {
  return size_t((2 * uint64_t(K > 0 ? K : 0) + 1) * (n_chunks ? n_chunks : 1) * sizeof(double));
}

int plato_agg_entry_stats(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                          const float* d_base_f32, const int64_t* d_base_i64, const float* d_v_f32,
                          const float* d_v_i64f, const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                          const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64, int n_entries,
                          size_t n_f32, size_t n_i64, double* d_workspace, double* d_out, hipStream_t stream) {
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (n_entries <= 0) return set_error(PLATO_AGG_EINVAL, "n_entries must be >= 1");
  if (!d_workspace || !d_out) return set_error(PLATO_AGG_EINVAL, "null workspace/output pointer");
  if (n_chunks_f32 && (!d_x_f32 || !d_chunks_f32)) return set_error(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_chunks_i64 && (!d_x_i64 || !d_chunks_i64 || (d_base_f32 && !d_base_i64) || (d_v_f32 && !d_v_i64f)))
    return set_error(PLATO_AGG_EINVAL, "null int64 pointer");
  if (misaligned(d_base_f32) || misaligned(d_v_f32))
    return set_error(PLATO_AGG_EINVAL, "fp32 baseline / v must be 16-byte aligned");
  if (n_f32 > 0xffffffffull || n_i64 > 0xffffffffull)
    return set_error(PLATO_AGG_EINVAL, "arena too large for 32-bit chunk offsets");
  const uint64_t nc = uint64_t(n_chunks_f32) + n_chunks_i64;
  if (nc == 0 || nc > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "bad chunk count");
  StatArgs a{};
  a.xf = d_x_f32;
  a.xi = d_x_i64;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.v_f = d_v_f32;
  a.v_if = d_v_i64f;
  a.cf = d_chunks_f32;
  a.ci = d_chunks_i64;
  a.ws = d_workspace;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.ncf = n_chunks_f32;
  a.nci = n_chunks_i64;
  a.nc = uint32_t(nc);
  a.K = K;
  const dim3 grid{uint32_t(nc)}, block{kBlock};
  const bool hb = d_base_f32 != nullptr, hv = d_v_f32 != nullptr;
  if (hb && hv) {
    hipLaunchKernelGGL((entry_stats_partial<true, true>), grid, block, 0, stream, a);
  } else if (hb) {
    hipLaunchKernelGGL((entry_stats_partial<true, false>), grid, block, 0, stream, a);
  } else if (hv) {
    hipLaunchKernelGGL((entry_stats_partial<false, true>), grid, block, 0, stream, a);
  } else {
    hipLaunchKernelGGL((entry_stats_partial<false, false>), grid, block, 0, stream, a);
  }
  const uint64_t rows = 2 * uint64_t(K) + 1;
  const uint64_t total = rows * uint64_t(n_entries);
  hipLaunchKernelGGL(entry_stats_final, dim3(uint32_t((total + kBlock - 1) / kBlock)), block, 0, stream,
                     d_workspace, a.nc, d_chunks_f32, n_chunks_f32, d_chunks_i64, n_chunks_i64,
                     uint32_t(n_entries), rows, hv, K, d_out);
  return launch_error("entry_stats launch");
}

int plato_agg_fedavg_entrywise(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                               const float* d_w, int n_entries, const plato_agg_chunk* d_chunks_f32,
                               uint32_t n_chunks_f32, const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                               const float* d_base_f32, const int64_t* d_base_i64, const float* d_noise_f32,
                               const float* d_noise_i64f, float scale, float noise_scale, int flags,
                               float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64,
                               hipStream_t stream) {
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (n_entries <= 0 || !d_w) return set_error(PLATO_AGG_EINVAL, "null weight table");
  if ((flags & PLATO_AGG_ADD_BASE) && !d_base_f32) return set_error(PLATO_AGG_EINVAL, "ADD_BASE needs a baseline");
  if (n_chunks_f32 && (!d_x_f32 || !d_chunks_f32 || !d_out_f32))
    return set_error(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_chunks_i64 && (!d_x_i64 || !d_chunks_i64 || !d_out_i64f || (d_base_f32 && !d_base_i64) ||
                       (d_noise_f32 && !d_noise_i64f)))
    return set_error(PLATO_AGG_EINVAL, "null int64 pointer");
  if (misaligned(d_base_f32) || misaligned(d_noise_f32) || misaligned(d_out_f32))
    return set_error(PLATO_AGG_EINVAL, "fp32 baseline / noise / output must be 16-byte aligned");
  if (n_f32 > 0xffffffffull || n_i64 > 0xffffffffull)
    return set_error(PLATO_AGG_EINVAL, "arena too large for 32-bit chunk offsets");
  const uint64_t nc = uint64_t(n_chunks_f32) + n_chunks_i64;
  if (nc == 0) return clear_error();
  if (nc > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "bad chunk count");
  EwArgs a{};
  a.xf = d_x_f32;
  a.xi = d_x_i64;
  a.w = d_w;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.noise_f = d_noise_f32;
  a.noise_if = d_noise_i64f;
  a.out_f = d_out_f32;
  a.out_if = d_out_i64f;
  a.cf = d_chunks_f32;
  a.ci = d_chunks_i64;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.ncf = n_chunks_f32;
  a.nci = n_chunks_i64;
  a.scale = scale;
  a.noise_scale = noise_scale;
  a.K = K;
  a.flags = flags;
  if (d_base_f32) {
    launch_entrywise<true>(a, uint32_t(nc), stream);
  } else {
    launch_entrywise<false>(a, uint32_t(nc), stream);
  }
  return launch_error("fedavg_entrywise launch");
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
void plato_agg_tune_set_entrywise_block(int threads) {
  g_ew_block = (threads == 64 || threads == 128 || threads == 256) ? threads : 0;
}
#endif

}  // extern "C"

namespace {
using NormFn = void (*)(const NormArgs&, bool, dim3, hipStream_t);
template <int T, int PS>
void launch_pc(const NormArgs& a, bool hb, dim3 grid, hipStream_t st) {
  if (hb) hipLaunchKernelGGL((entry_norms_pc_kernel<T, PS, true, true, -1>), grid, dim3(128), 0, st, a);
  else hipLaunchKernelGGL((entry_norms_pc_kernel<T, PS, false, true, -1>), grid, dim3(128), 0, st, a);
}
template <int T, int P, int D, int PRIO = -1>
void launch_rs(const NormArgs& a, bool hb, dim3 grid, hipStream_t st) {
  if (hb) hipLaunchKernelGGL((entry_norms_rs_kernel<T, P, D, true, PRIO>), grid, dim3(64 * (1 + P)), 0, st, a);
  else hipLaunchKernelGGL((entry_norms_rs_kernel<T, P, D, false, PRIO>), grid, dim3(64 * (1 + P)), 0, st, a);
}
// The per-wave pairs' launch beside the main one (round 6): it is independent of the main kernel (other
// (entry, client) pairs, other outputs), so it runs on the device's side stream, forked from and joined
// back into the caller's stream, instead of ~9 us after the main kernel.
template <class Main, class Side>
void launch_beside(hipStream_t st, Main&& main, Side&& side) {
  hipDevice_t dev = 0;
  int cur = 0;
  plato_agg_internal::SideStream* ss = nullptr;
  if (hipStreamGetDevice(st, &dev) == hipSuccess && hipGetDevice(&cur) == hipSuccess) {
    if (cur != int(dev)) (void)hipSetDevice(dev);
    ss = plato_agg_internal::side_stream(dev);
  }
  if (ss) {
    std::lock_guard<std::mutex> lk(ss->mu);
    (void)hipEventRecord(ss->fork, st);
    (void)hipStreamWaitEvent(ss->s, ss->fork, 0);
    side(ss->s);
    main(st);
    (void)hipEventRecord(ss->join, ss->s);
    (void)hipStreamWaitEvent(st, ss->join, 0);
  } else {
    main(st);
    side(st);
  }
  if (ss && cur != int(dev)) (void)hipSetDevice(cur);
}

template <int T, int P, int D, int PRIO = -1, int kOW = 0>
void launch_rs_split(const NormArgs& a, bool hb, dim3, hipStream_t st) {
  const dim3 g1{uint32_t(uint64_t(a.nef) * uint64_t(a.K))};  // the fp32 pairs; int64 pairs come after them
  const uint64_t waves = (uint64_t(a.nef) + a.nei) * uint64_t(a.K);
  const dim3 g2{uint32_t((waves + kBlock / 64 - 1) / (kBlock / 64))};
  launch_beside(
      st,
      [&](hipStream_t s) {
        if (!a.nef) return;
        if (hb) hipLaunchKernelGGL((entry_norms_rs_kernel<T, P, D, true, PRIO, true, kOW>), g1, dim3(64 * (1 + P)), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_rs_kernel<T, P, D, false, PRIO, true, kOW>), g1, dim3(64 * (1 + P)), 0, s, a);
      },
      [&](hipStream_t s) {
        if (hb) hipLaunchKernelGGL((entry_norms_kernel<true, true>), g2, dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_kernel<false, true>), g2, dim3(kBlock), 0, s, a);
      });
}
template <int T, int P, int D, int C, int PRIO = -1, int kOW = 2>
void launch_rsc_split(const NormArgs& a, bool hb, dim3, hipStream_t st) {
  const dim3 g1{uint32_t(uint64_t(a.nef) * uint64_t((a.K + C - 1) / C))};
  const uint64_t waves = (uint64_t(a.nef) + a.nei) * uint64_t(a.K);
  const dim3 g2{uint32_t((waves + kBlock / 64 - 1) / (kBlock / 64))};
  launch_beside(
      st,
      [&](hipStream_t s) {
        if (!a.nef) return;
        if (hb) hipLaunchKernelGGL((entry_norms_rsc_kernel<T, P, D, C, true, PRIO, kOW>), g1, dim3(64 * (C + P)), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_rsc_kernel<T, P, D, C, false, PRIO, kOW>), g1, dim3(64 * (C + P)), 0, s, a);
      },
      [&](hipStream_t s) {
        if (hb) hipLaunchKernelGGL((entry_norms_kernel<true, true>), g2, dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_kernel<false, true>), g2, dim3(kBlock), 0, s, a);
      });
}
template <int T, int P, int D, int C, int PRIO = -1, int kOW = 2>
void launch_rscf_split(const NormArgs& a, bool hb, dim3, hipStream_t st) {
  const dim3 g1{uint32_t(uint64_t(a.nef) * uint64_t((a.K + C - 1) / C))};
  const uint64_t waves = (uint64_t(a.nef) + a.nei) * uint64_t(a.K);
  const dim3 g2{uint32_t((waves + kBlock / 64 - 1) / (kBlock / 64))};
  launch_beside(
      st,
      [&](hipStream_t s) {
        if (!a.nef) return;
        if (hb) hipLaunchKernelGGL((entry_norms_rscf_kernel<T, P, D, C, true, PRIO, kOW>), g1, dim3(64 * (1 + P)), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_rscf_kernel<T, P, D, C, false, PRIO, kOW>), g1, dim3(64 * (1 + P)), 0, s, a);
      },
      [&](hipStream_t s) {
        if (hb) hipLaunchKernelGGL((entry_norms_kernel<true, true>), g2, dim3(kBlock), 0, s, a);
        else hipLaunchKernelGGL((entry_norms_kernel<false, true>), g2, dim3(kBlock), 0, s, a);
      });
}
#ifdef PLATO_AGG_TUNE
void launch_per_wave(const NormArgs& a, bool hb, dim3, hipStream_t st) {
  const uint64_t threads = (uint64_t(a.nef) + a.nei) * uint64_t(a.K) * 64;  // a wave per pair
  const dim3 grid{uint32_t((threads + kBlock - 1) / kBlock)};
  if (hb) hipLaunchKernelGGL(entry_norms_kernel<true>, grid, dim3(kBlock), 0, st, a);
  else hipLaunchKernelGGL(entry_norms_kernel<false>, grid, dim3(kBlock), 0, st, a);
}
#endif
// Variants (include/plato_agg_tune.h; every one bitwise identical).  The rounds 1-4 sweeps (natural
// tiles, LDS-DMA ring kernels with 1-4 clients per workgroup, flat priorities, 256-1,024-element
// tiles; round 4: 1-8 producer waves, 2-4 tiles in flight, 4,096-element tiles, a persistent
// long/short split, a three-slot lookahead ring; DESIGN.md §11, §14, profiles/r0*_norms*) are trimmed to the round-4
// default, two of its neighbours, the round-3 LDS-DMA defaults and the per-wave first version.
// Interleaved on one box (K = 128 / 64 / 32 / 4 ResNet-18 clients, profiles/r04j-l_norms_k*.log):
// <2048, 2, 2> 1.25-1.26 / 0.97 / 0.95 / 0.94 ms against the round-3 defaults' 1.29-1.37 / 1.01 /
// 1.00 / 0.99; with the per-wave pairs in a second launch (64 VGPRs at 4 producer waves), <2048, 4,
// 2> 1.13-1.20 / 0.97 / - / 0.94 (profiles/r04s_norms_k*.log).  Split shapes measured and dropped
// (K = 128 / 64, interleaved): <2048, 2, 2> 1.31 / 1.01, <2048, 2, 1> 1.29 / 1.02, <2048, 4, 1> 1.21 /
// 1.00, <2048, 4, 3> 1.16 / 0.97 against the default's 1.13 / 0.97.
// One s_waitcnt per 32 chain steps (kOW = 2): 0.832 against 0.939 ms at K = 4 and 1.139 against 1.157
// at K = 128, interleaved (profiles/r04za_norms_k*.log; 76 VGPRs, six waves per SIMD); on a second box
// 1.101 / 0.873 ms at K = 128 / 64 against 1.198 / 0.973, and neither long producers at priority 2,
// 2 producers nor 3 tiles in flight beat it (1.12-1.20 / 0.88-0.89; profiles/r04zc_norms_k*.log).
// Round 5, two clients of one entry per workgroup sharing the baseline tiles (entry_norms_rsc_kernel,
// profiles/r05s-u_norms.log, interleaved, K = 32 / 64 / 96 / 128 / 256): <2048, 8, 2, C = 2> 0.93 / 0.94 /
// 0.995 / 1.044-1.065 / 2.005 ms against the one-client default's 0.839 / 0.870 / 1.002 / 1.100-1.106 /
// 2.228.  Where the 10,000 short pairs' traffic binds (K >= 96) the halved b reads win; below it the
// long entries' serial chains bind, and a chain that shares its tile barrier with a second client's
// runs ~10 % slower.  The default picks by K.  Measured and dropped: four clients per workgroup (1.18-1.26
// at K = 128), three (1.19), and the long entries kept at one client per workgroup (1.18 at K = 128:
// their ten-wave workgroups crowd the short pairs out; 0.86 at K = 32).
// Round 6: the clients of a workgroup folded into one chain wave (entry_norms_rscf_kernel), interleaved on
// five leases (profiles/r06zi-zk_norms_fold.log, r06zm, r06zp, r06zq): two clients 0.95-0.97 ms against 1.006
// for the two-wave form at K = 96; at K = 128 every two-client form runs in two modes from launch to launch
// (samples ~1.03 or ~1.25 ms; medians 1.04-1.26 for both forms), while four clients hold 1.10-1.12 on every
// lease — the better expected time, and four clients win outright at K = 192 (1.393 against 1.49-1.97) and
// 256 (1.849 against 2.024).  At K = 112 four clients 1.059 against 1.042 (two-client samples to 1.23).
// Below K = 96 the one-client shape stays (four clients 0.962, two 0.902 against 0.894 ms at K = 64).
constexpr int kNormShareK = 96, kNormFold4K = 128;
void launch_norms_default(const NormArgs& a, bool hb, dim3 g, hipStream_t st) {
  if (a.K >= kNormFold4K) launch_rscf_split<2048, 8, 2, 4>(a, hb, g, st);
  else if (a.K >= kNormShareK) launch_rscf_split<2048, 8, 2, 2>(a, hb, g, st);
  else launch_rs_split<2048, 4, 2, -1, 2>(a, hb, g, st);
}
constexpr NormFn kNormDefault = &launch_norms_default;
#ifdef PLATO_AGG_TUNE
const NormFn kNormVariants[] = {
    &launch_norms_default,         // 0: the default: one client per workgroup below K = 96, two folded from 96,
                                   //    four folded from 128
    &launch_rs<2048, 2, 2>,        // 1: 2 producer waves, one launch (the first round-4 default)
    &launch_rs<2048, 2, 3, -2>,    // 2: 3 tiles in flight, the long entries' producers at priority 2
    &launch_pc<1024, 5>,           // 3: LDS-DMA producer / consumer, 1,024-element tiles (round 3, > 6,144 pairs)
    &launch_pc<2048, 3>,           // 4: the same, 2,048-element tiles (round 3, <= 6,144 pairs)
    &launch_per_wave,              // 5: one wavefront per (entry, client) (the first version)
    &launch_rs_split<2048, 4, 2, -1, 1>,  // 6: one s_waitcnt per 16 chain steps (64 VGPRs)
    &launch_rs_split<2048, 4, 2>,         // 7: the compiler's waits, one per ds_read_b128 (the first round-4
                                          //    split default)
    &launch_rs_split<2048, 4, 2, -1, 2>,  // 8: the one-client shape (register-staged, 4 producer waves, 2 tiles
                                          //    in flight, the per-wave pairs (int64, partial last group) in a
                                          //    second launch, one s_waitcnt per 32 chain steps): the default below
                                          //    K = 96, rounds 4-5's default at every K
    &launch_rsc_split<2048, 8, 2, 2>,     // 9: two clients per workgroup (two chain waves), 8 producer waves: round
                                          //    5's default from K = 96
    &launch_rsc_split<2048, 4, 2, 2>,     // 10: two clients, 4 producer waves
    &launch_rsc_split<2048, 8, 3, 2>,     // 11: two clients, 3 tiles of loads in flight
    &launch_rsc_split<2048, 8, 2, 4>,     // 12: four clients, 8 producer waves
    // round 6: the clients of a workgroup folded into one chain wave (entry_norms_rscf_kernel)
    &launch_rscf_split<2048, 8, 2, 2>,    // 13: two clients, 8 producer waves: the default for K = 96 .. 127
    &launch_rscf_split<2048, 4, 2, 2>,    // 14: two clients, 4 producer waves
    &launch_rscf_split<2048, 8, 2, 4>,    // 15: four clients, 8 producer waves: the default from K = 128
    &launch_rscf_split<2048, 4, 2, 4>,    // 16: four clients, 4 producer waves
    // measured and dropped (K = 128, interleaved, profiles/r06zm_norms_fold_shapes.log, against 1.110 for the
    // default): two clients with 3 tiles in flight 1.152, 4,096-element tiles 1.895, three clients 1.166,
    // 1,024-element tiles 1.282 ms; the dispatch order spread by 4 / 8 (dispatched workgroup b running
    // grid item (b mod 4) ceil(G / 4) + b / 4: the long entries start late) 3.11 / 5.69 ms, four clients
    // spread by 4 2.39 ms (profiles/r06zp_norms_spread.log)
};
constexpr int kNumNormVariants = sizeof(kNormVariants) / sizeof(kNormVariants[0]);
#endif

int run_norms(NormFn fn, const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
              const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_chunk* d_entries_f32,
              uint32_t n_entries_f32, const plato_agg_chunk* d_entries_i64, uint32_t n_entries_i64, int n_entries,
              size_t n_f32, size_t n_i64, float* d_out, hipStream_t stream) {
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (n_entries <= 0 || !d_out) return set_error(PLATO_AGG_EINVAL, "null output / no entries");
  if (n_entries_f32 && (!d_x_f32 || !d_entries_f32)) return set_error(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_entries_i64 && (!d_x_i64 || !d_entries_i64 || (d_base_f32 && !d_base_i64)))
    return set_error(PLATO_AGG_EINVAL, "null int64 pointer");
  if (n_f32 > 0xffffffffull || n_i64 > 0xffffffffull)
    return set_error(PLATO_AGG_EINVAL, "arena too large for 32-bit chunk offsets");
  const uint64_t pairs = (uint64_t(n_entries_f32) + n_entries_i64) * uint64_t(K);
  if (pairs == 0) return clear_error();
  if (pairs > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "too many (client, entry) pairs");
  NormArgs a{};
  a.xf = d_x_f32;
  a.xi = d_x_i64;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.ef = d_entries_f32;
  a.ei = d_entries_i64;
  a.out = d_out;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.nef = n_entries_f32;
  a.nei = n_entries_i64;
  a.n_entries = uint32_t(n_entries);
  a.K = K;
  fn(a, d_base_f32 != nullptr, dim3(uint32_t(pairs)), stream);  // one workgroup per (entry, client)
  return launch_error("entry_norms launch");
}
}  // namespace

extern "C" {

int plato_agg_entry_norms_f32(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                              const float* d_base_f32, const int64_t* d_base_i64,
                              const plato_agg_chunk* d_entries_f32, uint32_t n_entries_f32,
                              const plato_agg_chunk* d_entries_i64, uint32_t n_entries_i64, int n_entries,
                              size_t n_f32, size_t n_i64, float* d_out, hipStream_t stream) {
  // The register-staged producer / consumer kernel at every grid size.
  return run_norms(kNormDefault, d_x_f32, d_x_i64, K, d_base_f32, d_base_i64, d_entries_f32, n_entries_f32,
                   d_entries_i64, n_entries_i64, n_entries, n_f32, n_i64, d_out, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_entry_norms_variants(void) { return kNumNormVariants; }

int plato_agg_tune_entry_norms(int variant, const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                               const float* d_base_f32, const int64_t* d_base_i64,
                               const plato_agg_chunk* d_entries_f32, uint32_t n_entries_f32,
                               const plato_agg_chunk* d_entries_i64, uint32_t n_entries_i64, int n_entries,
                               size_t n_f32, size_t n_i64, float* d_out, hipStream_t stream) {
  if (variant < 0 || variant >= kNumNormVariants) return set_error(PLATO_AGG_EINVAL, "bad entry_norms variant");
  return run_norms(kNormVariants[variant], d_x_f32, d_x_i64, K, d_base_f32, d_base_i64, d_entries_f32, n_entries_f32,
                   d_entries_i64, n_entries_i64, n_entries, n_f32, n_i64, d_out, stream);
}
#endif  // PLATO_AGG_TUNE

}  // extern "C"
