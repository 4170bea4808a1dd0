// reduce.hip — per-client dot products / squared norms over whole model
// arenas (gfx950), for the FedAvg variants whose weights depend on model-wide
// reductions: Port's cosine similarity (examples/async/port/port_server.py:24-52),
// Polaris / FedAdp / FedAtt norms and angles.
//
// Two passes, deterministic order (run-to-run bitwise reproducible):
//  1. dots_partial: one workgroup per 1,024-element chunk walks every client
//     (like the FedAvg kernel: one float4 per lane, U clients per batch, NT
//     loads), accumulates dot(d_i, v) and |d_i|^2 per lane in fp64, reduces the
//     2U values across the 64-lane wavefront with butterfly shuffles, stages
//     the 4 wave results in LDS and writes one partial per (client, chunk).
//  2. dots_final: one workgroup per output row sums its chunk partials
//     (strided per lane, shuffle tree, LDS across waves).
// fp64 accumulation: torch's fp32 CPU reduction order is not reproducible, so
// these results match the reference within tolerance, not bit for bit.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "common.h"
#include "plato_agg.h"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gf4;

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kU = 8;

template <class T>
__device__ __forceinline__ T sld(const T* p, int i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

__device__ __forceinline__ f4 ldnt(const float* base, uint64_t i4) {
  return __builtin_nontemporal_load((gf4*)base + i4);
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ double dot4(f4 a, f4 b) {
  return (double)a.x * b.x + (double)a.y * b.y + (double)a.z * b.z + (double)a.w * b.w;
}

// part layout: rows [0, K) = dot(d_i, v), rows [K, 2K) = |d_i|^2, row 2K = |v|^2;
// each row has nblk chunk partials.
struct DotArgs {
  const float* const* xs;      // K fp32 arenas
  const int64_t* const* xi;    // K int64 arenas (n_i64 > 0)
  const float* base;           // fp32 baseline (HAS_BASE)
  const int64_t* base_i;       // int64 baseline (HAS_BASE, n_i64 > 0)
  const float* v;              // fp32 reference vector
  const int64_t* v_i;          // int64 entries of the reference vector (n_i64 > 0)
  double* part;
  uint64_t n4, n, n_i64;
  uint32_t nblk;
  int K;
};

// int64 entries as torch.cat((fp32, int64)) sees them: promoted to fp32.
__device__ __forceinline__ float i64_delta(const DotArgs& a, int i, uint64_t e, bool has_base) {
  const int64_t x = sld(a.xi, i)[e];
  const int64_t d = has_base ? (int64_t)((uint64_t)x - (uint64_t)a.base_i[e]) : x;
  return (float)d;
}

template <bool HAS_BASE>
__global__ __launch_bounds__(kBlock) void dots_partial(DotArgs a) {
  const float* const* xs = a.xs;
  const int K = a.K;
  const float* base = a.base;
  const float* v = a.v;
  const uint64_t n4 = a.n4, n = a.n;
  double* part = a.part;
  const uint32_t nblk = a.nblk;
  __shared__ double red[kWaves][2 * kU];
  const uint32_t blk = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t idx = uint64_t(blk) * kBlock + threadIdx.x;
  const bool live = idx < n4;
  const uint64_t i4 = live ? idx : (n4 ? n4 - 1 : 0);
  const bool has_vec = n4 > 0;
  // scalar tail (n % 4 elements) is folded into lane 0 of workgroup 0
  const bool tail_lane = blk == 0 && threadIdx.x == 0;
  const uint64_t tail0 = 4 * n4;

  f4 b = f4{0.f, 0.f, 0.f, 0.f};
  f4 vv = f4{0.f, 0.f, 0.f, 0.f};
  if (has_vec) {
    if (HAS_BASE) b = ldnt(base, i4);
    vv = ldnt(v, i4);
  }
  // |v|^2
  {
    double s = (live && has_vec) ? dot4(vv, vv) : 0.0;
    if (tail_lane) {
      for (uint64_t e = tail0; e < n; ++e) s += (double)v[e] * v[e];
      for (uint64_t e = 0; e < a.n_i64; ++e) s += (double)(float)a.v_i[e] * (float)a.v_i[e];
    }
    s = wave_sum(s);
    if (lane == 0) red[wave][0] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int w = 0; w < kWaves; ++w) t += red[w][0];
      part[uint64_t(2 * K) * nblk + blk] = t;
    }
    __syncthreads();
  }

  for (int i0 = 0; i0 < K; i0 += kU) {
    double acc[2 * kU];
    f4 x[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u < K ? i0 + u : K - 1;
      x[u] = has_vec ? ldnt(sld(xs, i), i4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      // the delta is formed in fp32 exactly like compute_weight_deltas
      const f4 d = HAS_BASE ? x[u] - b : x[u];
      acc[u] = (live && has_vec) ? dot4(d, vv) : 0.0;
      acc[kU + u] = (live && has_vec) ? dot4(d, d) : 0.0;
      if (tail_lane && i0 + u < K) {
        const float* p = sld(xs, i0 + u);
        for (uint64_t e = tail0; e < n; ++e) {
          const float de = HAS_BASE ? p[e] - base[e] : p[e];
          acc[u] += (double)de * v[e];
          acc[kU + u] += (double)de * de;
        }
        for (uint64_t e = 0; e < a.n_i64; ++e) {
          const float de = i64_delta(a, i0 + u, e, HAS_BASE);
          acc[u] += (double)de * (float)a.v_i[e];
          acc[kU + u] += (double)de * de;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2 * kU; ++j) acc[j] = wave_sum(acc[j]);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 2 * kU; ++j) red[wave][j] = acc[j];
    }
    __syncthreads();
    if (threadIdx.x < 2 * kU) {
      const int j = threadIdx.x;
      const int u = j % kU;
      if (i0 + u < K) {
        double t = 0.0;
        for (int w = 0; w < kWaves; ++w) t += red[w][j];
        const uint64_t row = (j < kU) ? uint64_t(i0 + u) : uint64_t(K + i0 + u);
        part[row * nblk + blk] = t;
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void dots_final(const double* part, uint32_t nblk, double* out) {
  __shared__ double red[kWaves];
  const uint64_t row = blockIdx.x;
  double s = 0.0;
  for (uint32_t c = threadIdx.x; c < nblk; c += kBlock) s += part[row * nblk + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kWaves; ++w) t += red[w];
    out[row] = t;
  }
}

}  // namespace

extern "C" {

size_t plato_agg_client_dots_workspace(int K, size_t n) {
  const uint64_t nblk = (n / 4 + kBlock - 1) / kBlock;
  return size_t((2 * uint64_t(K > 0 ? K : 0) + 1) * (nblk ? nblk : 1) * sizeof(double));
}

int plato_agg_client_dots(const float* const* d_x, const int64_t* const* d_x_i64, int K, const float* d_base,
                          const int64_t* d_base_i64, const float* d_v, const int64_t* d_v_i64, size_t n_f32,
                          size_t n_i64, double* d_workspace, double* d_out, hipStream_t stream) {
  using plato_agg_internal::set_error;
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (!d_x || !d_v || !d_workspace || !d_out) return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (n_i64 && (!d_x_i64 || !d_v_i64 || (d_base && !d_base_i64)))
    return set_error(PLATO_AGG_EINVAL, "null int64 pointer");
  if ((reinterpret_cast<uintptr_t>(d_v) & 15u) || (d_base && (reinterpret_cast<uintptr_t>(d_base) & 15u)))
    return set_error(PLATO_AGG_EINVAL, "fp32 arrays must be 16-byte aligned");
  DotArgs a{};
  a.xs = d_x;
  a.xi = d_x_i64;
  a.base = d_base;
  a.base_i = d_base_i64;
  a.v = d_v;
  a.v_i = d_v_i64;
  a.part = d_workspace;
  a.n4 = n_f32 / 4;
  a.n = n_f32;
  a.n_i64 = n_i64;
  a.K = K;
  uint64_t nblk = (a.n4 + kBlock - 1) / kBlock;
  if (nblk == 0) nblk = 1;
  if (nblk > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "arena too large");
  a.nblk = uint32_t(nblk);
  if (d_base) {
    hipLaunchKernelGGL(dots_partial<true>, dim3(a.nblk), dim3(kBlock), 0, stream, a);
  } else {
    hipLaunchKernelGGL(dots_partial<false>, dim3(a.nblk), dim3(kBlock), 0, stream, a);
  }
  hipLaunchKernelGGL(dots_final, dim3(uint32_t(2 * K + 1)), dim3(kBlock), 0, stream, d_workspace, a.nblk, d_out);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string("client_dots launch: ") + hipGetErrorString(err));
  return plato_agg_internal::clear_error();
}

}  // extern "C"
