// FedAdp producer stream shapes, without the chains (pure loads, summed in registers).
//
// fedadp_dots_kernel's producers gather, per (pair group, chain group) workgroup, the chain
// group's share of every 64-element block of x (the flattened global gradient), of b (the
// baseline arena) and of the kP client arenas.  This probe times that access shape alone, on
// 128 ResNet-18-sized client arenas, for:
//   * kP pairs x kC chains per workgroup (kP * kC = 32: 128 / kP-byte pieces per block),
//   * with or without the x and b streams (kXB),
//   * the arena offset of b and y shifted by `shift` elements against the flat position
//     (an entry whose arena offset differs from its flat position mod 4),
//   * kW producer waves and kD stages of loads in flight per wave,
//   * kSync: one s_barrier per stage (the product's producer / chain rhythm),
//   * kRange: the workgroups of a pair read whole 64-blocks of consecutive block ranges
//     instead of their chain group's share of every block (same bytes, contiguous lines).
// Output: one line per shape, median ms of 10 launches and GB/s of unique / CU-side bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint64_t bytes) {
  const uint64_t n = bytes < 0xffffffffull ? bytes : 0xffffffffull;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)uint32_t(n), 0x00020000);
}
template <int kAux>
__device__ __forceinline__ f4v ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAux));
}

struct Args {
  const float* x;
  const float* b;
  const float* const* y;
  uint64_t nsteps;
  uint64_t n_arena;
  uint32_t shift;
  int n_pairs;
  float* sink;
};

template <int kP, int kC, int kW, int kIt, int kD, bool kXB, int kAuxY, bool kSync, int kRange, bool kXBcg = false, bool kRealign = false>
__global__ __launch_bounds__(64 * kW) void stream_kernel(Args a) {
  constexpr int kCa = kRange ? 64 : kC;         // addressing width
  constexpr int kS = 64 * 4 * kW * kIt / kCa;   // steps per stage
  constexpr int kLpB = kCa / 4, kBlkPerIt = 256 / kCa;
  constexpr int kGroups = kRange ? kRange : 64 / kC;
  const int blk = int(blockIdx.x), lo = blk & 7;
  const int grp = (blk / 8) % kGroups;
  const int cg = kRange ? 0 : grp;
  const int rg = kRange ? grp : 0;
  const int pg = (blk / (8 * kGroups)) * 8 + lo;
  if (pg * kP >= a.n_pairs) return;
  const int w = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
  __amdgpu_buffer_rsrc_t rx = rsrc(a.x, a.nsteps * 512), rb = rsrc(a.b, a.n_arena * 4), ry[kP];
#pragma unroll
  for (int k = 0; k < kP; ++k) ry[k] = rsrc(a.y[min(pg * kP + k, a.n_pairs - 1)], a.n_arena * 4);
  const uint64_t nsteps_r = kRange ? (a.nsteps + kRange - 1) / kRange : a.nsteps;
  const uint64_t s_off = uint64_t(rg) * nsteps_r;
  const uint64_t nst = (nsteps_r + kS - 1) / kS;
  const uint32_t last = uint32_t(min(a.nsteps, s_off + nsteps_r) - 1);
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  f4v rxv[kD][kIt], rbv[kD][kIt], ryv[kD][kIt][kP], rnv[kD][kIt][kRealign ? kP : 1];
  auto issue = [&](int j, uint32_t t) {
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      const int g = i * kW + w;
      const uint32_t s = min(uint32_t(s_off) + t * kS + uint32_t(g * kBlkPerIt + lane / kLpB), last);
      const uint32_t p = s * 64 + uint32_t(cg * kCa + (lane % kLpB) * 4);
      const uint32_t e = p + a.shift;
      if (kXB && kXBcg) {  // xb[cg][s / 8][x: 256 floats, b: 256 floats]: every load 1 KB contiguous
        const uint32_t ngr = (last + kBlkPerIt) / kBlkPerIt;
        const uint32_t q = ((uint32_t(cg) * ngr + s / kBlkPerIt) * 512 + (s % kBlkPerIt) * kC + (lane % kLpB) * 4) * 4u;
        rxv[j][i] = ld4<0>(rx, q);
        rbv[j][i] = ld4<0>(rx, q + 1024u);
      } else if (kXB) {
        rxv[j][i] = ld4<0>(rx, p * 4u);
        rbv[j][i] = ld4<0>(rb, e * 4u);
      }
      if (kRealign) {  // aligned 16-byte loads (realigned at use): the lane's and, for the last lane of a
                       // half-block, the next 16 bytes (other lanes: an offset past num_records reads 0, no request)
        const uint32_t e0 = e & ~3u;
#pragma unroll
        for (int k = 0; k < kP; ++k) {
          ryv[j][i][k] = ld4<kAuxY>(ry[k], e0 * 4u);
          rnv[j][i][k] = ld4<kAuxY>(ry[k], (lane & 7) == 7 ? (e0 + 4u) * 4u : 0xfffffff0u);
        }
      } else {
#pragma unroll
        for (int k = 0; k < kP; ++k) ryv[j][i][k] = ld4<kAuxY>(ry[k], e * 4u);
      }
    }
  };
#pragma unroll
  for (int j = 0; j < kD; ++j) issue(j, uint32_t(j));
  const uint64_t nst2 = (nst + kD - 1) / kD * kD;
  for (uint32_t t = 0; t < uint32_t(nst2); t += kD) {
#pragma unroll
    for (int j = 0; j < kD; ++j) {
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
#pragma unroll
        for (int k = 0; k < kP; ++k) {
          f4v y = ryv[j][i][k];
          if (kRealign) {
            const uint32_t sh = a.shift & 3u;
            const f4v A = y;
            f4v M;
            M.x = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, A.x), 0x101, 0xf, 0xf, false));
            M.y = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, A.y), 0x101, 0xf, 0xf, false));
            M.z = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, A.z), 0x101, 0xf, 0xf, false));
            M.w = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, A.w), 0x101, 0xf, 0xf, false));
            const f4v N = (lane & 7) == 7 ? rnv[j][i][k] : M;
            if (sh == 1) y = f4v{A.y, A.z, A.w, N.x};
            else if (sh == 2) y = f4v{A.z, A.w, N.x, N.y};
            else if (sh == 3) y = f4v{A.w, N.x, N.y, N.z};
          }
          acc += kXB ? (y - rbv[j][i]) * rxv[j][i] : y;
        }
      }
      const uint32_t nxt = t + j + kD;
      issue(j, nxt < nst ? nxt : uint32_t(nst));
      if (kSync) __builtin_amdgcn_s_barrier();
    }
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) a.sink[blockIdx.x] = acc.x;
}

static size_t g_lds = 0;  // dynamic LDS per workgroup (96 KiB: one workgroup per CU, as the product kernel)

template <int kP, int kC, int kW, int kIt, int kD, bool kXB, int kAuxY = 0, bool kSync = false, int kRange = 0, bool kXBcg = false, bool kRealign = false>
int run(const char* name, Args a, int reps, uint64_t uniq_bytes) {
  constexpr int kGroups = kRange ? kRange : 64 / kC;
  uint32_t pgs = uint32_t((a.n_pairs + kP - 1) / kP);
  pgs = (pgs + 7) / 8 * 8;
  const dim3 grid(pgs * kGroups), block(64 * kW);
  auto kern = stream_kernel<kP, kC, kW, kIt, kD, kXB, kAuxY, kSync, kRange, kXBcg, kRealign>;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, grid, block, g_lds, 0, a);
  CHECK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kern, grid, block, g_lds, 0, a);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  const double med = ts[ts.size() / 2];
  const double per_pair = double(a.nsteps) * 256;  // bytes of one flat vector
  const double cu_side = double((a.n_pairs + kP - 1) / kP) * (kP + (kXB ? 2 : 0)) * per_pair;
  printf("{\"shape\": \"%s\", \"kP\": %d, \"kC\": %d, \"kW\": %d, \"kIt\": %d, \"kD\": %d, \"xb\": %d, \"sync\": %d, "
         "\"range\": %d, \"xbcg\": %d, \"realign\": %d, \"lds\": %zu, \"shift\": %u, \"grid\": %u, \"ms\": %.4f, \"GBps_unique\": %.1f, \"GBps_cu_side\": %.1f}\n",
         name, kP, kC, kW, kIt, kD, int(kXB), int(kSync), kRange, int(kXBcg), int(kRealign), g_lds, a.shift, grid.x, med,
         uniq_bytes / (med * 1e-3) / 1e9, cu_side / (med * 1e-3) / 1e9);
  fflush(stdout);
  return 0;
}

int main() {
  const int n_pairs = 128, reps = 10;  // the product: 128 client pairs, g . g rides in pair group 0
  const uint64_t n = 11183552;  // ResNet-18's fp32 elements, a multiple of 64
  const uint64_t n_arena = n + 64;
  float *x, *b, *ys, **yp;
  CHECK(hipMalloc(&x, n * 8 + 4096));  // also the [cg][block/8][x | b] form
  CHECK(hipMalloc(&b, n_arena * 4));
  CHECK(hipMalloc(&ys, uint64_t(n_pairs) * n_arena * 4));
  CHECK(hipMalloc(&yp, n_pairs * sizeof(float*)));
  CHECK(hipMemset(x, 0, n * 8 + 4096));
  CHECK(hipMemset(b, 0, n_arena * 4));
  CHECK(hipMemset(ys, 0, uint64_t(n_pairs) * n_arena * 4));
  std::vector<float*> h(n_pairs);
  for (int k = 0; k < n_pairs; ++k) h[k] = ys + uint64_t(k) * n_arena;
  CHECK(hipMemcpy(yp, h.data(), n_pairs * sizeof(float*), hipMemcpyHostToDevice));
  float* sink;
  CHECK(hipMalloc(&sink, 1 << 20));
  Args a{x, b, yp, n / 64, n_arena, 0, n_pairs, sink};
  const uint64_t uniq = uint64_t(n_pairs + 2) * n * 4;
  g_lds = 96 << 10;
  for (uint32_t sh : {0u, 1u}) {
    a.shift = sh;
    if (run<1, 32, 8, 2, 2, true, 0, true, 0, true>("xbcg_p1", a, reps, uniq)) return 1;
    if (run<2, 16, 8, 2, 2, true, 0, true, 0, true>("xbcg_p2", a, reps, uniq)) return 1;
    if (run<4, 8, 8, 2, 2, true, 0, true, 0, true>("xbcg_p4", a, reps, uniq)) return 1;
    if (run<1, 32, 8, 4, 2, true, 0, true, 0, true>("xbcg_p1_it4", a, reps, uniq)) return 1;
    if (run<2, 16, 8, 4, 2, true, 0, true, 0, true>("xbcg_p2_it4", a, reps, uniq)) return 1;
    if (run<4, 8, 8, 4, 2, true, 0, true, 0, true>("xbcg_p4_it4", a, reps, uniq)) return 1;
    if (run<1, 32, 12, 2, 2, true, 0, true, 0, true>("xbcg_p1_w12", a, reps, uniq)) return 1;
    if (run<2, 16, 12, 2, 2, true, 0, true, 0, true>("xbcg_p2_w12", a, reps, uniq)) return 1;
  }
  return 0;
}
