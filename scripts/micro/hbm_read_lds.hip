// Streaming-read ceiling of the FedAvg access shape ("K streams": every
// workgroup reads the same chunk of K separate arenas) with LDS-DMA
// (global_load_lds_dwordx4, no VGPRs per load) against register loads
// (global_load_dwordx4).  Question: does an LDS-DMA ring stream HBM faster
// than the register form the FedAvg kernel uses (MI355X_MICROARCH.md: an
// all-LDS-DMA prologue burst reads at ~12-13 B/cyc/CU vs ~11 for mixed loads)?
//
// dma<U, D>: each wave owns 64 float4 groups (1 KiB per arena); per batch it
// issues U LDS-DMA loads (clients i..i+U-1) into ring slot (batch mod D), keeps
// D-1 batches in flight, waits for the oldest with a counted vmcnt, then reads
// the slot back with ds_read_b128 and sums (the consumption the kernel would do).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gf4;
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int U, bool NT>
__global__ void k_streams(const f4* __restrict__ base, f4* __restrict__ sink, uint64_t n4, int K) {
  const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n4) return;
  f4 acc = {0, 0, 0, 0};
  for (int i = 0; i < K; i += U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4* p = base + uint64_t(i + u) * n4 + g;
      v[u] = NT ? __builtin_nontemporal_load((gf4*)p) : *((gf4*)p);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x == 1234.5f) sink[0] = acc;
}

template <int WAVES, int U, int D>
__global__ __launch_bounds__(WAVES * 64) void dma(const f4* __restrict__ base, f4* __restrict__ sink, uint64_t n4,
                                                 int K) {
  __shared__ f4 ring[WAVES][D][U][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;  // whole waves only (n4 % 64 == 0)
  const uint64_t gw = g - lane;
  if (gw >= n4) return;
  const int nb = K / U;
  f4 acc = {0, 0, 0, 0};
  auto issue = [&](int b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4* p = base + uint64_t(b * U + u) * n4 + g;
      __builtin_amdgcn_global_load_lds((gvoid*)p, (lvoid*)&ring[wave][b % D][u][0], 16, 0, 0);
    }
  };
#pragma unroll
  for (int b = 0; b < D - 1; ++b)
    if (b < nb) issue(b);
  for (int b = 0; b < nb; ++b) {
    if (b + D - 1 < nb) {
      issue(b + D - 1);
      wait_vmcnt<U * (D - 1)>();
    } else {
      wait_vmcnt<0>();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += ring[wave][b % D][u][lane];
  }
  if (acc.x == 1234.5f) sink[0] = acc;
}

template <class F>
double time_ms(F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();
  (void)hipDeviceSynchronize();
  std::vector<float> ts;
  for (int r = 0; r < 9; ++r) {
    (void)hipEventRecord(e0);
    f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int K = 128;
  const uint64_t per = 11183616;  // ResNet-18 fp32 arena, padded to 64
  const uint64_t n4 = per / 4;     // multiple of 64
  const uint64_t total4 = n4 * K;
  f4 *buf, *sink;
  if (hipMalloc(&buf, total4 * 16) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, total4 * 16);
  const double gb = double(total4) * 16 / 1e9;
  printf("buffer %.2f GB\n", gb);
  for (int rep = 0; rep < 2; ++rep) {
    for (int bs : {256, 512}) {
      const uint32_t nblk = uint32_t((n4 + bs - 1) / bs);
      double ms = time_ms([&] { k_streams<8, true><<<nblk, bs>>>(buf, sink, n4, K); });
      printf("regs nt U8 bs=%d: %.1f GB/s\n", bs, gb / ms * 1e3);
    }
    {
      const uint32_t nblk = uint32_t((n4 + 255) / 256);
      double ms = time_ms([&] { dma<4, 8, 2><<<nblk, 256>>>(buf, sink, n4, K); });
      printf("dma waves4 U8 D2: %.1f GB/s\n", gb / ms * 1e3);
      ms = time_ms([&] { dma<4, 8, 3><<<nblk, 256>>>(buf, sink, n4, K); });
      printf("dma waves4 U8 D3: %.1f GB/s\n", gb / ms * 1e3);
      ms = time_ms([&] { dma<4, 4, 4><<<nblk, 256>>>(buf, sink, n4, K); });
      printf("dma waves4 U4 D4: %.1f GB/s\n", gb / ms * 1e3);
      ms = time_ms([&] { dma<4, 16, 2><<<nblk, 256>>>(buf, sink, n4, K); });
      printf("dma waves4 U16 D2: %.1f GB/s\n", gb / ms * 1e3);
      ms = time_ms([&] { dma<4, 8, 4><<<nblk, 256>>>(buf, sink, n4, K); });
      printf("dma waves4 U8 D4: %.1f GB/s\n", gb / ms * 1e3);
    }
    {
      const uint32_t nblk = uint32_t((n4 + 511) / 512);
      double ms = time_ms([&] { dma<8, 8, 2><<<nblk, 512>>>(buf, sink, n4, K); });
      printf("dma waves8 U8 D2: %.1f GB/s\n", gb / ms * 1e3);
      ms = time_ms([&] { dma<8, 4, 3><<<nblk, 512>>>(buf, sink, n4, K); });
      printf("dma waves8 U4 D3: %.1f GB/s\n", gb / ms * 1e3);
    }
  }
  return 0;
}
