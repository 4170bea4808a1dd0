// HBM streaming-read ceiling on MI355X for access shapes the FedAvg kernel
// could take: contiguous grid-stride reads vs "K streams" (each workgroup reads
// the same chunk of K separate arenas, as the FedAvg kernel does), block size,
// loads in flight per lane, non-temporal or plain, XCD-contiguous chunk order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const f4 gf4;

template <int U, bool NT>
__global__ void grid_stride(const f4* __restrict__ src, f4* __restrict__ sink, uint64_t n4) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load((gf4*)src + i + u * stride) : *((gf4*)src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x == 1234.5f) sink[0] = acc;
}

// K arenas of n4 groups each; workgroup b owns group range [b*B, (b+1)*B) of every arena.
template <int U, bool NT, bool XCD>
__global__ void k_streams(const f4* __restrict__ base, f4* __restrict__ sink, uint64_t n4, int K, uint32_t nblk) {
  uint32_t b = blockIdx.x;
  if (XCD) {  // blocks land on XCD b % 8: give each XCD a contiguous range of chunks
    const uint32_t per = (nblk + 7) / 8;
    b = (b % 8) * per + b / 8;
    if (b >= nblk) return;
  }
  const uint64_t g = uint64_t(b) * blockDim.x + threadIdx.x;
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

template <class F>
double time_ms(F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();
  (void)hipDeviceSynchronize();
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
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
  const uint64_t n4 = per / 4;
  const uint64_t total4 = n4 * K;
  f4 *buf, *sink;
  (void)hipMalloc(&buf, total4 * 16);
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(buf, 0, total4 * 16);
  const double gb = double(total4) * 16 / 1e9;
  printf("buffer %.2f GB\n", gb);
  for (int bs : {256, 512}) {
    for (int blocks : {4096, 8192, 16384, 65536}) {
      double ms = time_ms([&] { grid_stride<8, true><<<blocks, bs>>>(buf, sink, total4); });
      printf("grid_stride nt U8 bs=%d blocks=%d: %.1f GB/s\n", bs, blocks, gb / ms * 1e3);
    }
  }
  for (int blocks : {8192, 32768}) {
    double ms = time_ms([&] { grid_stride<8, false><<<blocks, 256>>>(buf, sink, total4); });
    printf("grid_stride plain U8 bs=256 blocks=%d: %.1f GB/s\n", blocks, gb / ms * 1e3);
    ms = time_ms([&] { grid_stride<16, true><<<blocks, 256>>>(buf, sink, total4); });
    printf("grid_stride nt U16 bs=256 blocks=%d: %.1f GB/s\n", blocks, gb / ms * 1e3);
  }
  for (int bs : {256, 512, 1024}) {
    const uint32_t nblk = uint32_t((n4 + bs - 1) / bs);
    double ms = time_ms([&] { k_streams<8, true, false><<<nblk, bs>>>(buf, sink, n4, K, nblk); });
    printf("k_streams nt U8 bs=%d: %.1f GB/s\n", bs, gb / ms * 1e3);
    ms = time_ms([&] { k_streams<8, true, true><<<nblk + 8, bs>>>(buf, sink, n4, K, nblk); });
    printf("k_streams nt U8 xcd bs=%d: %.1f GB/s\n", bs, gb / ms * 1e3);
    ms = time_ms([&] { k_streams<16, true, false><<<nblk, bs>>>(buf, sink, n4, K, nblk); });
    printf("k_streams nt U16 bs=%d: %.1f GB/s\n", bs, gb / ms * 1e3);
    ms = time_ms([&] { k_streams<8, false, false><<<nblk, bs>>>(buf, sink, n4, K, nblk); });
    printf("k_streams plain U8 bs=%d: %.1f GB/s\n", bs, gb / ms * 1e3);
  }
  return 0;
}
