// Microbenchmark: an fma chain fed from LDS in the FedAtt-norm pattern (chain
// j reads positions j, j+8, j+16, ... of a 1,024-float tile, 8 chains on the
// wave, lanes 8..63 duplicating them), blocks of 16 steps with the next
// block's reads issued first.  Reports shader cycles per step.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void lds_chain(const float* in, float* out, long long* cyc, int tiles, int variant) {
  __shared__ float tile[1024];
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 1024; i += 64) tile[i] = in[i];
  __syncthreads();
  const float* p = tile + (lane & 7);
  float acc = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < tiles; ++t) {
    if (variant == 0) {
      constexpr int kCB = 16, kNB = 128 / kCB;
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
    } else if (variant == 2) {
      // hand-scheduled: one ds_read2 of the next block in the shadow of every two chain fmas
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 cur[8], nxt[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) cur[q] = f2{p[16 * q], p[16 * q + 8]};
      const uint32_t base = uint32_t(reinterpret_cast<uintptr_t>(p));
#pragma unroll
      for (int blk = 0; blk < 8; ++blk) {
        const uint32_t nb = base + 512u * uint32_t(blk + 1 < 8 ? blk + 1 : blk);
#define RD(q) "ds_read2_b32 %" #q ", %24 offset0:" #q "*16 offset1:" #q "*16+8\n"
#define FM(q) "v_fmac_f32 %25, %" #q "_lo, ..."
        asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read2_b32 %0, %25 offset0:0 offset1:8\n"
            "v_fmac_f32 %8, %9, %9\n"
            "ds_read2_b32 %1, %25 offset0:16 offset1:24\n"
            "v_fmac_f32 %8, %10, %10\n"
            "ds_read2_b32 %2, %25 offset0:32 offset1:40\n"
            "v_fmac_f32 %8, %11, %11\n"
            "ds_read2_b32 %3, %25 offset0:48 offset1:56\n"
            "v_fmac_f32 %8, %12, %12\n"
            "ds_read2_b32 %4, %25 offset0:64 offset1:72\n"
            "v_fmac_f32 %8, %13, %13\n"
            "ds_read2_b32 %5, %25 offset0:80 offset1:88\n"
            "v_fmac_f32 %8, %14, %14\n"
            "ds_read2_b32 %6, %25 offset0:96 offset1:104\n"
            "v_fmac_f32 %8, %15, %15\n"
            "ds_read2_b32 %7, %25 offset0:112 offset1:120\n"
            "v_fmac_f32 %8, %16, %16\n"
            "v_fmac_f32 %8, %17, %17\n"
            "v_fmac_f32 %8, %18, %18\n"
            "v_fmac_f32 %8, %19, %19\n"
            "v_fmac_f32 %8, %20, %20\n"
            "v_fmac_f32 %8, %21, %21\n"
            "v_fmac_f32 %8, %22, %22\n"
            "v_fmac_f32 %8, %23, %23\n"
            "v_fmac_f32 %8, %24, %24\n"
            : "=&v"(nxt[0]), "=&v"(nxt[1]), "=&v"(nxt[2]), "=&v"(nxt[3]), "=&v"(nxt[4]), "=&v"(nxt[5]),
              "=&v"(nxt[6]), "=&v"(nxt[7]), "+v"(acc)
            : "v"(cur[0].x), "v"(cur[0].y), "v"(cur[1].x), "v"(cur[1].y), "v"(cur[2].x), "v"(cur[2].y),
              "v"(cur[3].x), "v"(cur[3].y), "v"(cur[4].x), "v"(cur[4].y), "v"(cur[5].x), "v"(cur[5].y),
              "v"(cur[6].x), "v"(cur[6].y), "v"(cur[7].x), "v"(cur[7].y), "v"(nb)
            : "memory");
#pragma unroll
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      // no prefetch structure: plain loop, compiler schedules
#pragma unroll 16
      for (int u = 0; u < 128; ++u) {
        const float v = p[8 * u];
        acc = __builtin_fmaf(v, v, acc);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 4096 * 4);
  (void)hipMalloc(&out, 4096 * 64 * 4);
  (void)hipMalloc(&cyc, 4096 * 8);
  (void)hipMemset(in, 0, 4096 * 4);
  const int tiles = 2048;
  for (int variant : {0, 1, 2}) {
    for (int blocks : {1, 256, 1024}) {
      lds_chain<<<blocks, 64>>>(in, out, cyc, tiles, variant);
      (void)hipDeviceSynchronize();
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      lds_chain<<<blocks, 64>>>(in, out, cyc, tiles, variant);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      long long c;
      (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("variant=%d blocks=%d: %.3f ms, %.2f cycles/step\n", variant, blocks, ms, double(c) / (tiles * 128.0));
    }
  }
  return 0;
}
