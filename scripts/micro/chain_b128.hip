// Microbenchmark: where the LDS-fed fma chain of port_norms_kernel / entry_norms_rs_kernel loses
// its ~1 cycle per step against a bare register chain (6 shader cycles per dependent v_fmac_f32).
// One workgroup per CU; wave 0 runs the chain exactly as the product kernels do (8 chains, lane & 7,
// a transposed row of kSteps floats per chain, 16 steps per block as 4 ds_read_b128 with the next
// block's reads in flight), over the same LDS tile again and again (no barriers), and reports shader
// cycles per step.  The other P waves of the workgroup ("noise") do, per mode:
//   0: nothing (exit at once)           1: independent VALU work (fma on private registers)
//   2: ds_write_b32 into another LDS region (the producers' transposed tile writes)
//   3: global loads streaming a buffer (the producers' loads)   4: modes 1 + 2 + 3 together
// and mode 5 runs the chain with its operands from registers only (no LDS reads) with no noise;
// kNarrow runs the chain (reads and fmas) on lanes 0..7 only (exec mask 0xff).
// Modes 8-10 (round 5) feed the chain from global memory instead of LDS: the same transposed rows in a
// per-CU 33 KB buffer (L1 / L2 resident), 8 buffer_load_dwordx4 per 32-step block with the next block's
// in flight and one s_waitcnt vmcnt per block; cache policy aux 0 (8), sc0 (9), sc0 | sc1 (10: agent
// scope, past the CU's L1 — what producer-written rows would need).
// Build: hipcc --offload-arch=gfx950 -O3 -o chain_b128 chain_b128.hip; run: ./chain_b128
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kSteps = 1024;           // steps per row (an 8,192-position tile)
constexpr int kR = kSteps + 4;         // row pitch (floats)
constexpr int kTiles = 64;             // passes over the tile

template <int kMode, bool kNarrow = false>
__global__ void chain_b128(const float* in, float* out, long long* cyc, const float* big, unsigned long long nbig) {
  __shared__ __attribute__((aligned(16))) float tile[8 * kR];
  __shared__ __attribute__((aligned(16))) float junk[8 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 8 * kR; i += blockDim.x) tile[i] = in[i % 4096] * 1e-3f;
  __syncthreads();
  volatile __shared__ int done;
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  if (wave > 0) {  // noise
    if (kMode == 0 || kMode == 5 || kMode == 7) return;
    constexpr int nm = (kMode == 6 || kMode >= 8) ? 4 : kMode;  // modes 6, 8-10: all the noise
    float a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3;
    unsigned long long g = (unsigned long long)(blockIdx.x * 1024 + wave * 64 + lane) * 4;
    float sink = 0.f;
    int it = 0;
    while (!done && it < (1 << 22)) {
      ++it;
      if (nm == 1 || nm == 4) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          a0 = __builtin_fmaf(a0, 1.0001f, 0.5f);
          a1 = __builtin_fmaf(a1, 1.0001f, 0.5f);
          a2 = __builtin_fmaf(a2, 1.0001f, 0.5f);
          a3 = __builtin_fmaf(a3, 1.0001f, 0.5f);
        }
      }
      if (nm == 2 || nm == 4) {
#pragma unroll
        for (int k = 0; k < 8; ++k) junk[(k * 1024 + (wave * 64 + lane) * 4) & (8 * 1024 - 1)] = a0 + k;
      }
      if (nm == 3 || nm == 4) {
        f4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = *reinterpret_cast<const f4*>(big + (g % (nbig - 4)));
          g += 256ull * 1024;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) sink += v[k].x;
      }
    }
    if (sink + a0 + a1 + a2 + a3 == 12345.f) out[1 + threadIdx.x] = sink;  // keeps the work live
    return;
  }
  const int j = lane & 7;
  float acc = 0.f;
  long long t0 = __builtin_amdgcn_s_memtime();
  if (kMode == 5) {
    const f4* row = reinterpret_cast<const f4*>(tile + j * kR);
    f4 r[4] = {row[0], row[1], row[2], row[3]};
    for (int t = 0; t < kTiles; ++t) {
#pragma unroll
      for (int blk = 0; blk < kSteps / 16; ++blk) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc = __builtin_fmaf(r[q].x, r[q].x, acc);
          acc = __builtin_fmaf(r[q].y, r[q].y, acc);
          acc = __builtin_fmaf(r[q].z, r[q].z, acc);
          acc = __builtin_fmaf(r[q].w, r[q].w, acc);
        }
      }
    }
  } else if (kMode == 6 || kMode == 7) {
    // 6: one s_waitcnt per 16-step block (the next block's 4 reads stay in flight), not one per f4
    // 7: the reads issued as in the product but the fmas on register values (read issue cost alone)
    for (int t = 0; t < kTiles; ++t) {
      const f4* row = reinterpret_cast<const f4*>(tile + j * kR);
      f4 buf[2][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) buf[0][q] = row[q];
      f4 keep = buf[0][0];
#pragma unroll
      for (int blk = 0; blk < kSteps / 16; ++blk) {
        const int cb = blk & 1;
        if (blk + 1 < kSteps / 16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) buf[cb ^ 1][q] = row[4 * (blk + 1) + q];
          if (kMode == 6) __builtin_amdgcn_s_waitcnt(0xc07f | (4 << 8));  // lgkmcnt(4): this block's reads done
        } else if (kMode == 6) {
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 v = kMode == 6 ? buf[cb][q] : keep;
          acc = __builtin_fmaf(v.x, v.x, acc);
          acc = __builtin_fmaf(v.y, v.y, acc);
          acc = __builtin_fmaf(v.z, v.z, acc);
          acc = __builtin_fmaf(v.w, v.w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (kMode == 7) keep.x += buf[cb][0].x * 0.f;  // the reads stay live
      }
    }
  } else if (kMode >= 8 && kMode <= 10) {
    constexpr int kAux = kMode == 8 ? 0 : kMode == 9 ? 1 : 17;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(big + (unsigned long long)blockIdx.x * 8 * kR), (short)0, 8 * kR * 4, 0x00020000);
    const unsigned rowb = unsigned(j * kR) * 4u;
    for (int t = 0; t < kTiles; ++t) {
      f4 buf[2][8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        buf[0][q] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, rowb + 16u * q, 0, kAux));
#pragma unroll
      for (int blk = 0; blk < kSteps / 32; ++blk) {
        const int cb = blk & 1;
        if (blk + 1 < kSteps / 32) {
#pragma unroll
          for (int q = 0; q < 8; ++q)
            buf[cb ^ 1][q] = __builtin_bit_cast(
                f4, __builtin_amdgcn_raw_buffer_load_b128(rs, rowb + 16u * (8 * (blk + 1) + q), 0, kAux));
          __builtin_amdgcn_s_waitcnt(8 | (7 << 4) | (15 << 8));  // vmcnt(8): this block's loads landed
        } else {
          __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));  // vmcnt(0)
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          acc = __builtin_fmaf(buf[cb][q].x, buf[cb][q].x, acc);
          acc = __builtin_fmaf(buf[cb][q].y, buf[cb][q].y, acc);
          acc = __builtin_fmaf(buf[cb][q].z, buf[cb][q].z, acc);
          acc = __builtin_fmaf(buf[cb][q].w, buf[cb][q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else if (!kNarrow || lane < 8) {  // kNarrow: the chain (reads and fmas) on lanes 0..7 only
    for (int t = 0; t < kTiles; ++t) {
      const f4* row = reinterpret_cast<const f4*>(tile + j * kR);
      f4 cur4[4], nxt4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) cur4[q] = row[q];
#pragma unroll
      for (int blk = 0; blk < kSteps / 16; ++blk) {
        if (blk + 1 < kSteps / 16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) nxt4[q] = row[4 * (blk + 1) + q];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc = __builtin_fmaf(cur4[q].x, cur4[q].x, acc);
          acc = __builtin_fmaf(cur4[q].y, cur4[q].y, acc);
          acc = __builtin_fmaf(cur4[q].z, cur4[q].z, acc);
          acc = __builtin_fmaf(cur4[q].w, cur4[q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) cur4[q] = nxt4[q];
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) done = 1;
  if (lane == 0) {
    out[blockIdx.x] = acc;
    cyc[blockIdx.x] = t1 - t0;
  }
}

template <int kMode, bool kNarrow = false>
double run(int P, const float* in, float* out, long long* cyc, const float* big, unsigned long long nbig) {
  hipLaunchKernelGGL((chain_b128<kMode, kNarrow>), dim3(256), dim3(64 * (1 + P)), 0, 0, in, out, cyc, big, nbig);
  hipDeviceSynchronize();
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256; ++i) s += double(h[i]);
  return s / 256 / (double(kTiles) * kSteps);
}

int main() {
  float *in, *out, *big;
  long long* cyc;
  const unsigned long long nbig = 1ull << 28;  // 1 GiB of floats streamed by the loading noise
  hipMalloc(&in, 4096 * sizeof(float));
  hipMalloc(&out, 4096 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  hipMalloc(&big, nbig * sizeof(float));
  hipMemset(in, 0, 4096 * sizeof(float));
  hipMemset(big, 0, nbig * sizeof(float));
  for (int rep = 0; rep < 2; ++rep) {
    printf("global rows (aux 0 / sc0 / sc0|sc1), no noise: %.2f / %.2f / %.2f; P=8 all: %.2f / %.2f / %.2f cycles/step\n",
           run<8>(0, in, out, cyc, big, nbig), run<9>(0, in, out, cyc, big, nbig), run<10>(0, in, out, cyc, big, nbig),
           run<8>(8, in, out, cyc, big, nbig), run<9>(8, in, out, cyc, big, nbig), run<10>(8, in, out, cyc, big, nbig));
    printf("registers only, no noise: %.2f cycles/step\n", run<5>(0, in, out, cyc, big, nbig));
    printf("one s_waitcnt per block, no noise: %.2f; P=8 all: %.2f cycles/step\n", run<6>(0, in, out, cyc, big, nbig),
           run<6>(8, in, out, cyc, big, nbig));
    printf("reads issued, fmas on registers, no noise: %.2f cycles/step\n", run<7>(0, in, out, cyc, big, nbig));
    for (int P : {0, 4, 8}) {
      printf("P=%d  none %.2f  valu %.2f  ds_write %.2f  loads %.2f  all %.2f  cycles/step\n", P,
             run<0>(P, in, out, cyc, big, nbig), run<1>(P, in, out, cyc, big, nbig), run<2>(P, in, out, cyc, big, nbig),
             run<3>(P, in, out, cyc, big, nbig), run<4>(P, in, out, cyc, big, nbig));
      printf("P=%d  lanes 0-7 only:  none %.2f  valu %.2f  ds_write %.2f  loads %.2f  all %.2f  cycles/step\n", P,
             run<0, true>(P, in, out, cyc, big, nbig), run<1, true>(P, in, out, cyc, big, nbig),
             run<2, true>(P, in, out, cyc, big, nbig), run<3, true>(P, in, out, cyc, big, nbig),
             run<4, true>(P, in, out, cyc, big, nbig));
    }
  }
  return 0;
}
