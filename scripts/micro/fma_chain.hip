// Microbenchmark: cost of one dependent fp32 fma chain per lane (the shape of
// the FedAtt norm chains), register operands.  mode 0: every lane runs the
// chain; mode 1: only lanes < active run it (exec-masked).  Reports wall ns
// per step, shader-clock ticks (s_memtime) and 100 MHz ticks (s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(const float* in, float* out, long long* cyc, int steps, int active, int mode) {
  const int lane = threadIdx.x & 63;
  float v[16];
  for (int q = 0; q < 16; ++q) v[q] = in[q + lane];
  float acc = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  if (mode == 0 || lane < active) {
    for (int s = 0; s < steps; s += 16) {
#pragma unroll
      for (int q = 0; q < 16; ++q) acc = __builtin_fmaf(v[q], v[q], acc);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 64 + lane] = acc;
  if (lane == 0) {
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  float *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 1024 * 4);
  (void)hipMalloc(&out, 4096 * 64 * 4);
  (void)hipMalloc(&cyc, 4096 * 16);
  (void)hipMemset(in, 0, 1024 * 4);
  const int steps = 1 << 20;
  static long long host[8192];
  for (int mode : {0, 1}) {
    for (int active : {64, 8}) {
      if (mode == 0 && active != 64) continue;
      for (int blocks : {1, 256, 1024, 2048, 4096}) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        chain<<<blocks, 64>>>(in, out, cyc, steps, active, mode);
        (void)hipEventRecord(e0);
        chain<<<blocks, 64>>>(in, out, cyc, steps, active, mode);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(host, cyc, blocks * 16, hipMemcpyDeviceToHost);
        double tk = 0, rt = 0;
        for (int b = 0; b < blocks; ++b) {
          tk += host[2 * b];
          rt += host[2 * b + 1];
        }
        tk /= blocks;
        rt /= blocks;
        printf("mode=%d active=%d blocks=%d: %.3f ms total, block %.3f ms (realtime), %.2f shader ticks/step, "
               "clock %.2f GHz\n", mode, active, blocks, ms, rt / 1e5, tk / steps, tk / (rt * 10.0));
      }
    }
  }
  return 0;
}
