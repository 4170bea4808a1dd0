// Microbenchmark: does an LDS read with only 8 lanes active cost less LDS
// bandwidth than the same read with the full wave active?  (The FedAtt-norm
// chain wave reads each step's 8 chain values with all 64 lanes, lanes 8..63
// duplicating lanes 0..7.)  Many single-wave workgroups per CU issue
// independent reads; reports per-CU LDS cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0: b32 full wave, 1: b32 lanes<8, 2: b128 full wave, 3: b128 lanes<8
__global__ __launch_bounds__(64) void lds_reads(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float tile[4096];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4096; i += 64) tile[i] = float(i & 255);
  __syncthreads();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
    const int base = (it * 64) & 4095;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (MODE == 0 || MODE == 1) {
        float v = 0.f;
        if (MODE == 0 || lane < 8) v = tile[(base + u * 8 + (lane & 7)) & 4095];
        acc.x += v;
      } else {
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (MODE == 2 || lane < 8) v = *reinterpret_cast<const f4*>(&tile[(base + u * 32 + 4 * (lane & 7)) & 4095]);
        acc += v;
      }
    }
  }
  out[blockIdx.x * 64 + lane] = acc.x + acc.y + acc.z + acc.w;
}

template <int MODE>
void run(float* out, int blocks, int iters) {
  lds_reads<MODE><<<blocks, 64>>>(out, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  lds_reads<MODE><<<blocks, 64>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const double cus = prop.multiProcessorCount, clk = prop.clockRate * 1e3;  // Hz
  const double reads_per_cu = double(blocks) * iters * 8 / cus;
  printf("mode=%d (%s, %s) blocks=%d: %.3f ms, %.2f CU-cycles per wave read\n", MODE,
         MODE < 2 ? "ds_read_b32" : "ds_read_b128", (MODE & 1) ? "8 lanes" : "64 lanes", blocks, ms,
         ms * 1e-3 * clk / reads_per_cu);
}

int main() {
  float* out;
  const int blocks = 256 * 16;
  (void)hipMalloc(&out, size_t(blocks) * 64 * 4);
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, blocks, iters);
    run<1>(out, blocks, iters);
    run<2>(out, blocks, iters);
    run<3>(out, blocks, iters);
  }
  return 0;
}
