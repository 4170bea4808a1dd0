// decode.hip — coded client payloads (and the baseline) as fp32 rows of the promoted layout, gfx950.
// C ABI: include/plato_agg.h (plato_agg_decode_rows).
//
// The reference dequantizes coded payloads in its inbound processor before any
// server runs: model_dequantize (plato/processors/model_dequantize.py:15-18)
// casts every bf16 entry to float32, model_dequantize_qsgd
// (plato/processors/model_dequantize_qsgd.py:34-60) decodes
// x = fp32(fp32(fp32(zeta) * max_v) / (level - 1)) for every entry.  Every
// entry — the num_batches_tracked counters included — is then float32, so the
// variant servers' deltas of a counter are float32(x) - float32(b) (torch's
// fp32 - int64 promotion).  The plain FedAvg launches keep the codes in HBM and
// decode in registers (fedavg_agg.hip, qsgd.hip); the per-entry reductions of
// the variant servers (FedAtt, FedAdp, Polaris, Port) run on rows decoded here
// once per round, in the "promoted" layout where the counters are fp32 entries
// placed after the fp32 region (plato_amd.arena.ArenaLayout.promoted).  The
// baseline goes through the same kernel (codec NATIVE: fp32 copied, int64
// counters cast to fp32 with round-to-nearest-even, as the promotion does).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "common.h"
#include "plato_agg.h"

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;

namespace {

struct DecArgs {
  int codec;
  const void* const* src_f;  // K sources: fp32 region (fp32 / bf16 / code bytes)
  const void* const* src_i;  // K sources: int64 region (int64 / bf16 / code bytes)
  const float* mv;           // QSGD: [n_entries][K] max_v
  float divisor;             // QSGD: level - 1
  const plato_agg_chunk* cf;
  const plato_agg_chunk* ci;
  uint32_t ncf, nci;
  uint64_t i64_dst;          // where the int64 region starts in a destination row
  float* const* dst;         // K destination rows (fp32)
  int K;
};

// model_dequantize_qsgd.py:51-58: byte -> zeta (sign-magnitude), then the fp32 chain
__device__ __forceinline__ float qsgd_value(uint32_t byte, float max_v, float divisor) {
  const int z = byte >= 128 ? -int(byte - 128) : int(byte);
  return (float(z) * max_v) / divisor;
}

template <int CODEC, bool I64>
__device__ __forceinline__ float dec_value(const void* src, uint64_t e, float max_v, float divisor) {
  if (CODEC == PLATO_AGG_DECODE_NATIVE) {
    if (I64) return float(static_cast<const int64_t*>(src)[e]);  // RNE, as torch's fp32 - int64 promotion
    return static_cast<const float*>(src)[e];
  } else if (CODEC == PLATO_AGG_DECODE_BF16) {
    return __uint_as_float(uint32_t(static_cast<const uint16_t*>(src)[e]) << 16);  // exact widening
  } else {
    return qsgd_value(static_cast<const uint8_t*>(src)[e], max_v, divisor);
  }
}

// One workgroup per (chunk, client): the chunk's elements, consecutive on consecutive lanes.
template <int CODEC>
__global__ __launch_bounds__(256) void decode_rows_kernel(DecArgs a) {
  const uint32_t c = blockIdx.x, k = blockIdx.y;
  const bool i64 = c >= a.ncf;
  const plato_agg_chunk ch = i64 ? a.ci[c - a.ncf] : a.cf[c];
  const float mv = CODEC == PLATO_AGG_DECODE_QSGD ? a.mv[uint64_t(ch.entry) * a.K + k] : 0.f;
  float* out = a.dst[k] + (i64 ? a.i64_dst : 0);
  if (!i64) {
    const void* src = a.src_f[k];
    for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += 256)
      out[e] = dec_value<CODEC, false>(src, e, mv, a.divisor);
  } else {
    const void* src = a.src_i[k];
    for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += 256)
      out[e] = dec_value<CODEC, true>(src, e, mv, a.divisor);
  }
}

}  // namespace

extern "C" {

int plato_agg_decode_rows(int codec, const void* const* d_src_f32, const void* const* d_src_i64, int K,
                          const float* d_max_v, float divisor, const plato_agg_chunk* d_chunks_f32,
                          uint32_t n_chunks_f32, const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                          size_t i64_dst_offset, float* const* d_dst, hipStream_t stream) {
  if (K <= 0 || K > 65535) return set_error(PLATO_AGG_EINVAL, "K must be in [1, 65535]");
  if (codec < PLATO_AGG_DECODE_NATIVE || codec > PLATO_AGG_DECODE_QSGD) return set_error(PLATO_AGG_EINVAL, "bad codec");
  if (!d_dst || (n_chunks_f32 && (!d_src_f32 || !d_chunks_f32)) || (n_chunks_i64 && (!d_src_i64 || !d_chunks_i64)))
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (codec == PLATO_AGG_DECODE_QSGD && (!d_max_v || !(divisor != 0.f)))
    return set_error(PLATO_AGG_EINVAL, "QSGD needs max_v and a non-zero divisor (level - 1)");
  const uint64_t nc = uint64_t(n_chunks_f32) + n_chunks_i64;
  if (nc == 0) return clear_error();
  if (nc > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "bad chunk count");
  DecArgs a{};
  a.codec = codec;
  a.src_f = d_src_f32;
  a.src_i = d_src_i64;
  a.mv = d_max_v;
  a.divisor = divisor;
  a.cf = d_chunks_f32;
  a.ci = d_chunks_i64;
  a.ncf = n_chunks_f32;
  a.nci = n_chunks_i64;
  a.i64_dst = i64_dst_offset;
  a.dst = d_dst;
  a.K = K;
  const dim3 grid{uint32_t(nc), uint32_t(K)};
  if (codec == PLATO_AGG_DECODE_NATIVE)
    hipLaunchKernelGGL(decode_rows_kernel<PLATO_AGG_DECODE_NATIVE>, grid, dim3(256), 0, stream, a);
  else if (codec == PLATO_AGG_DECODE_BF16)
    hipLaunchKernelGGL(decode_rows_kernel<PLATO_AGG_DECODE_BF16>, grid, dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(decode_rows_kernel<PLATO_AGG_DECODE_QSGD>, grid, dim3(256), 0, stream, a);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string("decode_rows launch: ") + hipGetErrorString(err));
  return clear_error();
}

}  // extern "C"
