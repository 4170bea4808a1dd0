// qsgd.hip — FedAvg over QSGD-coded client payloads, dequantized in registers
// (server inbound codecs on the device).
//
// Plato's QSGD pair (plato/processors/model_quantize_qsgd.py:95-139,
// model_dequantize_qsgd.py:34-60) sends one byte per element (bit 7 sign,
// bits 0-6 |zeta|) plus one fp32 max_v per entry, and the server decodes
//     x = fp32(fp32(fp32(zeta) * max_v) / (level - 1))
// before FedAvg.  Here the payload stays one byte per element through PCIe
// and HBM (client traffic / 4 vs fp32), and each workgroup — one chunk of one
// entry, so max_v is workgroup-uniform — builds a 256-entry decode table per
// client in LDS with the exact (IEEE) division, then every element-client is
// one LDS lookup: the division is paid 256 times per (client, chunk) instead
// of once per element.  The FedAvg arithmetic after decoding is the same
// separately rounded chain as fedavg_agg.hip (int64 entries: the decoded fp32
// value minus fp32(b), as torch promotes fp32 - int64).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include <type_traits>

#include "common.h"
#include "plato_agg.h"
#include "plato_agg_tune.h"

namespace {

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));
typedef unsigned int u1 __attribute__((ext_vector_type(1)));
typedef __attribute__((address_space(1))) const f4 gf4;
typedef __attribute__((address_space(1))) f4 gf4w;
typedef __attribute__((address_space(1))) const u4 gu4;
typedef __attribute__((address_space(1))) const u2 gu2;
typedef __attribute__((address_space(1))) const u1 gu1;

// Kernel shape (tuning space, plato_agg_tune_fedavg_qsgd): B threads per
// workgroup share each batch's decode tables, U clients per table batch, G
// elements per lane (one 16/8/4-byte code load per client).  The default
// (round 6, tuning variant 29) is the plain form (two barriers per table batch) at B = 256, U = 4 and
// two 8-element groups per lane (4,096-element chunks), tables built with the float64 reciprocal
// product, max_v by scalar loads and each batch's codes issued before its table build: 0.290 ms
// interleaved on one box against 0.308 for the round-5 default (B = 256, U = 8, one group; variant 0),
// 0.333 for the round-1 plain form (variant 5) and 0.373 for the pipelined form of rounds 2-3
// (variant 1); DESIGN.md §11, §14, §15.
constexpr int kG = 16;      // elements per lane group of the plain kernel's template default

template <class T>
__device__ __forceinline__ T sld(const T* p, uint64_t i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

struct QArgs {
  const uint8_t* const* cf;   // K code arenas (fp32 region, one byte per element)
  const uint8_t* const* ci;   // K code arenas (int64 region)
  const float* mv;            // [n_entries][K] max_v
  const float* w;             // [K]
  const float* s;             // [K] or null
  const plato_agg_chunk* tf;
  const plato_agg_chunk* ti;
  const float* base_f;
  const int64_t* base_i;
  float* out_f;
  float* out_if;
  uint64_t n_f32, n_i64;
  uint32_t ncf, nci;
  float divisor;
  int K;
};

struct Chunk {
  uint32_t entry, begin, end;
};

__device__ __forceinline__ Chunk load_chunk(const plato_agg_chunk* t, uint32_t c, uint64_t n) {
  const uint32_t* p = reinterpret_cast<const uint32_t*>(t + c);
  Chunk ch{sld(p, 0), sld(p, 1), sld(p, 2)};
  if (ch.end > n) ch.end = uint32_t(n);
  if (ch.begin > ch.end) ch.begin = ch.end;
  return ch;
}

// model_dequantize_qsgd.py:51-58: byte -> zeta (sign-magnitude), then the fp32 chain
__device__ __forceinline__ float decode(uint32_t byte, float max_v, float divisor) {
  const int z = byte >= 128 ? -int(byte - 128) : int(byte);
  return (float(z) * max_v) / divisor;
}

__device__ __forceinline__ float term(float x, float b, float w, float s, bool two) {
  float t = (x - b) * w;
  if (two) t = t * s;
  return t;
}

// kAbs: the decode table holds |zeta| = 0..127 only (128 entries per client) and the code's sign bit is
// flipped into the decoded value's bit 31 (round-to-nearest is sign-symmetric: decode(128 + z) =
// -decode(z) for z != 0).  Code 128 (zeta = -0, the integer 0) then decodes to -decode(0) instead of
// decode(0): a zero of the other sign (or a NaN of the other sign when max_v is not finite), which
// cannot change any result bit — x - b with x = -0 or +0 differs only for b = +-0, where it is +-0 again,
// and the accumulator, which starts at +0 and only becomes zero again by an exact cancellation (+0),
// absorbs a zero term of either sign (NaN payloads are not compared).  Halving the table
// puts the frequent small |zeta| of both signs on one address (a broadcast) instead of two addresses in
// one bank: the lookups' LDS bank conflicts fall from ~2.1 extra cycles per ds_read_b32 (SQ counters,
// profiles/r06c_qsgd_pmc.json) to the ~0.5 a 128-entry table's random collisions cost.
template <int kBlock, int kU, bool TWO, int kG = ::kG, bool kSM = false, bool kAbs = false>
__device__ void qsgd_f32_chunk(const QArgs& a, uint32_t c, float (*lut)[kAbs ? 128 : 256]) {
  static_assert(kG == 16 || kG == 8 || kG == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG, g1 = (uint64_t(ch.end) + kG - 1) / kG;
  const int K = a.K;
  for (uint64_t gp = g0; gp < g1; gp += kBlock) {  // one pass for chunks <= 8192 elements
    const uint64_t g = gp + threadIdx.x;
    const bool have = g < g1;
    const uint64_t e0 = g * kG;
    const bool full = have && e0 >= ch.begin && e0 + kG <= ch.end;
    float b[kG], acc[kG];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      acc[q] = 0.f;
      b[q] = 0.f;
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = *((gf4*)(a.base_f + e0) + q);
        b[4 * q] = v.x;
        b[4 * q + 1] = v.y;
        b[4 * q + 2] = v.z;
        b[4 * q + 3] = v.w;
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) b[q] = a.base_f[e];
      }
    }
    using CodeT = std::conditional_t<kG == 16, u4, std::conditional_t<kG == 8, u2, u1>>;
    using GCodeT = std::conditional_t<kG == 16, gu4, std::conditional_t<kG == 8, gu2, gu1>>;
    for (int i0 = 0; i0 < K; i0 += kU) {
      const int nu = K - i0 < kU ? K - i0 : kU;
      __syncthreads();  // previous batch's lookups are done
      CodeT code[kU];
      if (kSM && full) {  // the batch's codes in flight during its table build and barrier
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int i = i0 + u < K ? i0 + u : K - 1;
          code[u] = __builtin_nontemporal_load((GCodeT*)(sld(a.cf, i) + e0));
        }
      }
      // codes 128 + z decode to exactly -decode(z) (round-to-nearest is sign-symmetric),
      // except 128 itself: zeta = -0 is the integer 0
      for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
            // kSM: u is wave-uniform (128 table slots per client, 64 lanes per wave): max_v by a scalar load
        const int u = kSM ? __builtin_amdgcn_readfirstlane(t >> 7) : t >> 7, z = t & 127;
        if (u < nu) {
          const float v = decode(uint32_t(z), sld(mrow, i0 + u), a.divisor);
          lut[u][z] = v;
          if (!kAbs) lut[u][z + 128] = z ? -v : v;
        }
      }
      __syncthreads();
      if (full) {
        if (!kSM) {
#pragma unroll
          for (int u = 0; u < kU; ++u) {
            const int i = i0 + u < K ? i0 + u : K - 1;
            code[u] = __builtin_nontemporal_load((GCodeT*)(sld(a.cf, i) + e0));
          }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (u < nu) {
            const float wu = sld(a.w, i0 + u);
            const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
            for (int q = 0; q < kG; ++q) {
              const uint32_t word = code[u][q >> 2];
              float x;
              if (kAbs) {
                const uint32_t sbit = (word << (24 - 8 * (q & 3))) & 0x80000000u;
                x = __uint_as_float(__float_as_uint(lut[u][(word >> (8 * (q & 3))) & 127u]) ^ sbit);
              } else {
                x = lut[u][(word >> (8 * (q & 3))) & 255u];
              }
              acc[q] = acc[q] + term(x, b[q], wu, su, TWO);
            }
          }
        }
      } else if (have) {
        for (int u = 0; u < nu; ++u) {
          const uint8_t* p = sld(a.cf, i0 + u);
          const float wu = sld(a.w, i0 + u);
          const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
          for (int q = 0; q < kG; ++q) {
            const uint64_t e = e0 + q;
            if (e >= ch.begin && e < ch.end) {
              const uint32_t byte = p[e];
              const float x = kAbs ? __uint_as_float(__float_as_uint(lut[u][byte & 127u]) ^ ((byte & 128u) << 24))
                                   : lut[u][byte];
              acc[q] = acc[q] + term(x, b[q], wu, su, TWO);
            }
          }
        }
      }
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = f4{b[4 * q] + acc[4 * q], b[4 * q + 1] + acc[4 * q + 1], b[4 * q + 2] + acc[4 * q + 2],
                        b[4 * q + 3] + acc[4 * q + 3]};
        __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0) + q);
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) a.out_f[e] = b[q] + acc[q];
      }
    }
  }
}

// The int64 entries' codes: K clients in order, one code load at a time.  Their chunks are the grid's
// first blocks, so these K round trips run beside the stream from its start (at the end of the grid they
// outlasted it).  Batching the loads, as the FedAvg kernel does, raised the kernel's VGPR count past the
// 64 that keep two 512-thread workgroups per CU (0.353 against 0.311 ms, profiles/r05k_qsgd.log).
template <int kBlock, bool TWO>
__device__ void qsgd_i64_chunk(const QArgs& a, uint32_t cc) {
  const Chunk ch = load_chunk(a.ti, cc, a.n_i64);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  for (uint64_t e = ch.begin + threadIdx.x; e < ch.end; e += kBlock) {
    // fp32 payload - int64 baseline promotes the baseline to fp32 (algorithms/fedavg.py:23)
    const float b = (float)a.base_i[e];
    float acc = 0.f;
    for (int i = 0; i < a.K; ++i) {
      const float x = decode(sld(a.ci, i)[e], sld(mrow, i), a.divisor);
      acc = acc + term(x, b, sld(a.w, i), TWO ? sld(a.s, i) : 1.f, TWO);
    }
    a.out_if[e] = b + acc;
  }
}

// Pipelined form: the decode tables are double-buffered and the next batch's
// codes are loaded into registers before the current batch is summed, so each
// batch costs one s_barrier and its code loads are in flight while the wave
// does the previous batch's lookups (the plain form above waits for them after
// every barrier).  The batch's weights are read before its lookups so the
// lgkmcnt waits of the lookups do not also cover scalar loads.
template <int kG2>
using CodeOf = std::conditional_t<kG2 == 16, u4, std::conditional_t<kG2 == 8, u2, u1>>;
template <int kG2>
using GCodeOf = std::conditional_t<kG2 == 16, gu4, std::conditional_t<kG2 == 8, gu2, gu1>>;

template <int kBlock, int kU>
__device__ __forceinline__ void build_tables(const QArgs& a, const float* mrow, int i0, int nu, float (*lut)[256]) {
  for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
    // u is wave-uniform (128 table slots per client, 64 lanes per wave): a scalar load of max_v,
    // so the table build never waits on the vector-memory counter of the code loads in flight
    const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;
    if (u < nu) {
      const float v = decode(uint32_t(z), sld(mrow, i0 + u), a.divisor);
      lut[u][z] = v;
      lut[u][z + 128] = z ? -v : v;
    }
  }
}

template <int kU, int kG2>
__device__ __forceinline__ void load_codes(const QArgs& a, int i0, int K, uint64_t e0, CodeOf<kG2> (&code)[kU]) {
  // element offsets fit 32 bits (run_qsgd): scalar base + 32-bit vector offset (global_load ... saddr),
  // and a batch that lies inside [0, K) loads its pointers unclamped (adjacent scalar loads merge)
  const uint32_t off = uint32_t(e0);
  if (i0 + kU <= K) {
#pragma unroll
    for (int u = 0; u < kU; ++u) code[u] = __builtin_nontemporal_load((GCodeOf<kG2>*)(sld(a.cf, i0 + u) + off));
  } else {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u < K ? i0 + u : K - 1;
      code[u] = __builtin_nontemporal_load((GCodeOf<kG2>*)(sld(a.cf, i) + off));
    }
  }
}

template <int kU, int kG2, bool TWO, bool kNoLds = false>
__device__ __forceinline__ void sum_batch(int nu, const CodeOf<kG2> (&code)[kU], const float (&wu)[kU],
                                          const float (&su)[kU], const float (*lut)[256], const float (&b)[kG2],
                                          float (&acc)[kG2]) {
  if (nu == kU) {  // every batch but a ragged last one: no per-client branches
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint32_t word = code[u][q >> 2];
        const float x = kNoLds ? float((word >> (8 * (q & 3))) & 255u) : lut[u][(word >> (8 * (q & 3))) & 255u];
        acc[q] = acc[q] + term(x, b[q], wu[u], su[u], TWO);
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (u < nu) {
#pragma unroll
        for (int q = 0; q < kG2; ++q) {
          const uint32_t word = code[u][q >> 2];
          const float x = lut[u][(word >> (8 * (q & 3))) & 255u];
          acc[q] = acc[q] + term(x, b[q], wu[u], su[u], TWO);
        }
      }
    }
  }
}

template <int kU, bool TWO>
__device__ __forceinline__ void load_weights(const QArgs& a, int i0, float (&wu)[kU], float (&su)[kU]) {
  if (i0 + kU <= a.K) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      wu[u] = sld(a.w, i0 + u);
      su[u] = TWO ? sld(a.s, i0 + u) : 1.f;
    }
  } else {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u < a.K ? i0 + u : a.K - 1;
      wu[u] = sld(a.w, i);
      su[u] = TWO ? sld(a.s, i) : 1.f;
    }
  }
}

// The plain form with its lookups software-pipelined (round 6): the counters of the default
// (profiles/r06c_qsgd_pmc.json) show each wave issuing one client's kG lookups, then waiting for all of
// them (s_waitcnt lgkmcnt(0): the scalar weight loads between the clients share the counter) before its
// arithmetic.  Here the batch's weights are loaded with its codes, ahead of the tables, so the lookups
// are the only LDS-counter operations in the batch, and client u + 1's lookups are issued before client
// u's arithmetic: each wait leaves the next client's kG reads in flight.
template <int kG, bool kAbs>
__device__ __forceinline__ void sp_lookup(const float* tab, const CodeOf<kG>& code, float (&x)[kG]) {
#pragma unroll
  for (int q = 0; q < kG; ++q) {
    const uint32_t word = code[q >> 2];
    if (kAbs) {
      const uint32_t sbit = (word << (24 - 8 * (q & 3))) & 0x80000000u;
      x[q] = __uint_as_float(__float_as_uint(tab[(word >> (8 * (q & 3))) & 127u]) ^ sbit);
    } else {
      x[q] = tab[(word >> (8 * (q & 3))) & 255u];
    }
  }
}

template <int kG, bool TWO>
__device__ __forceinline__ void sp_sum(const float (&x)[kG], const float (&b)[kG], float w, float s, float (&acc)[kG]) {
#pragma unroll
  for (int q = 0; q < kG; ++q) acc[q] = acc[q] + term(x[q], b[q], w, s, TWO);
}

template <int kBlock, int kU, bool TWO, int kG, bool kAbs>
__device__ void qsgd_f32_chunk_sp(const QArgs& a, uint32_t c, float (*lut)[kAbs ? 128 : 256]) {
  static_assert(kG == 16 || kG == 8 || kG == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG, g1 = (uint64_t(ch.end) + kG - 1) / kG;
  const int K = a.K;
  for (uint64_t gp = g0; gp < g1; gp += kBlock) {
    const uint64_t g = gp + threadIdx.x;
    const bool have = g < g1;
    const uint64_t e0 = g * kG;
    const bool full = have && e0 >= ch.begin && e0 + kG <= ch.end;
    float b[kG], acc[kG];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      acc[q] = 0.f;
      b[q] = 0.f;
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = *((gf4*)(a.base_f + e0) + q);
        b[4 * q] = v.x;
        b[4 * q + 1] = v.y;
        b[4 * q + 2] = v.z;
        b[4 * q + 3] = v.w;
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) b[q] = a.base_f[e];
      }
    }
    for (int i0 = 0; i0 < K; i0 += kU) {
      const int nu = K - i0 < kU ? K - i0 : kU;
      __syncthreads();  // previous batch's lookups are done
      CodeOf<kG> code[kU];
      if (full) load_codes<kU, kG>(a, i0, K, e0, code);  // in flight during the table build and barrier
      float wu[kU], su[kU];
      load_weights<kU, TWO>(a, i0, wu, su);
      for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
        const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;  // wave-uniform: scalar max_v
        if (u < nu) {
          const float v = decode(uint32_t(z), sld(mrow, i0 + u), a.divisor);
          lut[u][z] = v;
          if (!kAbs) lut[u][z + 128] = z ? -v : v;
        }
      }
      __syncthreads();
      if (full && nu == kU) {
        float xa[kG], xb[kG];
        sp_lookup<kG, kAbs>(lut[0], code[0], xa);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (u % 2 == 0) {
            if (u + 1 < kU) sp_lookup<kG, kAbs>(lut[u + 1], code[u + 1], xb);
            sp_sum<kG, TWO>(xa, b, wu[u], su[u], acc);
          } else {
            if (u + 1 < kU) sp_lookup<kG, kAbs>(lut[u + 1], code[u + 1], xa);
            sp_sum<kG, TWO>(xb, b, wu[u], su[u], acc);
          }
        }
      } else if (full) {  // a ragged last batch
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (u < nu) {
            float x[kG];
            sp_lookup<kG, kAbs>(lut[u], code[u], x);
            sp_sum<kG, TWO>(x, b, wu[u], su[u], acc);
          }
        }
      } else if (have) {
        for (int u = 0; u < nu; ++u) {
          const uint8_t* p = sld(a.cf, i0 + u);
#pragma unroll
          for (int q = 0; q < kG; ++q) {
            const uint64_t e = e0 + q;
            if (e >= ch.begin && e < ch.end) {
              const uint32_t byte = p[e];
              const float x = kAbs ? __uint_as_float(__float_as_uint(lut[u][byte & 127u]) ^ ((byte & 128u) << 24))
                                   : lut[u][byte];
              acc[q] = acc[q] + term(x, b[q], wu[u], su[u], TWO);
            }
          }
        }
      }
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = f4{b[4 * q] + acc[4 * q], b[4 * q + 1] + acc[4 * q + 1], b[4 * q + 2] + acc[4 * q + 2],
                        b[4 * q + 3] + acc[4 * q + 3]};
        __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0) + q);
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) a.out_f[e] = b[q] + acc[q];
      }
    }
  }
}

// Round 6, the VALU side of the plain form: a wave64 VALU instruction holds a SIMD for 4 cycles, so the
// default's 3.87 VALU instructions per 64 element-clients already keep the SIMDs ~53 % busy beside the
// LDS array's ~60 % (profiles/r06c_qsgd_pmc.json).  Two levers on it:
//  * kFastTab: the decode table built with the float64 reciprocal product (RN32(RN64(p) * RN64(1 / d))
//    = RN32(p / d) for every float pair, tests/test_division.py; fedadp.hip adp_div_lr_f64) instead of the
//    IEEE division's ~10-instruction sequence: the table build was ~a quarter of the VALU instructions;
//  * kP element groups per lane: each table batch serves kP groups of kG elements (a kP-times longer chunk
//    per workgroup), so the table build and its two barriers are paid once per kP groups.
[[maybe_unused]] __device__ __forceinline__ float decode_tab(uint32_t z, float max_v, double inv_div) {
  return float(double(float(z) * max_v) * inv_div);
}

template <int kBlock, int kU, bool TWO, int kG, int kP, bool kFastTab>
__device__ void qsgd_f32_chunk_mp(const QArgs& a, uint32_t c, float (*lut)[256]) {
  static_assert(kG == 16 || kG == 8 || kG == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG, g1 = (uint64_t(ch.end) + kG - 1) / kG;
  const int K = a.K;
  const double inv_div = 1.0 / double(a.divisor);
  for (uint64_t gp = g0; gp < g1; gp += uint64_t(kBlock) * kP) {
    uint64_t e0[kP];
    bool have[kP], full[kP];
    float b[kP][kG], acc[kP][kG];
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const uint64_t g = gp + uint64_t(p) * kBlock + threadIdx.x;
      have[p] = g < g1;
      e0[p] = g * kG;
      full[p] = have[p] && e0[p] >= ch.begin && e0[p] + kG <= ch.end;
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        acc[p][q] = 0.f;
        b[p][q] = 0.f;
      }
      if (full[p]) {
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) {
          const f4 v = *((gf4*)(a.base_f + e0[p]) + q);
          b[p][4 * q] = v.x;
          b[p][4 * q + 1] = v.y;
          b[p][4 * q + 2] = v.z;
          b[p][4 * q + 3] = v.w;
        }
      } else if (have[p]) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0[p] + q;
          if (e >= ch.begin && e < ch.end) b[p][q] = a.base_f[e];
        }
      }
    }
    for (int i0 = 0; i0 < K; i0 += kU) {
      const int nu = K - i0 < kU ? K - i0 : kU;
      __syncthreads();  // previous batch's lookups are done
      CodeOf<kG> code[kP][kU];
#pragma unroll
      for (int p = 0; p < kP; ++p)
        if (full[p]) load_codes<kU, kG>(a, i0, K, e0[p], code[p]);  // in flight during the table build
      float wu[kU], su[kU];
      load_weights<kU, TWO>(a, i0, wu, su);
      for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
        const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;  // wave-uniform: scalar max_v
        if (u < nu) {
          const float mv = sld(mrow, i0 + u);
          const float v = kFastTab ? decode_tab(uint32_t(z), mv, inv_div) : decode(uint32_t(z), mv, a.divisor);
          lut[u][z] = v;
          lut[u][z + 128] = z ? -v : v;
        }
      }
      __syncthreads();
#pragma unroll
      for (int p = 0; p < kP; ++p) {
        if (full[p]) {
#pragma unroll
          for (int u = 0; u < kU; ++u) {
            if (u < nu) {
#pragma unroll
              for (int q = 0; q < kG; ++q) {
                const uint32_t word = code[p][u][q >> 2];
                const float x = lut[u][(word >> (8 * (q & 3))) & 255u];
                acc[p][q] = acc[p][q] + term(x, b[p][q], wu[u], su[u], TWO);
              }
            }
          }
        } else if (have[p]) {
          for (int u = 0; u < nu; ++u) {
            const uint8_t* ptr = sld(a.cf, i0 + u);
#pragma unroll
            for (int q = 0; q < kG; ++q) {
              const uint64_t e = e0[p] + q;
              if (e >= ch.begin && e < ch.end) acc[p][q] = acc[p][q] + term(lut[u][ptr[e]], b[p][q], wu[u], su[u], TWO);
            }
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      if (full[p]) {
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) {
          const f4 v = f4{b[p][4 * q] + acc[p][4 * q], b[p][4 * q + 1] + acc[p][4 * q + 1],
                          b[p][4 * q + 2] + acc[p][4 * q + 2], b[p][4 * q + 3] + acc[p][4 * q + 3]};
          __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0[p]) + q);
        }
      } else if (have[p]) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0[p] + q;
          if (e >= ch.begin && e < ch.end) a.out_f[e] = b[p][q] + acc[p][q];
        }
      }
    }
  }
}

// kP element groups per lane with the next batch's codes in flight (round 6): the codes of batch i0 + kU
// are issued right after batch i0's table barrier, so their HBM latency runs under batch i0's lookups and
// batch i0 + kU's table build instead of stalling every wave after its own table build.  Two register
// sets of codes alternate by batch (a copy would wait for the loads).
template <int kBlock, int kU, bool TWO, int kG, int kP, bool kFastTab>
__device__ __forceinline__ void mpf_batch(const QArgs& a, const float* mrow, int i0, double inv_div,
                                          const bool (&full)[kP], const bool (&have)[kP], const uint64_t (&e0)[kP],
                                          const Chunk& ch, const CodeOf<kG> (&cur)[kP][kU],
                                          CodeOf<kG> (&nxt)[kP][kU], float (*lut)[256], const float (&b)[kP][kG],
                                          float (&acc)[kP][kG]) {
  const int K = a.K;
  const int nu = K - i0 < kU ? K - i0 : kU;
  __syncthreads();  // previous batch's lookups are done
  float wu[kU], su[kU];
  load_weights<kU, TWO>(a, i0, wu, su);
  for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
    const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;  // wave-uniform: scalar max_v
    if (u < nu) {
      const float mv = sld(mrow, i0 + u);
      const float v = kFastTab ? decode_tab(uint32_t(z), mv, inv_div) : decode(uint32_t(z), mv, a.divisor);
      lut[u][z] = v;
      lut[u][z + 128] = z ? -v : v;
    }
  }
  __syncthreads();
  if (i0 + kU < K) {
#pragma unroll
    for (int p = 0; p < kP; ++p)
      if (full[p]) load_codes<kU, kG>(a, i0 + kU, K, e0[p], nxt[p]);
  }
#pragma unroll
  for (int p = 0; p < kP; ++p) {
    if (full[p]) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (u < nu) {
#pragma unroll
          for (int q = 0; q < kG; ++q) {
            const uint32_t word = cur[p][u][q >> 2];
            const float x = lut[u][(word >> (8 * (q & 3))) & 255u];
            acc[p][q] = acc[p][q] + term(x, b[p][q], wu[u], su[u], TWO);
          }
        }
      }
    } else if (have[p]) {
      for (int u = 0; u < nu; ++u) {
        const uint8_t* ptr = sld(a.cf, i0 + u);
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0[p] + q;
          if (e >= ch.begin && e < ch.end) acc[p][q] = acc[p][q] + term(lut[u][ptr[e]], b[p][q], wu[u], su[u], TWO);
        }
      }
    }
  }
}

template <int kBlock, int kU, bool TWO, int kG, int kP, bool kFastTab>
__device__ void qsgd_f32_chunk_mpf(const QArgs& a, uint32_t c, float (*lut)[256]) {
  static_assert(kG == 16 || kG == 8 || kG == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG, g1 = (uint64_t(ch.end) + kG - 1) / kG;
  const int K = a.K;
  const double inv_div = 1.0 / double(a.divisor);
  for (uint64_t gp = g0; gp < g1; gp += uint64_t(kBlock) * kP) {
    uint64_t e0[kP];
    bool have[kP], full[kP];
    float b[kP][kG], acc[kP][kG];
    CodeOf<kG> ca[kP][kU], cb[kP][kU];
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const uint64_t g = gp + uint64_t(p) * kBlock + threadIdx.x;
      have[p] = g < g1;
      e0[p] = g * kG;
      full[p] = have[p] && e0[p] >= ch.begin && e0[p] + kG <= ch.end;
      if (full[p]) load_codes<kU, kG>(a, 0, K, e0[p], ca[p]);  // batch 0's codes, ahead of the baseline
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        acc[p][q] = 0.f;
        b[p][q] = 0.f;
      }
      if (full[p]) {
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) {
          const f4 v = *((gf4*)(a.base_f + e0[p]) + q);
          b[p][4 * q] = v.x;
          b[p][4 * q + 1] = v.y;
          b[p][4 * q + 2] = v.z;
          b[p][4 * q + 3] = v.w;
        }
      } else if (have[p]) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0[p] + q;
          if (e >= ch.begin && e < ch.end) b[p][q] = a.base_f[e];
        }
      }
    }
    for (int i0 = 0; i0 < K; i0 += 2 * kU) {
      mpf_batch<kBlock, kU, TWO, kG, kP, kFastTab>(a, mrow, i0, inv_div, full, have, e0, ch, ca, cb, lut, b, acc);
      if (i0 + kU < K)
        mpf_batch<kBlock, kU, TWO, kG, kP, kFastTab>(a, mrow, i0 + kU, inv_div, full, have, e0, ch, cb, ca, lut, b,
                                                     acc);
    }
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      if (full[p]) {
#pragma unroll
        for (int q = 0; q < kG / 4; ++q) {
          const f4 v = f4{b[p][4 * q] + acc[p][4 * q], b[p][4 * q + 1] + acc[p][4 * q + 1],
                          b[p][4 * q + 2] + acc[p][4 * q + 2], b[p][4 * q + 3] + acc[p][4 * q + 3]};
          __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0[p]) + q);
        }
      } else if (have[p]) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0[p] + q;
          if (e >= ch.begin && e < ch.end) a.out_f[e] = b[p][q] + acc[p][q];
        }
      }
    }
  }
}

template <int kBlock, int kU, bool TWO, int kG, int kP, bool kFastTab>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_mpf_kernel(QArgs a) {
  __shared__ float lut[kU][256];
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk_mpf<kBlock, kU, TWO, kG, kP, kFastTab>(a, c - a.nci, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}

template <int kBlock, int kU, bool TWO, int kG, int kP, bool kFastTab>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_mp_kernel(QArgs a) {
  __shared__ float lut[kU][256];
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk_mp<kBlock, kU, TWO, kG, kP, kFastTab>(a, c - a.nci, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}

template <int kBlock, int kU, bool TWO, int kG, bool kAbs>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_sp_kernel(QArgs a) {
  __shared__ float lut[kU][kAbs ? 128 : 256];
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk_sp<kBlock, kU, TWO, kG, kAbs>(a, c - a.nci, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}

// Timing probes of the pipelined kernel (kP; results are NOT the FedAvg, never a default, not
// parity-tested): kP 1 without the code loads, 2 without the table lookups, 3 without either.
// One batch of the pipelined loop: tables and codes of batch bi+1 go out, batch bi (codes in
// `cur`, tables in lut[bi & 1]) is summed, then one barrier.
template <int kBlock, int kU, bool TWO, int kG2, int kP>
__device__ __forceinline__ void pipe_step(const QArgs& a, const Chunk& ch, const float* mrow, int bi, int nb,
                                          bool full, bool have, uint64_t e0, const CodeOf<kG2> (&cur)[kU],
                                          CodeOf<kG2> (&nxt)[kU], float (*lut)[kU][256], const float (&b)[kG2],
                                          float (&acc)[kG2]) {
  const int K = a.K;
  const int i0 = bi * kU;
  const int nu = K - i0 < kU ? K - i0 : kU;
  float wu[kU], su[kU];
  load_weights<kU, TWO>(a, i0, wu, su);
  if (bi + 1 < nb) {
    const int i1 = i0 + kU;
    build_tables<kBlock, kU>(a, mrow, i1, K - i1 < kU ? K - i1 : kU, lut[(bi + 1) & 1]);
    if (full) {
      if (kP == 1 || kP == 3) {
#pragma unroll
        for (int u = 0; u < kU; ++u) nxt[u] = CodeOf<kG2>(uint32_t(e0 * 2654435761u + i1 + u));
      } else {
        load_codes<kU, kG2>(a, i1, K, e0, nxt);
      }
    }
  }
  if (full) {
    sum_batch<kU, kG2, TWO, (kP == 2 || kP == 3)>(nu, cur, wu, su, lut[bi & 1], b, acc);
  } else if (have) {
    for (int u = 0; u < nu; ++u) {
      const uint8_t* p = sld(a.cf, i0 + u);
      const float wu = sld(a.w, i0 + u);
      const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) acc[q] = acc[q] + term(lut[bi & 1][u][p[e]], b[q], wu, su, TWO);
      }
    }
  }
  __syncthreads();  // batch bi+1's tables are written; batch bi's lookups are done
}

template <int kBlock, int kU, bool TWO, int kG2, int kP>
__device__ void qsgd_f32_chunk_pipe(const QArgs& a, uint32_t c, float (*lut)[kU][256]) {
  static_assert(kG2 == 16 || kG2 == 8 || kG2 == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG2, g1 = (uint64_t(ch.end) + kG2 - 1) / kG2;
  const int K = a.K;
  const int nb = (K + kU - 1) / kU;
  for (uint64_t gp = g0; gp < g1; gp += kBlock) {  // one pass for chunks <= kBlock * kG2 elements
    const uint64_t g = gp + threadIdx.x;
    const bool have = g < g1;
    const uint64_t e0 = g * kG2;
    const bool full = have && e0 >= ch.begin && e0 + kG2 <= ch.end;
    float b[kG2], acc[kG2];
#pragma unroll
    for (int q = 0; q < kG2; ++q) {
      acc[q] = 0.f;
      b[q] = 0.f;
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG2 / 4; ++q) {
        const f4 v = *((gf4*)(a.base_f + e0) + q);
        b[4 * q] = v.x;
        b[4 * q + 1] = v.y;
        b[4 * q + 2] = v.z;
        b[4 * q + 3] = v.w;
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) b[q] = a.base_f[e];
      }
    }
    // two register sets of codes, alternating by batch (no copies: a copy would wait for the loads)
    CodeOf<kG2> ca[kU], cb[kU];
    if (gp != g0) __syncthreads();  // the previous pass's last lookups are done (multi-pass chunks only)
    build_tables<kBlock, kU>(a, mrow, 0, K < kU ? K : kU, lut[0]);
    if (full) load_codes<kU, kG2>(a, 0, K, e0, ca);
    __syncthreads();
    for (int bi = 0; bi < nb; bi += 2) {
      pipe_step<kBlock, kU, TWO, kG2, kP>(a, ch, mrow, bi, nb, full, have, e0, ca, cb, lut, b, acc);
      if (bi + 1 < nb)
        pipe_step<kBlock, kU, TWO, kG2, kP>(a, ch, mrow, bi + 1, nb, full, have, e0, cb, ca, lut, b, acc);
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG2 / 4; ++q) {
        const f4 v = f4{b[4 * q] + acc[4 * q], b[4 * q + 1] + acc[4 * q + 1], b[4 * q + 2] + acc[4 * q + 2],
                        b[4 * q + 3] + acc[4 * q + 3]};
        __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0) + q);
      }
    } else if (have) {
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) a.out_f[e] = b[q] + acc[q];
      }
    }
  }
}

template <int kBlock, int kU, bool TWO, int kGE, int kP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 8))) void fedavg_qsgd_pipe_kernel(
    QArgs a) {
  __shared__ float lut[2][kU][256];
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk_pipe<kBlock, kU, TWO, kGE, kP>(a, c - a.nci, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}

template <int kBlock, int kU, bool TWO, int kGE = kG, bool kSM = false, bool kAbs = false>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_kernel(QArgs a) {
  __shared__ float lut[kU][kAbs ? 128 : 256];
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk<kBlock, kU, TWO, kGE, kSM, kAbs>(a, c - a.nci, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}

#ifdef PLATO_AGG_TUNE  // round-6 candidates (libplato_agg_tune.so)
// ---------------------------------------------------------------------------
// Arithmetic decode (no tables, no LDS, no barriers): x = RN32(p / divisor) as
// RN32(RN64(p) * RN64(1 / divisor)) with p = RN32(|zeta| * max_v) — the exact float32 division's bits
// for every float pair (the argument of fedadp.hip adp_div_lr_f64, tests/test_division.py: the float64
// product lies within 2^-52 of the quotient, which is never that close to a float32 midpoint unless it
// is one, and then it is a float64 the product rounds to exactly).  The sign is applied afterwards by
// flipping bit 31 of the decoded value for codes with bit 7 set and |zeta| != 0: round-to-nearest is
// sign-symmetric, so decode(128 + z) = -decode(z) for z != 0, and code 128 (zeta = -0, the integer 0)
// decodes as code 0.  A lane owns kG consecutive elements (one kG-byte code load per client), clients in
// batches of kU whose code loads are issued one batch ahead.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float decode_arith(uint32_t zabs, float max_v, double inv_div) {
  const float p = float(zabs) * max_v;  // fp32(zeta * max_v): zeta exact in fp32 (v_cvt_f32_ubyte)
  return float(double(p) * inv_div);     // fp32(p / divisor)
}

template <int kG, int kU, bool TWO>
__device__ __forceinline__ void arith_batch(const QArgs& a, const float* mrow, int i0, int nu, double inv_div,
                                            const CodeOf<kG> (&code)[kU], const float (&b)[kG], float (&acc)[kG]) {
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    if (u < nu) {
      const float mv = sld(mrow, i0 + u);
      const float wu = sld(a.w, i0 + u);
      const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
      for (int j = 0; j < kG / 4; ++j) {
        const uint32_t word = code[u][j];
        const uint32_t mag = word & 0x7f7f7f7fu;
        // bit 7 of each byte: set iff the code is negative and |zeta| != 0 (|zeta| + 127 carries into bit 7)
        const uint32_t neg = word & (mag + 0x7f7f7f7fu) & 0x80808080u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = decode_arith((mag >> (8 * q)) & 0xffu, mv, inv_div);
          const uint32_t sbit = (neg << (24 - 8 * q)) & 0x80000000u;
          const float x = __uint_as_float(__float_as_uint(v) ^ sbit);
          acc[4 * j + q] = acc[4 * j + q] + term(x, b[4 * j + q], wu, su, TWO);
        }
      }
    }
  }
}

template <int kBlock, int kG, int kU, bool TWO>
__device__ void qsgd_f32_chunk_arith(const QArgs& a, uint32_t c) {
  static_assert(kG == 16 || kG == 8 || kG == 4, "one 16-, 8- or 4-byte code load per lane");
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG, g1 = (uint64_t(ch.end) + kG - 1) / kG;
  const int K = a.K;
  const double inv_div = 1.0 / double(a.divisor);
  for (uint64_t gp = g0; gp < g1; gp += kBlock) {
    const uint64_t g = gp + threadIdx.x;
    const bool have = g < g1;
    const uint64_t e0 = g * kG;
    const bool full = have && e0 >= ch.begin && e0 + kG <= ch.end;
    float b[kG], acc[kG];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      acc[q] = 0.f;
      b[q] = 0.f;
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = *((gf4*)(a.base_f + e0) + q);
        b[4 * q] = v.x;
        b[4 * q + 1] = v.y;
        b[4 * q + 2] = v.z;
        b[4 * q + 3] = v.w;
      }
      CodeOf<kG> ca[kU], cb[kU];
      load_codes<kU, kG>(a, 0, K, e0, ca);
      for (int i0 = 0; i0 < K; i0 += 2 * kU) {  // two register sets, alternating by batch
        if (i0 + kU < K) load_codes<kU, kG>(a, i0 + kU, K, e0, cb);
        arith_batch<kG, kU, TWO>(a, mrow, i0, K - i0 < kU ? K - i0 : kU, inv_div, ca, b, acc);
        if (i0 + kU >= K) break;
        if (i0 + 2 * kU < K) load_codes<kU, kG>(a, i0 + 2 * kU, K, e0, ca);
        arith_batch<kG, kU, TWO>(a, mrow, i0 + kU, K - i0 - kU < kU ? K - i0 - kU : kU, inv_div, cb, b, acc);
      }
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f4 v = f4{b[4 * q] + acc[4 * q], b[4 * q + 1] + acc[4 * q + 1], b[4 * q + 2] + acc[4 * q + 2],
                        b[4 * q + 3] + acc[4 * q + 3]};
        __builtin_nontemporal_store(v, (gf4w*)(a.out_f + e0) + q);
      }
    } else if (have) {  // a group cut by the chunk's ends: byte by byte
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) b[q] = a.base_f[e];
      }
      for (int i = 0; i < K; ++i) {
        const uint8_t* p = sld(a.cf, i);
        const float mv = sld(mrow, i), wu = sld(a.w, i), su = TWO ? sld(a.s, i) : 1.f;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
          const uint64_t e = e0 + q;
          if (e >= ch.begin && e < ch.end) {
            const uint32_t byte = p[e];
            const float v = decode_arith(byte & 127u, mv, inv_div);
            const float x = (byte > 128u) ? -v : v;
            acc[q] = acc[q] + term(x, b[q], wu, su, TWO);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kG; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) a.out_f[e] = b[q] + acc[q];
      }
    }
  }
}

template <int kBlock, int kG, int kU, bool TWO>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_arith_kernel(QArgs a) {
  const uint32_t c = blockIdx.x;  // the int64 chunks first (qsgd_i64_chunk)
  if (c >= a.nci) {
    qsgd_f32_chunk_arith<kBlock, kG, kU, TWO>(a, c - a.nci);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c);
  }
}
#endif  // PLATO_AGG_TUNE

using QFn = void (*)(const QArgs&, hipStream_t, uint32_t);
template <int B, int U, bool TWO, int G = kG, bool SM = false, bool ABS = false>
void launch_q(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_kernel<B, U, TWO, G, SM, ABS>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int U, bool TWO, int G, int P = 0>
void launch_qp(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_pipe_kernel<B, U, TWO, G, P>), dim3(nc), dim3(B), 0, st, a);
}
#ifdef PLATO_AGG_TUNE
template <int B, int G, int U, bool TWO>
void launch_qa(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_arith_kernel<B, G, U, TWO>), dim3(nc), dim3(B), 0, st, a);
}
#endif
template <int B, int U, bool TWO, int G, bool ABS>
void launch_qs(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_sp_kernel<B, U, TWO, G, ABS>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int U, bool TWO, int G, int P, bool FT>
void launch_qm(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_mp_kernel<B, U, TWO, G, P, FT>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int U, bool TWO, int G, int P, bool FT>
void launch_qf(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_mpf_kernel<B, U, TWO, G, P, FT>), dim3(nc), dim3(B), 0, st, a);
}
struct QVariant {
  int block, u, g;  // threads, clients per table batch, elements per lane
  QFn fn[2];        // [TWO]
};
// The rounds 1-4 sweeps (table-batch widths, two-level batching, resident tables, hybrid arithmetic
// decode, sign-rotated tables, globally built tables; round 4: software-pipelined lookups, a
// persistent grid, the plain form with prefetched codes) are recorded in DESIGN.md §11, §14 and
// profiles/r01_qsgd_*, r02d_qsgd_*, r02g_*, r03m_qsgd_*, r04*_qsgd_*; kept: the default, the pipelined
// form of rounds 2-3 and its timing probes.
#ifdef PLATO_AGG_TUNE  // libplato_agg_tune.so (scripts/bench_variants.py, tests/test_qsgd_gpu.py)
const QVariant kQVariants[] = {
    {256, 8, 8, {&launch_q<256, 8, false, 8, true>, &launch_q<256, 8, true, 8, true>}},  // 0 (round-5 default)
    {512, 4, 8, {&launch_qp<512, 4, false, 8>, &launch_qp<512, 4, true, 8>}},        // 1: pipelined (rounds 2-3)
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1>, &launch_qp<512, 4, true, 8, 1>}},  // 2: probe, no code loads
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 2>, &launch_qp<512, 4, true, 8, 2>}},  // 3: probe, no lookups
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 3>, &launch_qp<512, 4, true, 8, 3>}},  // 4: probe, neither
    {1024, 8, 8, {&launch_q<1024, 8, false, 8>, &launch_q<1024, 8, true, 8>}},       // 5: round 1 (vector max_v loads)
    {512, 8, 8, {&launch_q<512, 8, false, 8, true>, &launch_q<512, 8, true, 8, true>}},  // 6: the round-4 default
    // round 6: arithmetic decode (float64 reciprocal product, no tables): {block, clients per batch, elements/lane}
    {256, 4, 8, {&launch_qa<256, 8, 4, false>, &launch_qa<256, 8, 4, true>}},     // 7
    {256, 8, 8, {&launch_qa<256, 8, 8, false>, &launch_qa<256, 8, 8, true>}},     // 8
    {256, 4, 16, {&launch_qa<256, 16, 4, false>, &launch_qa<256, 16, 4, true>}},  // 9
    {128, 4, 16, {&launch_qa<128, 16, 4, false>, &launch_qa<128, 16, 4, true>}},  // 10
    {64, 4, 16, {&launch_qa<64, 16, 4, false>, &launch_qa<64, 16, 4, true>}},     // 11
    {256, 2, 16, {&launch_qa<256, 16, 2, false>, &launch_qa<256, 16, 2, true>}},  // 12
    // round 6: |zeta| tables (128 entries) with the sign flipped into bit 31 (kAbs)
    {256, 8, 8, {&launch_q<256, 8, false, 8, true, true>, &launch_q<256, 8, true, 8, true, true>}},      // 13
    {256, 16, 8, {&launch_q<256, 16, false, 8, true, true>, &launch_q<256, 16, true, 8, true, true>}},   // 14
    {512, 8, 8, {&launch_q<512, 8, false, 8, true, true>, &launch_q<512, 8, true, 8, true, true>}},      // 15
    {256, 8, 16, {&launch_q<256, 8, false, 16, true, true>, &launch_q<256, 8, true, 16, true, true>}},   // 16
    {128, 8, 8, {&launch_q<128, 8, false, 8, true, true>, &launch_q<128, 8, true, 8, true, true>}},      // 17
    // round 6: software-pipelined lookups, weights loaded with the codes ({block, U, G}; ABS as 13-17)
    {256, 8, 8, {&launch_qs<256, 8, false, 8, false>, &launch_qs<256, 8, true, 8, false>}},     // 18
    {256, 8, 8, {&launch_qs<256, 8, false, 8, true>, &launch_qs<256, 8, true, 8, true>}},       // 19
    {256, 16, 8, {&launch_qs<256, 16, false, 8, false>, &launch_qs<256, 16, true, 8, false>}},  // 20
    {256, 8, 16, {&launch_qs<256, 8, false, 16, false>, &launch_qs<256, 8, true, 16, false>}},  // 21
    {512, 8, 8, {&launch_qs<512, 8, false, 8, false>, &launch_qs<512, 8, true, 8, false>}},     // 22
    {128, 8, 8, {&launch_qs<128, 8, false, 8, false>, &launch_qs<128, 8, true, 8, false>}},     // 23
    // round 6: kP element groups per lane per table batch, float64-product table decode ({block, U, G * P})
    {256, 8, 8, {&launch_qm<256, 8, false, 8, 1, true>, &launch_qm<256, 8, true, 8, 1, true>}},    // 24: P 1, fast tables
    {256, 8, 16, {&launch_qm<256, 8, false, 8, 2, true>, &launch_qm<256, 8, true, 8, 2, true>}},   // 25: P 2, fast tables
    {256, 8, 16, {&launch_qm<256, 8, false, 8, 2, false>, &launch_qm<256, 8, true, 8, 2, false>}}, // 26: P 2, IEEE tables
    {128, 8, 16, {&launch_qm<128, 8, false, 8, 2, true>, &launch_qm<128, 8, true, 8, 2, true>}},   // 27: P 2, 128 threads
    {256, 8, 32, {&launch_qm<256, 8, false, 8, 4, true>, &launch_qm<256, 8, true, 8, 4, true>}},   // 28: P 4
    {256, 4, 16, {&launch_qm<256, 4, false, 8, 2, true>, &launch_qm<256, 4, true, 8, 2, true>}},   // 29: P 2, U 4 (default)
    {256, 4, 8, {&launch_qm<256, 4, false, 8, 1, true>, &launch_qm<256, 4, true, 8, 1, true>}},    // 30: P 1, U 4
    {256, 4, 16, {&launch_qm<256, 4, false, 8, 2, false>, &launch_qm<256, 4, true, 8, 2, false>}}, // 31: P 2, U 4, IEEE
    {256, 4, 32, {&launch_qm<256, 4, false, 8, 4, true>, &launch_qm<256, 4, true, 8, 4, true>}},   // 32: P 4, U 4
    {256, 2, 16, {&launch_qm<256, 2, false, 8, 2, true>, &launch_qm<256, 2, true, 8, 2, true>}},   // 33: P 2, U 2
    {512, 4, 16, {&launch_qm<512, 4, false, 8, 2, true>, &launch_qm<512, 4, true, 8, 2, true>}},   // 34: P 2, U 4, 512
    {128, 4, 16, {&launch_qm<128, 4, false, 8, 2, true>, &launch_qm<128, 4, true, 8, 2, true>}},   // 35: P 2, U 4, 128
    {256, 4, 24, {&launch_qm<256, 4, false, 8, 3, true>, &launch_qm<256, 4, true, 8, 3, true>}},   // 36: P 3, U 4
    {256, 4, 16, {&launch_qm<256, 4, false, 4, 4, true>, &launch_qm<256, 4, true, 4, 4, true>}},   // 37: G 4 x P 4, U 4
    // round 6: as 24-37 with the next batch's codes in flight during the current batch ({block, U, G * P})
    {256, 4, 16, {&launch_qf<256, 4, false, 8, 2, true>, &launch_qf<256, 4, true, 8, 2, true>}},   // 38: P 2, U 4
    {256, 8, 16, {&launch_qf<256, 8, false, 8, 2, true>, &launch_qf<256, 8, true, 8, 2, true>}},   // 39: P 2, U 8
    {256, 4, 8, {&launch_qf<256, 4, false, 8, 1, true>, &launch_qf<256, 4, true, 8, 1, true>}},    // 40: P 1, U 4
    {256, 2, 16, {&launch_qf<256, 2, false, 8, 2, true>, &launch_qf<256, 2, true, 8, 2, true>}},   // 41: P 2, U 2
    {512, 4, 16, {&launch_qf<512, 4, false, 8, 2, true>, &launch_qf<512, 4, true, 8, 2, true>}},   // 42: P 2, U 4, 512
};
#else  // libplato_agg.so: the default only
// = tuning variant 29 (round 6): two 8-element groups per lane per table batch of 4 clients, tables by
// the float64 reciprocal product: 0.290 against 0.308 ms for the round-5 default (tuning variant 0),
// interleaved on one box (profiles/r06g_qsgd_variants.log)
const QVariant kQVariants[] = {
    {256, 4, 16, {&launch_qm<256, 4, false, 8, 2, true>, &launch_qm<256, 4, true, 8, 2, true>}},  // 0 (default)
};
#endif
constexpr int kNumQVariants = sizeof(kQVariants) / sizeof(kQVariants[0]);

bool misaligned(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) != 0; }


int run_qsgd(int variant, const uint8_t* const* d_codes_f32, const uint8_t* const* d_codes_i64, int K,
                          const float* d_max_v, int n_entries, float divisor, const float* d_w, const float* d_s,
                          const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                          const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64, const float* d_base_f32,
                          const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                          size_t n_i64, hipStream_t stream) {
  if (variant < 0 || variant >= kNumQVariants) return set_error(PLATO_AGG_EINVAL, "bad qsgd variant");
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (n_entries <= 0 || !d_max_v || !d_w) return set_error(PLATO_AGG_EINVAL, "null max_v / weight table");
  if (!(divisor != 0.f)) return set_error(PLATO_AGG_EINVAL, "divisor (quantization_level - 1) must be non-zero");
  if (n_chunks_f32 && (!d_codes_f32 || !d_chunks_f32 || !d_base_f32 || !d_out_f32))
    return set_error(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_chunks_i64 && (!d_codes_i64 || !d_chunks_i64 || !d_base_i64 || !d_out_i64f))
    return set_error(PLATO_AGG_EINVAL, "null int64 pointer");
  if (misaligned(d_base_f32) || misaligned(d_out_f32))
    return set_error(PLATO_AGG_EINVAL, "fp32 baseline / output must be 16-byte aligned");
  if (n_f32 > 0xffffffffull || n_i64 > 0xffffffffull)
    return set_error(PLATO_AGG_EINVAL, "arena too large for 32-bit chunk offsets");
  const uint64_t nc = uint64_t(n_chunks_f32) + n_chunks_i64;
  if (nc == 0) return clear_error();
  if (nc > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "bad chunk count");
  QArgs a{};
  a.cf = d_codes_f32;
  a.ci = d_codes_i64;
  a.mv = d_max_v;
  a.w = d_w;
  a.s = d_s;
  a.tf = d_chunks_f32;
  a.ti = d_chunks_i64;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.out_f = d_out_f32;
  a.out_if = d_out_i64f;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.ncf = n_chunks_f32;
  a.nci = n_chunks_i64;
  a.divisor = divisor;
  a.K = K;
  kQVariants[variant].fn[d_s ? 1 : 0](a, stream, uint32_t(nc));
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string("fedavg_qsgd launch: ") + hipGetErrorString(err));
  return clear_error();
}

}  // namespace

extern "C" {

int plato_agg_fedavg_qsgd(const uint8_t* const* d_codes_f32, const uint8_t* const* d_codes_i64, int K,
                          const float* d_max_v, int n_entries, float divisor, const float* d_w, const float* d_s,
                          const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                          const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64, const float* d_base_f32,
                          const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                          size_t n_i64, hipStream_t stream) {
  return run_qsgd(0, d_codes_f32, d_codes_i64, K, d_max_v, n_entries, divisor, d_w, d_s, d_chunks_f32, n_chunks_f32,
                  d_chunks_i64, n_chunks_i64, d_base_f32, d_base_i64, d_out_f32, d_out_i64f, n_f32, n_i64, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_qsgd_variants(void) { return kNumQVariants; }

int plato_agg_tune_qsgd_chunk(int variant) {
  if (variant < 0 || variant >= kNumQVariants) return set_error(PLATO_AGG_EINVAL, "bad qsgd variant");
  return kQVariants[variant].block * kQVariants[variant].g;
}

int plato_agg_tune_fedavg_qsgd(int variant, const uint8_t* const* d_codes_f32, const uint8_t* const* d_codes_i64,
                               int K, const float* d_max_v, int n_entries, float divisor, const float* d_w,
                               const float* d_s, const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                               const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64, const float* d_base_f32,
                               const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                               size_t n_i64, hipStream_t stream) {
  return run_qsgd(variant, d_codes_f32, d_codes_i64, K, d_max_v, n_entries, divisor, d_w, d_s, d_chunks_f32,
                  n_chunks_f32, d_chunks_i64, n_chunks_i64, d_base_f32, d_base_i64, d_out_f32, d_out_i64f, n_f32,
                  n_i64, stream);
}
#endif  // PLATO_AGG_TUNE

}  // extern "C"
