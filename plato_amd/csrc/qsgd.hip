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
// (variant 0) is the pipelined form below at B = 512, U = 4, G = 8 (4,096-element
// chunks); the round-1 default (B = 1024, U = 8, G = 8, not pipelined) is variant 27.
// Every shape, pipelined, two-level or resident-table form measured lands within
// 0.32-0.34 ms on C2-sized inputs; DESIGN.md §11 has the counters and probes.
constexpr int kG = 16;      // elements per lane group (one 16-byte code load) of the default

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

template <int kBlock, int kU, bool TWO, int kG = ::kG>
__device__ void qsgd_f32_chunk(const QArgs& a, uint32_t c, float (*lut)[256]) {
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
    for (int i0 = 0; i0 < K; i0 += kU) {
      const int nu = K - i0 < kU ? K - i0 : kU;
      __syncthreads();  // previous batch's lookups are done
      // codes 128 + z decode to exactly -decode(z) (round-to-nearest is sign-symmetric),
      // except 128 itself: zeta = -0 is the integer 0
      for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
        const int u = t >> 7, z = t & 127;
        if (u < nu) {
          const float v = decode(uint32_t(z), sld(mrow, i0 + u), a.divisor);
          lut[u][z] = v;
          lut[u][z + 128] = z ? -v : v;
        }
      }
      __syncthreads();
      if (full) {
        using CodeT = std::conditional_t<kG == 16, u4, std::conditional_t<kG == 8, u2, u1>>;
        using GCodeT = std::conditional_t<kG == 16, gu4, std::conditional_t<kG == 8, gu2, gu1>>;
        CodeT code[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int i = i0 + u < K ? i0 + u : K - 1;
          code[u] = __builtin_nontemporal_load((GCodeT*)(sld(a.cf, i) + e0));
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          if (u < nu) {
            const float wu = sld(a.w, i0 + u);
            const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
            for (int q = 0; q < kG; ++q) {
              const uint32_t word = code[u][q >> 2];
              const float x = lut[u][(word >> (8 * (q & 3))) & 255u];
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
            if (e >= ch.begin && e < ch.end) acc[q] = acc[q] + term(lut[u][p[e]], b[q], wu, su, TWO);
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

// The arithmetic decode of |zeta| (hybrid kernels): q0 = t * r with r = RN(1 / divisor), then one
// fma correction step (rem = t - q0 * divisor is exact).  Markstein's theorem makes this the correctly
// rounded t / divisor away from underflow / overflow; it is not trusted blindly: the table build checks
// it against the IEEE division for all 256 codes of every (client, chunk) and a batch with any
// mismatch is summed from the tables alone.
__device__ __forceinline__ float decode_fast(float zf, float max_v, float divisor, float rcp) {
  const float t = zf * max_v;
  const float q0 = t * rcp;
  const float rem = __builtin_fmaf(-q0, divisor, t);
  return __builtin_fmaf(rem, rcp, q0);
}

// Sign of a code byte onto the arithmetic |zeta| decode: bit 7 of byte q of `word` -> bit 31.  Code 128
// (zeta = -0, the integer 0) comes out as -0 where the table holds +0; -0 and +0 give the same sum
// (x - b differs only in the sign of a zero, and the running sum, which starts at +0, never becomes -0
// and is unchanged by adding a zero of either sign).
template <int q>
__device__ __forceinline__ float apply_sign(uint32_t word, float mag) {
  const uint32_t s = q == 3 ? word : word << (24 - 8 * q);
  return __uint_as_float((s & 0x80000000u) | __float_as_uint(mag));
}

// Sign-rotated tables (kRot): the entry of code b sits at index b ^ ((b & 0x80) >> 2), so a code +z and
// its negative 128 + z fall 32 banks apart instead of into the same bank (bank = index mod 64) — the
// 2-way conflict that QSGD's sign-symmetric, small-magnitude codes produce in most 32-lane groups.
__device__ __forceinline__ uint32_t rot_word(uint32_t w) { return w ^ ((w & 0x80808080u) >> 2); }
__device__ __forceinline__ uint32_t rot_byte(uint32_t b) { return b ^ ((b & 0x80u) >> 2); }

template <int kBlock, int kU, bool kVerify = false, bool kRot = false>
__device__ __forceinline__ void build_tables(const QArgs& a, const float* mrow, int i0, int nu, float (*lut)[256],
                                             int* bad = nullptr, float rcp = 0.f) {
  for (int t = threadIdx.x; t < kU * 128; t += kBlock) {
    // u is wave-uniform (128 table slots per client, 64 lanes per wave): a scalar load of max_v,
    // so the table build never waits on the vector-memory counter of the code loads in flight
    const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;
    bool mismatch = false;
    if (u < nu) {
      const float m = sld(mrow, i0 + u);
      const float v = decode(uint32_t(z), m, a.divisor);
      lut[u][z] = v;
      lut[u][kRot ? rot_byte(uint32_t(z + 128)) : z + 128] = z ? -v : v;
      if (kVerify) {
        const float f = decode_fast(float(z), m, a.divisor, rcp);
        const uint32_t neg = __float_as_uint(f) | 0x80000000u;  // what apply_sign makes of code 128 + z
        mismatch = __float_as_uint(f) != __float_as_uint(v) || (z && neg != __float_as_uint(-v));
      }
    }
    if (kVerify) {
      const uint64_t ballot = __ballot(mismatch);
      if ((threadIdx.x & 63) == 0) bad[t >> 6] = ballot != 0;
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

template <int kU, int kG2, bool TWO, bool kNoLds = false, bool kRot = false>
__device__ __forceinline__ void sum_batch(int nu, const CodeOf<kG2> (&code)[kU], const float (&wu)[kU],
                                          const float (&su)[kU], const float (*lut)[256], const float (&b)[kG2],
                                          float (&acc)[kG2]) {
  if (nu == kU) {  // every batch but a ragged last one: no per-client branches
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint32_t word = kRot ? rot_word(code[u][q >> 2]) : code[u][q >> 2];
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
          const uint32_t word = kRot ? rot_word(code[u][q >> 2]) : code[u][q >> 2];
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

// Hybrid sum of a full batch: the first kA elements of each lane's group are decoded arithmetically
// (VALU), the others through the tables (LDS), so neither pipe carries the whole decode.
template <int kU, int kG2, bool TWO, int kA>
__device__ __forceinline__ void sum_batch_hybrid(const CodeOf<kG2> (&code)[kU], const float (&wu)[kU],
                                                 const float (&su)[kU], const float (&mu)[kU], float divisor,
                                                 float rcp, const float (*lut)[256], const float (&b)[kG2],
                                                 float (&acc)[kG2]) {
#pragma unroll
  for (int u = 0; u < kU; ++u) {
#pragma unroll
    for (int q = 0; q < kG2; ++q) {
      const uint32_t word = code[u][q >> 2];
      float x;
      if (q < kA) {
        const uint32_t mag = (word >> (8 * (q & 3))) & 127u;
        const float f = decode_fast(float(mag), mu[u], divisor, rcp);
        switch (q & 3) {
          case 0: x = apply_sign<0>(word, f); break;
          case 1: x = apply_sign<1>(word, f); break;
          case 2: x = apply_sign<2>(word, f); break;
          default: x = apply_sign<3>(word, f); break;
        }
      } else {
        x = lut[u][(word >> (8 * (q & 3))) & 255u];
      }
      acc[q] = acc[q] + term(x, b[q], wu[u], su[u], TWO);
    }
  }
}

// One batch of the pipelined loop: tables and codes of batch bi+1 go out, batch bi (codes in
// `cur`, tables in lut[bi & 1]) is summed, then one barrier.
template <int kBlock, int kU, bool TWO, int kG2, int kA>
__device__ __forceinline__ void pipe_step(const QArgs& a, const Chunk& ch, const float* mrow, int bi, int nb,
                                          bool full, bool have, uint64_t e0, const CodeOf<kG2> (&cur)[kU],
                                          CodeOf<kG2> (&nxt)[kU], float (*lut)[kU][256], int (*bad)[2 * kU],
                                          float rcp, const float (&b)[kG2], float (&acc)[kG2]) {
  const int K = a.K;
  const int i0 = bi * kU;
  const int nu = K - i0 < kU ? K - i0 : kU;
  float wu[kU], su[kU];
  load_weights<kU, TWO>(a, i0, wu, su);
  if (bi + 1 < nb) {
    const int i1 = i0 + kU;
    build_tables<kBlock, kU, (kA > 0), (kA == -4)>(a, mrow, i1, K - i1 < kU ? K - i1 : kU, lut[(bi + 1) & 1],
                                                   bad[(bi + 1) & 1], rcp);
    if (full) {
      if (kA == -1 || kA == -3) {  // timing probe: no code loads
#pragma unroll
        for (int u = 0; u < kU; ++u) nxt[u] = CodeOf<kG2>(uint32_t(e0 * 2654435761u + i1 + u));
      } else {
        load_codes<kU, kG2>(a, i1, K, e0, nxt);
      }
    }
  }
  bool fast = false;
  if (kA > 0 && nu == kU) {
    int any = 0;
#pragma unroll
    for (int j = 0; j < 2 * kU; ++j) any |= bad[bi & 1][j];
    fast = __builtin_amdgcn_readfirstlane(any) == 0;
  }
  if (full && fast) {
    float mu[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) mu[u] = sld(mrow, i0 + u);
    sum_batch_hybrid<kU, kG2, TWO, (kA > 0 ? kA : 1)>(cur, wu, su, mu, a.divisor, rcp, lut[bi & 1], b, acc);
  } else if (full) {
    sum_batch<kU, kG2, TWO, (kA == -2 || kA == -3), (kA == -4)>(nu, cur, wu, su, lut[bi & 1], b, acc);
  } else if (have) {
    for (int u = 0; u < nu; ++u) {
      const uint8_t* p = sld(a.cf, i0 + u);
      const float wu = sld(a.w, i0 + u);
      const float su = TWO ? sld(a.s, i0 + u) : 1.f;
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end)
          acc[q] = acc[q] + term(lut[bi & 1][u][kA == -4 ? rot_byte(p[e]) : p[e]], b[q], wu, su, TWO);
      }
    }
  }
  __syncthreads();  // batch bi+1's tables are written; batch bi's lookups are done
}

template <int kBlock, int kU, bool TWO, int kG2, int kA>
__device__ void qsgd_f32_chunk_pipe(const QArgs& a, uint32_t c, float (*lut)[kU][256], int (*bad)[2 * kU]) {
  static_assert(kG2 == 16 || kG2 == 8 || kG2 == 4, "one 16-, 8- or 4-byte code load per lane");
  static_assert(kBlock * (kG2 / 4) >= 1, "");
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
    const float rcp = 1.0f / a.divisor;  // RN(1 / divisor): the IEEE division
    build_tables<kBlock, kU, (kA > 0), (kA == -4)>(a, mrow, 0, K < kU ? K : kU, lut[0], bad[0], rcp);
    if (full) load_codes<kU, kG2>(a, 0, K, e0, ca);
    __syncthreads();
    for (int bi = 0; bi < nb; bi += 2) {
      pipe_step<kBlock, kU, TWO, kG2, kA>(a, ch, mrow, bi, nb, full, have, e0, ca, cb, lut, bad, rcp, b, acc);
      if (bi + 1 < nb)
        pipe_step<kBlock, kU, TWO, kG2, kA>(a, ch, mrow, bi + 1, nb, full, have, e0, cb, ca, lut, bad, rcp, b, acc);
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

// Two-level batching: the decode tables are built kUt clients at a time (one barrier per table
// batch, double-buffered), the codes are streamed kUr clients at a time through two register
// sets (each sub-batch's codes are loaded while the previous one is summed).  The per-barrier
// fixed costs (scalar loads, table division, the barrier itself) are paid K / kUt times per chunk
// instead of K / kUr times.
template <int kBlock, int kUt, int kUr, bool TWO, int kG2>
__device__ __forceinline__ void tb_step(const QArgs& a, int j, int nsb, bool full, bool have, const Chunk& ch,
                                        uint64_t e0, const CodeOf<kG2> (&cur)[kUr], CodeOf<kG2> (&nxt)[kUr],
                                        float (*lut)[kUt][256], const float (&b)[kG2], float (&acc)[kG2]) {
  constexpr int S = kUt / kUr;
  const int K = a.K;
  const int i0 = j * kUr;
  const int nu = K - i0 < kUr ? K - i0 : kUr;
  float wu[kUr], su[kUr];
  load_weights<kUr, TWO>(a, i0, wu, su);
  if (full && j + 1 < nsb) load_codes<kUr, kG2>(a, i0 + kUr, K, e0, nxt);
  const float (*tab)[256] = &lut[(j / S) & 1][(j % S) * kUr];
  if (full) {
    sum_batch<kUr, kG2, TWO>(nu, cur, wu, su, tab, b, acc);
  } else if (have) {
    for (int u = 0; u < nu; ++u) {
      const uint8_t* p = sld(a.cf, i0 + u);
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) acc[q] = acc[q] + term(tab[u][p[e]], b[q], wu[u], su[u], TWO);
      }
    }
  }
}

template <int kBlock, int kUt, int kUr, bool TWO, int kG2>
__device__ void qsgd_f32_chunk_tb(const QArgs& a, uint32_t c, float (*lut)[kUt][256]) {
  static_assert(kUt % (2 * kUr) == 0, "an even number of register sub-batches per table batch");
  constexpr int S = kUt / kUr;
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG2, g1 = (uint64_t(ch.end) + kG2 - 1) / kG2;
  const int K = a.K;
  const int ntb = (K + kUt - 1) / kUt;
  const int nsb = (K + kUr - 1) / kUr;
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
    CodeOf<kG2> ca[kUr], cb[kUr];
    if (gp != g0) __syncthreads();  // the previous pass's last lookups are done (multi-pass chunks only)
    build_tables<kBlock, kUt>(a, mrow, 0, K < kUt ? K : kUt, lut[0]);
    if (full) load_codes<kUr, kG2>(a, 0, K, e0, ca);
    __syncthreads();
    for (int tb = 0; tb < ntb; ++tb) {
      if (tb + 1 < ntb) {
        const int i1 = (tb + 1) * kUt;
        build_tables<kBlock, kUt>(a, mrow, i1, K - i1 < kUt ? K - i1 : kUt, lut[(tb + 1) & 1]);
      }
      const int jb = tb * S, je = jb + S < nsb ? jb + S : nsb;
      for (int j = jb; j < je; j += 2) {  // S is even: every table batch starts with its codes in ca
        tb_step<kBlock, kUt, kUr, TWO, kG2>(a, j, nsb, full, have, ch, e0, ca, cb, lut, b, acc);
        if (j + 1 < je) tb_step<kBlock, kUt, kUr, TWO, kG2>(a, j + 1, nsb, full, have, ch, e0, cb, ca, lut, b, acc);
      }
      __syncthreads();  // table batch tb+1 is written; table batch tb's lookups are done
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

template <int kBlock, int kUt, int kUr, bool TWO, int kGE>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_tb_kernel(QArgs a) {
  __shared__ float lut[2][kUt][256];
  const uint32_t c = blockIdx.x;
  if (c < a.ncf) {
    qsgd_f32_chunk_tb<kBlock, kUt, kUr, TWO, kGE>(a, c, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c - a.ncf);
  }
}

// Resident tables: a workgroup decodes the tables of up to kKmax clients into LDS once per chunk (one
// barrier), then streams every client's codes with no further barrier: no per-batch table build,
// scalar loads of max_v or s_barrier inside the client loop.  K > kKmax runs in phases of kKmax
// clients (a barrier and a table build per phase).
template <int kUr, bool TWO, int kG2>
__device__ __forceinline__ void rt_step(const QArgs& a, int i0, int iend, bool full, bool have, const Chunk& ch,
                                        uint64_t e0, const CodeOf<kG2> (&cur)[kUr], CodeOf<kG2> (&nxt)[kUr],
                                        const float (*tab)[256], const float (&b)[kG2], float (&acc)[kG2]) {
  const int nu = iend - i0 < kUr ? iend - i0 : kUr;
  float wu[kUr], su[kUr];
  load_weights<kUr, TWO>(a, i0, wu, su);
  if (full && i0 + kUr < iend) load_codes<kUr, kG2>(a, i0 + kUr, iend, e0, nxt);
  if (full) {
    sum_batch<kUr, kG2, TWO>(nu, cur, wu, su, tab, b, acc);
  } else if (have) {
    for (int u = 0; u < nu; ++u) {
      const uint8_t* p = sld(a.cf, i0 + u);
#pragma unroll
      for (int q = 0; q < kG2; ++q) {
        const uint64_t e = e0 + q;
        if (e >= ch.begin && e < ch.end) acc[q] = acc[q] + term(tab[u][p[e]], b[q], wu[u], su[u], TWO);
      }
    }
  }
}

template <int kBlock, int kUr, bool TWO, int kG2, int kKmax>
__device__ void qsgd_f32_chunk_rt(const QArgs& a, uint32_t c, float (*lut)[256]) {
  const Chunk ch = load_chunk(a.tf, c, a.n_f32);
  const float* mrow = a.mv + uint64_t(ch.entry) * a.K;
  const uint64_t g0 = ch.begin / kG2, g1 = (uint64_t(ch.end) + kG2 - 1) / kG2;
  const int K = a.K;
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
    for (int p0 = 0; p0 < K; p0 += kKmax) {
      const int pend = K - p0 < kKmax ? K : p0 + kKmax;
      CodeOf<kG2> ca[kUr], cb[kUr];
      if (full) load_codes<kUr, kG2>(a, p0, pend, e0, ca);  // in flight during the table build
      if (gp != g0 || p0) __syncthreads();                 // the previous phase's lookups are done
      for (int t = threadIdx.x; t < (pend - p0) * 128; t += kBlock) {
        const int u = __builtin_amdgcn_readfirstlane(t >> 7), z = t & 127;
        const float v = decode(uint32_t(z), sld(mrow, p0 + u), a.divisor);
        lut[u][z] = v;
        lut[u][z + 128] = z ? -v : v;
      }
      __syncthreads();
      for (int i0 = p0; i0 < pend; i0 += 2 * kUr) {
        rt_step<kUr, TWO, kG2>(a, i0, pend, full, have, ch, e0, ca, cb, &lut[i0 - p0], b, acc);
        if (i0 + kUr < pend)
          rt_step<kUr, TWO, kG2>(a, i0 + kUr, pend, full, have, ch, e0, cb, ca, &lut[i0 + kUr - p0], b, acc);
      }
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

template <int kBlock, int kUr, bool TWO, int kGE, int kKmax>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_rt_kernel(QArgs a) {
  __shared__ float lut[kKmax][256];
  const uint32_t c = blockIdx.x;
  if (c < a.ncf) {
    qsgd_f32_chunk_rt<kBlock, kUr, TWO, kGE, kKmax>(a, c, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c - a.ncf);
  }
}

template <int kBlock, int kU, bool TWO, int kGE, int kWaves, int kA>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kWaves, 8))) void fedavg_qsgd_pipe_kernel(
    QArgs a) {
  __shared__ float lut[2][kU][256];
  __shared__ int bad[2][2 * kU];  // per table buffer: one flag per 64 codes whose fast decode mismatched
  const uint32_t c = blockIdx.x;
  if (c < a.ncf) {
    qsgd_f32_chunk_pipe<kBlock, kU, TWO, kGE, kA>(a, c, lut, bad);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c - a.ncf);
  }
}

template <int kBlock, int kU, bool TWO, int kGE = kG>
__global__ __launch_bounds__(kBlock) void fedavg_qsgd_kernel(QArgs a) {
  __shared__ float lut[kU][256];
  const uint32_t c = blockIdx.x;
  if (c < a.ncf) {
    qsgd_f32_chunk<kBlock, kU, TWO, kGE>(a, c, lut);
  } else {
    qsgd_i64_chunk<kBlock, TWO>(a, c - a.ncf);
  }
}

using QFn = void (*)(const QArgs&, hipStream_t, uint32_t);
template <int B, int U, bool TWO, int G = kG>
void launch_q(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_kernel<B, U, TWO, G>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int UR, bool TWO, int G, int KMAX>
void launch_qr(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_rt_kernel<B, UR, TWO, G, KMAX>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int UT, int UR, bool TWO, int G>
void launch_qt(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_tb_kernel<B, UT, UR, TWO, G>), dim3(nc), dim3(B), 0, st, a);
}
template <int B, int U, bool TWO, int G, int W = 1, int A = 0>
void launch_qp(const QArgs& a, hipStream_t st, uint32_t nc) {
  hipLaunchKernelGGL((fedavg_qsgd_pipe_kernel<B, U, TWO, G, W, A>), dim3(nc), dim3(B), 0, st, a);
}
struct QVariant {
  int block, u, g;  // threads, clients per table batch, elements per lane
  QFn fn[2];        // [TWO]
};
#ifdef PLATO_AGG_TUNE  // libplato_agg_tune.so: every shape (scripts/, tests/test_qsgd_gpu.py)
const QVariant kQVariants[] = {
    {512, 4, 8, {&launch_qp<512, 4, false, 8>, &launch_qp<512, 4, true, 8>}},  // 0 (default): pipelined
    {256, 8, 16, {&launch_q<256, 8, false>, &launch_q<256, 8, true>}},      // 1
    {512, 16, 16, {&launch_q<512, 16, false>, &launch_q<512, 16, true>}},   // 2
    {256, 4, 16, {&launch_q<256, 4, false>, &launch_q<256, 4, true>}},      // 3
    {1024, 8, 16, {&launch_q<1024, 8, false>, &launch_q<1024, 8, true>}},   // 4
    {256, 8, 8, {&launch_q<256, 8, false, 8>, &launch_q<256, 8, true, 8>}},  // 5
    {512, 8, 8, {&launch_q<512, 8, false, 8>, &launch_q<512, 8, true, 8>}},  // 6
    {128, 8, 16, {&launch_q<128, 8, false>, &launch_q<128, 8, true>}},      // 7
    {512, 16, 8, {&launch_q<512, 16, false, 8>, &launch_q<512, 16, true, 8>}},  // 8
    {512, 8, 4, {&launch_q<512, 8, false, 4>, &launch_q<512, 8, true, 4>}},    // 9
    {512, 8, 16, {&launch_q<512, 8, false>, &launch_q<512, 8, true>}},      // 10 (the first default)
    {256, 16, 8, {&launch_q<256, 16, false, 8>, &launch_q<256, 16, true, 8>}},  // 11
    {1024, 16, 8, {&launch_q<1024, 16, false, 8>, &launch_q<1024, 16, true, 8>}},  // 12
    {1024, 4, 8, {&launch_q<1024, 4, false, 8>, &launch_q<1024, 4, true, 8>}},  // 13
    // pipelined: double-buffered tables, next batch's codes in registers, one barrier per batch;
    // last field: minimum waves per SIMD asked of the register allocator
    {1024, 8, 8, {&launch_qp<1024, 8, false, 8>, &launch_qp<1024, 8, true, 8>}},          // 14
    {512, 8, 8, {&launch_qp<512, 8, false, 8>, &launch_qp<512, 8, true, 8>}},             // 15
    {1024, 8, 8, {&launch_qp<1024, 8, false, 8, 8>, &launch_qp<1024, 8, true, 8, 8>}},    // 16
    {512, 8, 8, {&launch_qp<512, 8, false, 8, 6>, &launch_qp<512, 8, true, 8, 6>}},       // 17
    {256, 8, 8, {&launch_qp<256, 8, false, 8, 6>, &launch_qp<256, 8, true, 8, 6>}},       // 18
    {1024, 4, 8, {&launch_qp<1024, 4, false, 8, 8>, &launch_qp<1024, 4, true, 8, 8>}},    // 19
    {512, 16, 8, {&launch_qp<512, 16, false, 8>, &launch_qp<512, 16, true, 8>}},          // 20
    {1024, 8, 4, {&launch_qp<1024, 8, false, 4, 8>, &launch_qp<1024, 8, true, 4, 8>}},    // 21
    {512, 8, 16, {&launch_qp<512, 8, false, 16>, &launch_qp<512, 8, true, 16>}},          // 22
    {256, 8, 16, {&launch_qp<256, 8, false, 16>, &launch_qp<256, 8, true, 16>}},          // 23
    {1024, 8, 4, {&launch_qp<1024, 8, false, 4>, &launch_qp<1024, 8, true, 4>}},          // 24
    {512, 8, 4, {&launch_qp<512, 8, false, 4>, &launch_qp<512, 8, true, 4>}},             // 25
    {1024, 4, 8, {&launch_qp<1024, 4, false, 8>, &launch_qp<1024, 4, true, 8>}},          // 26
    {1024, 8, 8, {&launch_q<1024, 8, false, 8>, &launch_q<1024, 8, true, 8>}},            // 27 (round-1 default)
    // hybrid decode: last field = elements per lane decoded arithmetically (the rest via the tables)
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, 4>, &launch_qp<512, 4, true, 8, 1, 4>}},       // 28
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, 2>, &launch_qp<512, 4, true, 8, 1, 2>}},       // 29
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, 6>, &launch_qp<512, 4, true, 8, 1, 6>}},       // 30
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, 8>, &launch_qp<512, 4, true, 8, 1, 8>}},       // 31
    {1024, 8, 8, {&launch_qp<1024, 8, false, 8, 1, 4>, &launch_qp<1024, 8, true, 8, 1, 4>}},    // 32
    {512, 8, 8, {&launch_qp<512, 8, false, 8, 1, 4>, &launch_qp<512, 8, true, 8, 1, 4>}},       // 33
    {256, 4, 8, {&launch_qp<256, 4, false, 8, 1, 4>, &launch_qp<256, 4, true, 8, 1, 4>}},       // 34
    {512, 4, 4, {&launch_qp<512, 4, false, 4, 1, 2>, &launch_qp<512, 4, true, 4, 1, 2>}},       // 35
    {256, 4, 8, {&launch_qp<256, 4, false, 8>, &launch_qp<256, 4, true, 8>}},                   // 36
    {512, 2, 8, {&launch_qp<512, 2, false, 8>, &launch_qp<512, 2, true, 8>}},                   // 37
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 7>, &launch_qp<512, 4, true, 8, 7>}},             // 38
    {512, 4, 4, {&launch_qp<512, 4, false, 4>, &launch_qp<512, 4, true, 4>}},                   // 39
    {128, 4, 8, {&launch_qp<128, 4, false, 8>, &launch_qp<128, 4, true, 8>}},                   // 40
    // timing probes of variant 0 (results are NOT the FedAvg; never a default, not parity-tested):
    // 41 without the code loads, 42 without the table lookups, 43 without either
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, -1>, &launch_qp<512, 4, true, 8, 1, -1>}},     // 41
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, -2>, &launch_qp<512, 4, true, 8, 1, -2>}},     // 42
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, -3>, &launch_qp<512, 4, true, 8, 1, -3>}},     // 43
    // two-level batching (table batch x register sub-batch): u = clients per table batch
    {512, 16, 8, {&launch_qt<512, 16, 4, false, 8>, &launch_qt<512, 16, 4, true, 8>}},          // 44
    {512, 32, 8, {&launch_qt<512, 32, 4, false, 8>, &launch_qt<512, 32, 4, true, 8>}},          // 45
    {512, 16, 8, {&launch_qt<512, 16, 2, false, 8>, &launch_qt<512, 16, 2, true, 8>}},          // 46
    {1024, 16, 8, {&launch_qt<1024, 16, 4, false, 8>, &launch_qt<1024, 16, 4, true, 8>}},       // 47
    {256, 16, 8, {&launch_qt<256, 16, 4, false, 8>, &launch_qt<256, 16, 4, true, 8>}},          // 48
    {512, 16, 16, {&launch_qt<512, 16, 2, false, 16>, &launch_qt<512, 16, 2, true, 16>}},       // 49
    {512, 32, 8, {&launch_qt<512, 32, 8, false, 8>, &launch_qt<512, 32, 8, true, 8>}},          // 50
    // resident tables (u = clients per LDS phase), register sub-batches of 4 (55: 8)
    {1024, 128, 8, {&launch_qr<1024, 4, false, 8, 128>, &launch_qr<1024, 4, true, 8, 128>}},    // 51
    {1024, 64, 8, {&launch_qr<1024, 4, false, 8, 64>, &launch_qr<1024, 4, true, 8, 64>}},       // 52
    {1024, 128, 16, {&launch_qr<1024, 4, false, 16, 128>, &launch_qr<1024, 4, true, 16, 128>}}, // 53
    {512, 32, 8, {&launch_qr<512, 4, false, 8, 32>, &launch_qr<512, 4, true, 8, 32>}},          // 54
    {1024, 128, 8, {&launch_qr<1024, 8, false, 8, 128>, &launch_qr<1024, 8, true, 8, 128>}},    // 55
    {512, 64, 8, {&launch_qr<512, 4, false, 8, 64>, &launch_qr<512, 4, true, 8, 64>}},          // 56
    {256, 32, 8, {&launch_qr<256, 4, false, 8, 32>, &launch_qr<256, 4, true, 8, 32>}},          // 57
    {512, 32, 8, {&launch_qr<512, 8, false, 8, 32>, &launch_qr<512, 8, true, 8, 32>}},          // 58
    {512, 32, 4, {&launch_qr<512, 16, false, 4, 32>, &launch_qr<512, 16, true, 4, 32>}},        // 59
    {512, 32, 4, {&launch_qr<512, 8, false, 4, 32>, &launch_qr<512, 8, true, 4, 32>}},          // 60
    // sign-rotated tables (+z and -z 32 banks apart) on the default's shape and two others
    {512, 4, 8, {&launch_qp<512, 4, false, 8, 1, -4>, &launch_qp<512, 4, true, 8, 1, -4>}},     // 61
    {1024, 8, 8, {&launch_qp<1024, 8, false, 8, 1, -4>, &launch_qp<1024, 8, true, 8, 1, -4>}},  // 62
    {512, 4, 16, {&launch_qp<512, 4, false, 16, 1, -4>, &launch_qp<512, 4, true, 16, 1, -4>}},  // 63
};
#else  // libplato_agg.so: the default only
const QVariant kQVariants[] = {
    {512, 4, 8, {&launch_qp<512, 4, false, 8>, &launch_qp<512, 4, true, 8>}},  // 0 (default): pipelined
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
