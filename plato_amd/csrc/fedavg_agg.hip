// fedavg_agg.hip — gfx950 (MI355X / CDNA4) kernels for Plato's server-side
// FedAvg aggregation, exported through the C ABI in include/plato_agg.h.
//
// Design:
//  * The hot op is an HBM-bound streaming reduction: every output element reads
//    the same element of K client arenas plus the baseline and writes one value
//    ((K+2)*4 bytes per fp32 element, 3K flops: ~0.75 flop/B).  No MFMA, no LDS
//    reuse to exploit; the kernel is built to keep enough 16-byte loads in
//    flight to saturate HBM3E.
//  * Bit-exactness with the reference CPU path forbids splitting the K-sum
//    across lanes/waves/GPUs: each lane owns whole elements (f4 groups) and
//    walks the clients in order, with separately rounded sub/mul/add (the
//    library is compiled with -ffp-contract=off; no fmaf anywhere).
//  * Memory-level parallelism therefore comes from (a) V f4 per lane per
//    client and (b) U clients unrolled, i.e. U*V independent dwordx4 loads per
//    lane before the first dependent add.  Client pointers and weights are
//    wave-uniform -> scalar (s_load) reads from the device pointer table.
//  * The fp32 arena tail (n % 4) and the int64 entries are tiny: they run on a
//    few extra workgroups at the end of the same grid, so one launch does the
//    whole model.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "common.h"
#include "plato_agg.h"
#include "plato_agg_tune.h"

namespace {
thread_local std::string g_last_error;
}  // namespace

namespace plato_agg_internal {
int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
int clear_error() {
  g_last_error.clear();
  return PLATO_AGG_OK;
}
}  // namespace plato_agg_internal

namespace {

int fail(int code, const std::string& msg) { return plato_agg_internal::set_error(code, msg); }

int check_launch(const char* what) {
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    return fail(PLATO_AGG_EHIP, std::string(what) + ": " + hipGetErrorString(err));
  }
  g_last_error.clear();
  return PLATO_AGG_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

constexpr int kBlock = 256;  // 4 waves of 64

// ---------------------------------------------------------------------------
// Loads
// ---------------------------------------------------------------------------
// Native 4 x fp32 vector: one dwordx4 load/store; element-wise IEEE ops.
typedef float f4 __attribute__((ext_vector_type(4)));

// Client arenas are plain hipMalloc'd global memory: load through an
// address_space(1) pointer so hipcc emits global_load_dwordx4 (vmcnt only)
// instead of flat loads (which also tick lgkmcnt and force vmcnt(0)+lgkmcnt(0)
// waits next to the scalar loads).
typedef __attribute__((address_space(1))) const f4 gf4;
typedef __attribute__((address_space(1))) const float gfloat;

template <bool NT>
__device__ __forceinline__ f4 ld4(const f4* p) {
  gf4* g = (gf4*)p;
  if constexpr (NT) {
    return __builtin_nontemporal_load(g);
  } else {
    return *g;
  }
}

// Wave-uniform base + 32-bit per-lane byte offset: lets hipcc use the
// global_load saddr form (base in SGPRs, one offset VGPR per stream).
template <bool NT>
__device__ __forceinline__ f4 ld4_off(const float* base, uint32_t byte_off) {
  gf4* g = (gf4*)((__attribute__((address_space(1))) const char*)base + byte_off);
  if constexpr (NT) {
    return __builtin_nontemporal_load(g);
  } else {
    return *g;
  }
}

// The pointer table and the weights are wave-uniform and read-only for the
// whole launch: read them through the constant address space -> s_load
// (scalar cache), so no VGPRs and no vector-memory round trip per client.
template <class T>
__device__ __forceinline__ T sld(const T* p, int i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

__device__ __forceinline__ f4 f4_sub(f4 a, f4 b) { return a - b; }
__device__ __forceinline__ f4 f4_add(f4 a, f4 b) { return a + b; }
__device__ __forceinline__ f4 f4_scale(f4 a, float s) { return a * s; }
__device__ __forceinline__ f4 f4_zero() { return f4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------------------
// Main kernel: fp32 arena body (f4 groups) + scalar work items
// (fp32 tail and int64 entries) on extra workgroups at the end of the grid.
// HAS_BASE: weights mode (subtract the baseline, add it back at the end);
//           otherwise deltas mode (x are deltas, out = sum).
// ---------------------------------------------------------------------------
struct AggArgs {
  const float* const* xf;      // K pointers to fp32 arenas
  const int64_t* const* xi;    // K pointers to int64 arenas (may be null)
  const float* w;              // K fp32 weights
  const float* s;              // K fp32 second scalars (TWO only)
  const float* base_f;         // baseline fp32 (HAS_BASE only)
  const int64_t* base_i;       // baseline int64 (HAS_BASE only)
  float* out_f;
  float* out_if;               // fp32 results of the int64 entries
  uint64_t n4;                 // number of f4 groups in the fp32 arena
  uint64_t n_f32;              // fp32 elements (tail = n_f32 - 4*n4)
  uint64_t n_i64;
  uint32_t nb_vec;             // workgroups of the f4 body
  uint32_t nb_vec_full;        // of which fully in range (no bounds checks)
  uint32_t nb_grid;            // PERSIST: workgroups striding over the chunks; XCD: vector blocks in the grid
  uint32_t xcd_per;            // XCD: chunks per XCD (contiguous range)
  uint32_t nb_scalar;          // workgroups of scalar items: the FIRST blocks of the grid
  uint64_t x_off;              // element offset of this launch's range in every client arena
  int K;
};

// Kernel configuration (tuning space; DESIGN.md §5 has the sweep):
//   B   threads per workgroup      V  f4 groups per lane per client
//   U   clients per batch          NTL/NTS  non-temporal loads / stores
//   PIPE  software-pipelined: batch j+1's loads issue before batch j's adds
//   BUF   buffer_load_dwordx4 (SRD per client, 32-bit voffset) instead of global_load
//   PERSIST  0: one workgroup per chunk; N: N workgroups per CU-slot grid-stride
//            over the chunks (grid = min(chunks, 256*N))
//   XCD   workgroups are dealt to the 8 XCDs round-robin by blockIdx; remap so
//         that each XCD streams one contiguous eighth of the arena
//   BAL   balanced grid: as many workgroups as the chip holds at once (occupancy x CUs), each
//         owning one contiguous, equal share of the f4 groups, so every workgroup finishes at the
//         same time instead of a partial last round draining on part of the chip
template <int B_, int V_, int U_, bool NTL_, bool NTS_, bool PIPE_, bool BUF_ = false, int PERSIST_ = 0,
          bool XCD_ = false, bool BAL_ = false>
struct Cfg {
  static constexpr int B = B_, V = V_, U = U_;
  static constexpr bool NTL = NTL_, NTS = NTS_, PIPE = PIPE_, BUF = BUF_;
  static constexpr int PERSIST = PERSIST_;
  static constexpr bool XCD = XCD_, BAL = BAL_;
};

template <bool NT>
__device__ __forceinline__ f4 ld4_buf(const float* base, uint32_t byte_off, uint32_t bytes) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, NT ? 2 : 0));
}

template <bool NT>
__device__ __forceinline__ void st4_off(float* base, uint32_t byte_off, f4 v) {
  __attribute__((address_space(1))) f4* g =
      (__attribute__((address_space(1))) f4*)((__attribute__((address_space(1))) char*)base + byte_off);
  if constexpr (NT) {
    __builtin_nontemporal_store(v, g);
  } else {
    *g = v;
  }
}

template <class C, bool HAS_BASE, bool TWO>
__device__ __forceinline__ void accumulate(f4 (&acc)[C::V], const f4 (&x)[C::U][C::V], const f4 (&b)[C::V],
                                           const AggArgs& a, int i0) {
#pragma unroll
  for (int u = 0; u < C::U; ++u) {
    const float wu = sld(a.w, i0 + u);
    float su = 1.f;
    if constexpr (TWO) su = sld(a.s, i0 + u);
#pragma unroll
    for (int v = 0; v < C::V; ++v) {
      f4 d = HAS_BASE ? f4_sub(x[u][v], b[v]) : x[u][v];
      f4 t = f4_scale(d, wu);
      if constexpr (TWO) t = f4_scale(t, su);
      acc[v] = f4_add(acc[v], t);
    }
  }
}

template <class C>
__device__ __forceinline__ f4 ld_client(const float* p, uint32_t off, const AggArgs& a) {
  if constexpr (C::BUF) {
    return ld4_buf<C::NTL>(p, off, uint32_t(a.n4 * 16u));
  } else {
    return ld4_off<C::NTL>(p, off);
  }
}

template <class C>
__device__ __forceinline__ void load_batch(f4 (&x)[C::U][C::V], const AggArgs& a, int i0,
                                           const uint32_t (&off)[C::V]) {
#pragma unroll
  for (int u = 0; u < C::U; ++u) {
    const float* p = sld(a.xf, i0 + u) + a.x_off;
#pragma unroll
    for (int v = 0; v < C::V; ++v) x[u][v] = ld_client<C>(p, off[v], a);
  }
}

// The lanes of one workgroup own f4 groups g0 + threadIdx.x + v*B (v < V); groups at or past `lim`
// (CHECK only) are clamped loads with no store.
template <class C, bool HAS_BASE, bool TWO, bool CHECK>
__device__ __forceinline__ void vec_at(const AggArgs& a, uint64_t g0, uint64_t lim) {
  constexpr int V = C::V, U = C::U;
  const uint64_t first = g0 + threadIdx.x;

  // Element groups this lane owns, as 32-bit byte offsets (host guarantees an
  // fp32 arena < 4 GiB per launch).  In the (single) partial workgroup the
  // out-of-range lanes load a clamped in-range address (no per-load branch:
  // a predicated load makes hipcc branch around every load and drain vmcnt)
  // and skip only the store.
  uint32_t off[V];
  bool live[V];
  f4 b[V];
  f4 acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const uint64_t e = first + uint64_t(v) * C::B;
    live[v] = !CHECK || e < lim;
    off[v] = uint32_t((CHECK ? (e < lim ? e : lim - 1) : e) * 16u);
    acc[v] = f4_zero();
    b[v] = HAS_BASE ? ld4_off<false>(a.base_f, off[v]) : f4_zero();
  }

  const int K = a.K;
  const int nbatch = K / U;
  if constexpr (C::PIPE) {
    if (nbatch > 0) {
      f4 x0[U][V], x1[U][V];
      load_batch<C>(x0, a, 0, off);
      int j = 0;
      // Two named register sets (no runtime-indexed arrays -> no scratch).
      for (; j + 2 <= nbatch; j += 2) {
        load_batch<C>(x1, a, (j + 1) * U, off);
        accumulate<C, HAS_BASE, TWO>(acc, x0, b, a, j * U);
        if (j + 2 < nbatch) load_batch<C>(x0, a, (j + 2) * U, off);
        accumulate<C, HAS_BASE, TWO>(acc, x1, b, a, (j + 1) * U);
      }
      if (j < nbatch) accumulate<C, HAS_BASE, TWO>(acc, x0, b, a, j * U);
    }
  } else {
    for (int j = 0; j < nbatch; ++j) {
      f4 x[U][V];
      load_batch<C>(x, a, j * U, off);
      accumulate<C, HAS_BASE, TWO>(acc, x, b, a, j * U);
    }
  }
  for (int i = nbatch * U; i < K; ++i) {
    const float* p = sld(a.xf, i) + a.x_off;
    const float wu = sld(a.w, i);
    float su = 1.f;
    if constexpr (TWO) su = sld(a.s, i);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      f4 x = ld_client<C>(p, off[v], a);
      f4 d = HAS_BASE ? f4_sub(x, b[v]) : x;
      f4 t = f4_scale(d, wu);
      if constexpr (TWO) t = f4_scale(t, su);
      acc[v] = f4_add(acc[v], t);
    }
  }

#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (live[v]) st4_off<C::NTS>(a.out_f, off[v], HAS_BASE ? f4_add(b[v], acc[v]) : acc[v]);
  }
}

template <class C, bool HAS_BASE, bool TWO, bool CHECK>
__device__ __forceinline__ void vec_body(const AggArgs& a, uint32_t blk) {
  vec_at<C, HAS_BASE, TWO, CHECK>(a, uint64_t(blk) * (uint64_t(C::B) * C::V), a.n4);
}

// One scalar work item: the fp32 tail element or an int64 entry.  These lanes walk the same K clients
// as the vector lanes, so their loads are batched kSU clients at a time (kSU independent loads in
// flight, then the in-order adds): a one-load-at-a-time walk is K round trips to HBM under the full
// stream's queueing, which outlasted the vector part of the grid (C2: +23 us per launch).
constexpr int kSU = 16;

template <bool HAS_BASE, bool TWO>
__device__ __forceinline__ void scalar_item(const AggArgs& a, uint64_t j) {
  const uint64_t tail = a.n_f32 - 4 * a.n4;
  const int K = a.K;
  if (j < tail) {
    const uint64_t e = 4 * a.n4 + j;
    const float b = HAS_BASE ? a.base_f[e] : 0.f;
    float acc = 0.f;
    int i = 0;
    for (; i + kSU <= K; i += kSU) {
      float x[kSU];
#pragma unroll
      for (int u = 0; u < kSU; ++u) x[u] = ((gfloat*)(sld(a.xf, i + u) + a.x_off))[e];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const float d = HAS_BASE ? x[u] - b : x[u];
        float t = d * sld(a.w, i + u);
        if constexpr (TWO) t = t * sld(a.s, i + u);
        acc = acc + t;
      }
    }
    for (; i < K; ++i) {
      const float x = ((gfloat*)(sld(a.xf, i) + a.x_off))[e];
      const float d = HAS_BASE ? x - b : x;
      float t = d * sld(a.w, i);
      if constexpr (TWO) t = t * sld(a.s, i);
      acc = acc + t;
    }
    a.out_f[e] = HAS_BASE ? b + acc : acc;
    return;
  }
  const uint64_t e = j - tail;
  if (e >= a.n_i64) return;
  typedef __attribute__((address_space(1))) const int64_t gi64;
  const int64_t b = HAS_BASE ? a.base_i[e] : 0;
  float acc = 0.f;
  // int64 subtraction wraps like torch's; the promotion to fp32 happens at the scalar multiply
  // (servers/fedavg.py:154, int tensor * Python float).
  int i = 0;
  for (; i + kSU <= K; i += kSU) {
    int64_t x[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) x[u] = ((gi64*)sld(a.xi, i + u))[e];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x[u] - (uint64_t)b) : x[u];
      float t = (float)d * sld(a.w, i + u);
      if constexpr (TWO) t = t * sld(a.s, i + u);
      acc = acc + t;
    }
  }
  for (; i < K; ++i) {
    const int64_t x = ((gi64*)sld(a.xi, i))[e];
    const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x - (uint64_t)b) : x;
    float t = (float)d * sld(a.w, i);
    if constexpr (TWO) t = t * sld(a.s, i);
    acc = acc + t;
  }
  // update_weights: int64 weight + fp32 delta -> fp32 (float(b) + acc).
  a.out_if[e] = HAS_BASE ? (float)b + acc : acc;
}

template <class C, bool HAS_BASE, bool TWO>
__global__ __launch_bounds__(C::B) void fedavg_kernel(AggArgs a) {
  // the scalar items (fp32 tail, int64 entries) are the first blocks: dispatched first, they run beside
  // the stream from its start instead of after its last round
  if (blockIdx.x < a.nb_scalar) {
    scalar_item<HAS_BASE, TWO>(a, uint64_t(blockIdx.x) * C::B + threadIdx.x);
    return;
  }
  const uint32_t blk = blockIdx.x - a.nb_scalar;
  if constexpr (C::BAL) {
    if (blk < a.nb_grid) {
      // workgroup blk owns f4 groups [lo, hi): equal shares (to one group) of the arena
      const uint64_t lo = uint64_t(blk) * a.n4 / a.nb_grid;
      const uint64_t hi = uint64_t(blk + 1) * a.n4 / a.nb_grid;
      constexpr uint64_t kChunk = uint64_t(C::B) * C::V;
      for (uint64_t g0 = lo; g0 < hi; g0 += kChunk) {
        if (g0 + kChunk <= hi) {
          vec_at<C, HAS_BASE, TWO, false>(a, g0, hi);
        } else {
          vec_at<C, HAS_BASE, TWO, true>(a, g0, hi);
        }
      }
    }
  } else if constexpr (C::XCD) {
    if (blk < a.nb_grid) {
      const uint32_t c = (blk % 8) * a.xcd_per + blk / 8;
      if (c < a.nb_vec_full) {
        vec_body<C, HAS_BASE, TWO, false>(a, c);
      } else if (c < a.nb_vec) {
        vec_body<C, HAS_BASE, TWO, true>(a, c);
      }
    }
  } else if constexpr (C::PERSIST > 0) {
    // a.nb_grid workgroups stride over the nb_vec chunks
    if (blk < a.nb_grid) {
      for (uint32_t c = blk; c < a.nb_vec; c += a.nb_grid) {
        if (c < a.nb_vec_full) {
          vec_body<C, HAS_BASE, TWO, false>(a, c);
        } else {
          vec_body<C, HAS_BASE, TWO, true>(a, c);
        }
      }
    }
  } else {
    if (blk < a.nb_vec_full) {
      vec_body<C, HAS_BASE, TWO, false>(a, blk);
    } else if (blk < a.nb_vec) {
      vec_body<C, HAS_BASE, TWO, true>(a, blk);
    }
  }
}

// ---------------------------------------------------------------------------
// Variant table
// ---------------------------------------------------------------------------
using LaunchFn = void (*)(const AggArgs&, dim3, hipStream_t);

template <class C, bool HAS_BASE, bool TWO>
void launch_one(const AggArgs& a, dim3 grid, hipStream_t st) {
  if constexpr (C::BAL) {
    // the grid the chip holds at once: occupancy of this instantiation x CUs (queried once)
    static int resident = [] {
      int per_cu = 0, cus = 0, dev = 0;
      const bool ok = hipGetDevice(&dev) == hipSuccess &&
                      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fedavg_kernel<C, HAS_BASE, TWO>, C::B,
                                                                   0) == hipSuccess;
      return ok && per_cu > 0 && cus > 0 ? per_cu * cus : 2048;
    }();
    AggArgs b = a;
    b.nb_grid = a.nb_vec < uint32_t(resident) ? a.nb_vec : uint32_t(resident);
    hipLaunchKernelGGL((fedavg_kernel<C, HAS_BASE, TWO>), dim3(b.nb_grid + a.nb_scalar), dim3(C::B), 0, st, b);
    return;
  }
  hipLaunchKernelGGL((fedavg_kernel<C, HAS_BASE, TWO>), grid, dim3(C::B), 0, st, a);
}

struct Variant {
  int B, V, U;
  bool NTL, NTS, PIPE, BUF;
  int PERSIST;
  bool XCD, BAL;
  LaunchFn fn[2][2];  // [HAS_BASE][TWO]
};

template <class C>
constexpr Variant make_variant() {
  return Variant{C::B, C::V, C::U, C::NTL, C::NTS, C::PIPE, C::BUF, C::PERSIST, C::XCD, C::BAL,
                 {{&launch_one<C, false, false>, &launch_one<C, false, true>},
                  {&launch_one<C, true, false>, &launch_one<C, true, true>}}};
}

// Variant 0 is the default of the public entry points: one-wave (64-thread) workgroups, NT loads and
// stores.  256-thread workgroups were the default of rounds 1-4; with the scalar items
// moved to the front of the grid the one-wave form ran 1-2.5 % faster on every C2 / C3 shape and up to
// 9 % on the small per-rank pieces of N > 1, on two boxes (profiles/r05b_anchor.log, r05c_anchor.log;
// DESIGN.md §15).
#ifdef PLATO_AGG_TUNE  // libplato_agg_tune.so: every variant (bench.py --sweep, scripts/)
// The round-1 sweep of 18 shapes (profiles/r01_sweep.log) is trimmed to one of each
// kind; bench.py --sweep interleaves these.
const Variant kVariants[] = {
    make_variant<Cfg<64, 1, 8, true, true, false>>(),                    // 0 (default): one wave, NT loads + stores
    make_variant<Cfg<256, 2, 8, false, false, false>>(),                 // 1 first version
    make_variant<Cfg<256, 1, 8, false, false, false>>(),                 // 2 plain loads
    make_variant<Cfg<256, 1, 8, true, true, true>>(),                    // 3 pipelined
    make_variant<Cfg<256, 1, 8, true, true, false, true>>(),             // 4 buffer loads (nt)
    make_variant<Cfg<256, 1, 8, true, true, false, false, 8>>(),         // 5 persistent 8/CU
    make_variant<Cfg<256, 1, 8, true, true, false, false, 0, true>>(),   // 6 XCD-contiguous chunks
    make_variant<Cfg<256, 1, 16, true, true, false>>(),                  // 7 16 clients per batch
    make_variant<Cfg<256, 1, 32, true, true, false>>(),                  // 8 32 clients per batch
    make_variant<Cfg<256, 1, 8, true, true, false, false, 0, false, true>>(),   // 9 balanced grid
    make_variant<Cfg<256, 1, 16, true, true, false, false, 0, false, true>>(),  // 10 balanced, U=16
    make_variant<Cfg<256, 1, 8, true, true, false>>(),                   // 11 the rounds 1-4 default (4 waves)
    make_variant<Cfg<64, 1, 16, true, true, false>>(),                   // 12 one wave, 16 clients per batch
    make_variant<Cfg<128, 1, 8, true, true, false>>(),                   // 13 two waves
};
#else  // libplato_agg.so: the default only
const Variant kVariants[] = {
    make_variant<Cfg<64, 1, 8, true, true, false>>(),               // 0 (default): one wave, NT loads + stores
};
#endif
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// Tuning/test knob: f4 groups per launch (0 = the 4 GiB limit); lets tests
// exercise the split path on small arenas.
uint64_t g_launch_groups = 0;

int run_agg_range(const Variant& vr, bool has_base, const float* const* xf, const int64_t* const* xi,
                  const float* w, const float* s, int K, const float* base_f, const int64_t* base_i,
                  float* out_f, float* out_if, size_t n_f32, size_t n_i64, uint64_t x_off, hipStream_t st);

int run_agg(int variant, bool has_base, const float* const* xf, const int64_t* const* xi,
            const float* w, const float* s, int K, const float* base_f, const int64_t* base_i,
            float* out_f, float* out_if, size_t n_f32, size_t n_i64, hipStream_t st) {
  if (variant < 0 || variant >= kNumVariants) return fail(PLATO_AGG_EINVAL, "bad variant");
  if (K <= 0) return fail(PLATO_AGG_EINVAL, "K must be >= 1");
  if (!w) return fail(PLATO_AGG_EINVAL, "null weight array");
  if (n_f32 && (!xf || !out_f)) return fail(PLATO_AGG_EINVAL, "null fp32 arena pointer");
  if (n_i64 && (!xi || !out_if)) return fail(PLATO_AGG_EINVAL, "null int64 arena pointer");
  if (has_base && n_f32 && !base_f) return fail(PLATO_AGG_EINVAL, "null fp32 baseline");
  if (has_base && n_i64 && !base_i) return fail(PLATO_AGG_EINVAL, "null int64 baseline");
  if (n_f32 && (!aligned16(out_f) || (has_base && !aligned16(base_f))))
    return fail(PLATO_AGG_EINVAL, "fp32 baseline/output must be 16-byte aligned");
  if (n_f32 == 0 && n_i64 == 0) {
    g_last_error.clear();
    return PLATO_AGG_OK;
  }
  const Variant& vr = kVariants[variant];
  // Lanes address their element groups with 32-bit byte offsets, so one launch
  // covers < 4 GiB of the fp32 arena; larger arenas (models > ~1 B parameters)
  // run as consecutive launches over whole-chunk ranges, each offsetting the
  // client pointers in the kernel (x_off) and the baseline/output on the host.
  // Every element still sums its K clients in order: results do not depend on
  // the split.
  const uint64_t chunk = uint64_t(vr.B) * vr.V;
  const uint64_t n4_all = n_f32 / 4;
  const uint64_t range = g_launch_groups ? (g_launch_groups + chunk - 1) / chunk * chunk
                                         : ((0xffffffffull / 16) / chunk) * chunk;
  uint64_t g0 = 0;
  for (; n4_all - g0 > range; g0 += range) {
    const int rc = run_agg_range(vr, has_base, xf, nullptr, w, s, K, base_f ? base_f + 4 * g0 : nullptr, nullptr,
                                 out_f + 4 * g0, nullptr, 4 * range, 0, 4 * g0, st);
    if (rc != PLATO_AGG_OK) return rc;
  }
  return run_agg_range(vr, has_base, xf, xi, w, s, K, base_f ? base_f + 4 * g0 : nullptr, base_i,
                       n_f32 ? out_f + 4 * g0 : out_f, out_if, n_f32 - 4 * g0, n_i64, 4 * g0, st);
}

int run_agg_range(const Variant& vr, bool has_base, const float* const* xf, const int64_t* const* xi,
                  const float* w, const float* s, int K, const float* base_f, const int64_t* base_i,
                  float* out_f, float* out_if, size_t n_f32, size_t n_i64, uint64_t x_off, hipStream_t st) {
  if (n_f32 == 0 && n_i64 == 0) {
    g_last_error.clear();
    return PLATO_AGG_OK;
  }
  AggArgs a{};
  a.x_off = x_off;
  a.xf = xf;
  a.xi = xi;
  a.w = w;
  a.s = s;
  a.base_f = base_f;
  a.base_i = base_i;
  a.out_f = out_f;
  a.out_if = out_if;
  a.n4 = n_f32 / 4;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.K = K;
  const uint64_t chunk = uint64_t(vr.B) * vr.V;
  const uint64_t nb_vec = (a.n4 + chunk - 1) / chunk;
  const uint64_t n_scalar = (n_f32 - 4 * a.n4) + n_i64;
  const uint64_t nb_scalar = (n_scalar + vr.B - 1) / vr.B;
  if (nb_vec + nb_scalar > 0x7fffffffull || a.n4 * 16ull > 0xffffffffull)
    return fail(PLATO_AGG_EINVAL, "launch range exceeds 4 GiB (internal split error)");
  a.nb_vec = uint32_t(nb_vec);
  a.nb_vec_full = uint32_t(a.n4 / chunk);
  a.nb_grid = a.nb_vec;
  a.xcd_per = 0;
  if (vr.XCD) {
    a.xcd_per = uint32_t((nb_vec + 7) / 8);
    a.nb_grid = 8 * a.xcd_per;  // up to 7 vector blocks idle
  }
  if (vr.PERSIST > 0) {
    const uint64_t cap = uint64_t(256) * vr.PERSIST;  // 256 CUs on MI355X
    a.nb_grid = uint32_t(nb_vec < cap ? nb_vec : cap);
  }
  a.nb_scalar = uint32_t(nb_scalar);
  dim3 grid(uint32_t(a.nb_grid + nb_scalar));
  vr.fn[has_base ? 1 : 0][s ? 1 : 0](a, grid, st);
  return check_launch("fedavg kernel launch");
}

// ---------------------------------------------------------------------------
// bf16 client payloads (Plato's model_quantize / model_dequantize codec,
// plato/processors/model_quantize.py:15, model_dequantize.py:15-18): the
// server dequantizes with .to(float32) before aggregating, which is exact, so
// the kernel keeps the payload in bf16 through PCIe and HBM and widens in
// registers (bits << 16).  Each lane owns 8 elements: one 16-byte bf16 load
// per client, two float4 for the baseline and the result.  int64 entries
// arrive as bf16 too (model_quantize converts every layer), and the
// reference then subtracts the int64 baseline in fp32 (tensor promotion):
// d = fp32(x) - fp32(b).
// ---------------------------------------------------------------------------
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u4 gu4;

__device__ __forceinline__ float bf16_lo(unsigned int w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(unsigned int w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf16_at(const uint16_t* p, uint64_t e) {
  return __uint_as_float(uint32_t(p[e]) << 16);
}

struct Bf16Args {
  const uint16_t* const* xf;   // K pointers to n_f32 bf16
  const uint16_t* const* xi;   // K pointers to n_i64 bf16 (int64 entries, quantized)
  const float* w;
  const float* s;
  const float* base_f;
  const int64_t* base_i;
  float* out_f;
  float* out_if;
  uint64_t n8, n_f32, n_i64;
  uint32_t nb_vec, nb_vec_full;
  uint32_t nb_scalar;  // workgroups of scalar items: the FIRST blocks of the grid
  uint64_t x_off;  // element offset of this launch's range in every client arena
  int K;
};

template <bool TWO, bool CHECK, int U, int B>
__device__ __forceinline__ void bf16_body(const Bf16Args& a, uint32_t blk) {
  const uint64_t e8 = uint64_t(blk) * B + threadIdx.x;
  const bool live = !CHECK || e8 < a.n8;
  const uint64_t g = CHECK ? (e8 < a.n8 ? e8 : a.n8 - 1) : e8;
  const uint32_t xoff = uint32_t(g * 16u);   // bf16 bytes
  const uint32_t foff = uint32_t(g * 32u);   // fp32 bytes
  const f4 b0 = ld4_off<false>(a.base_f, foff);
  const f4 b1 = ld4_off<false>(a.base_f, foff + 16u);
  f4 acc0 = f4_zero(), acc1 = f4_zero();
  const int K = a.K;
  int i = 0;
  for (; i + U <= K; i += U) {
    u4 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint16_t* p = sld(a.xf, i + u) + a.x_off;
      q[u] = __builtin_nontemporal_load((gu4*)((__attribute__((address_space(1))) const char*)p + xoff));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wu = sld(a.w, i + u);
      float su = 1.f;
      if constexpr (TWO) su = sld(a.s, i + u);
      const f4 x0 = f4{bf16_lo(q[u].x), bf16_hi(q[u].x), bf16_lo(q[u].y), bf16_hi(q[u].y)};
      const f4 x1 = f4{bf16_lo(q[u].z), bf16_hi(q[u].z), bf16_lo(q[u].w), bf16_hi(q[u].w)};
      f4 t0 = f4_scale(x0 - b0, wu), t1 = f4_scale(x1 - b1, wu);
      if constexpr (TWO) {
        t0 = f4_scale(t0, su);
        t1 = f4_scale(t1, su);
      }
      acc0 = acc0 + t0;
      acc1 = acc1 + t1;
    }
  }
  for (; i < K; ++i) {
    const uint16_t* p = sld(a.xf, i) + a.x_off;
    const u4 q = __builtin_nontemporal_load((gu4*)((__attribute__((address_space(1))) const char*)p + xoff));
    const float wu = sld(a.w, i);
    float su = 1.f;
    if constexpr (TWO) su = sld(a.s, i);
    const f4 x0 = f4{bf16_lo(q.x), bf16_hi(q.x), bf16_lo(q.y), bf16_hi(q.y)};
    const f4 x1 = f4{bf16_lo(q.z), bf16_hi(q.z), bf16_lo(q.w), bf16_hi(q.w)};
    f4 t0 = f4_scale(x0 - b0, wu), t1 = f4_scale(x1 - b1, wu);
    if constexpr (TWO) {
      t0 = f4_scale(t0, su);
      t1 = f4_scale(t1, su);
    }
    acc0 = acc0 + t0;
    acc1 = acc1 + t1;
  }
  if (live) {
    st4_off<true>(a.out_f, foff, b0 + acc0);
    st4_off<true>(a.out_f, foff + 16u, b1 + acc1);
  }
}

// 4 elements per lane: one 8-byte bf16 load per client, one float4 for the
// baseline and the result (the fp32 kernel's lane mapping: 1 KiB per wave
// instruction on the fp32 side, twice the workgroups of the 8-per-lane body).
typedef unsigned int u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u2 gu2;

template <bool TWO, bool CHECK, int U, int B>
__device__ __forceinline__ void bf16_body4(const Bf16Args& a, uint32_t blk) {
  const uint64_t n4 = a.n8 * 2;  // groups of 4 (n8 counts groups of 8 in this mode: see launcher)
  const uint64_t e4 = uint64_t(blk) * B + threadIdx.x;
  const bool live = !CHECK || e4 < n4;
  const uint64_t g = CHECK ? (e4 < n4 ? e4 : n4 - 1) : e4;
  const uint32_t xoff = uint32_t(g * 8u);
  const uint32_t foff = uint32_t(g * 16u);
  const f4 b = ld4_off<false>(a.base_f, foff);
  f4 acc = f4_zero();
  const int K = a.K;
  int i = 0;
  for (; i + U <= K; i += U) {
    u2 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint16_t* p = sld(a.xf, i + u) + a.x_off;
      q[u] = __builtin_nontemporal_load((gu2*)((__attribute__((address_space(1))) const char*)p + xoff));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wu = sld(a.w, i + u);
      const f4 x = f4{bf16_lo(q[u].x), bf16_hi(q[u].x), bf16_lo(q[u].y), bf16_hi(q[u].y)};
      f4 t = f4_scale(x - b, wu);
      if constexpr (TWO) t = f4_scale(t, sld(a.s, i + u));
      acc = acc + t;
    }
  }
  for (; i < K; ++i) {
    const uint16_t* p = sld(a.xf, i) + a.x_off;
    const u2 q = __builtin_nontemporal_load((gu2*)((__attribute__((address_space(1))) const char*)p + xoff));
    const f4 x = f4{bf16_lo(q.x), bf16_hi(q.x), bf16_lo(q.y), bf16_hi(q.y)};
    f4 t = f4_scale(x - b, sld(a.w, i));
    if constexpr (TWO) t = f4_scale(t, sld(a.s, i));
    acc = acc + t;
  }
  if (live) st4_off<true>(a.out_f, foff, b + acc);
}

// One scalar item (fp32 tail element or int64 entry): K clients in order, kSU loads per round trip.
template <bool TWO>
__device__ __forceinline__ void bf16_scalar(const Bf16Args& a, uint64_t j) {
  const uint64_t tail = a.n_f32 - 8 * a.n8;
  const int K = a.K;
  const bool f32 = j < tail;
  const uint64_t e = f32 ? 8 * a.n8 + j : j - tail;
  if (!f32 && e >= a.n_i64) return;
  const uint16_t* const* xs = f32 ? a.xf : a.xi;
  const uint64_t xe = f32 ? a.x_off + e : e;
  const float b = f32 ? a.base_f[e] : (float)a.base_i[e];
  float acc = 0.f;
  int i = 0;
  for (; i + kSU <= K; i += kSU) {
    float x[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) x[u] = bf16_at(sld(xs, i + u), xe);
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      float t = (x[u] - b) * sld(a.w, i + u);
      if constexpr (TWO) t = t * sld(a.s, i + u);
      acc = acc + t;
    }
  }
  for (; i < K; ++i) {
    float t = (bf16_at(sld(xs, i), xe) - b) * sld(a.w, i);
    if constexpr (TWO) t = t * sld(a.s, i);
    acc = acc + t;
  }
  if (f32) {
    a.out_f[e] = b + acc;
  } else {
    a.out_if[e] = b + acc;
  }
}

template <bool TWO, int LANE, int U, int B>
__global__ __launch_bounds__(B) void fedavg_bf16_kernel(Bf16Args a) {
  // scalar items first (dispatched first, beside the stream: see fedavg_kernel)
  if (blockIdx.x < a.nb_scalar) {
    bf16_scalar<TWO>(a, uint64_t(blockIdx.x) * B + threadIdx.x);
    return;
  }
  const uint32_t blk = blockIdx.x - a.nb_scalar;
  if (blk < a.nb_vec_full) {
    if constexpr (LANE == 8) bf16_body<TWO, false, U, B>(a, blk); else bf16_body4<TWO, false, U, B>(a, blk);
  } else if (blk < a.nb_vec) {
    if constexpr (LANE == 8) bf16_body<TWO, true, U, B>(a, blk); else bf16_body4<TWO, true, U, B>(a, blk);
  }
}

using Bf16Fn = void (*)(const Bf16Args&, dim3, hipStream_t);
template <bool TWO, int LANE, int U, int B>
void launch_bf16(const Bf16Args& a, dim3 g, hipStream_t st) {
  hipLaunchKernelGGL((fedavg_bf16_kernel<TWO, LANE, U, B>), g, dim3(B), 0, st, a);
}
struct Bf16Variant {
  int lane, u, block;
  Bf16Fn fn[2];
};
// variant 0 is the default of plato_agg_fedavg_weights_bf16: one-wave workgroups, as fedavg_kernel's
#ifdef PLATO_AGG_TUNE
const Bf16Variant kBf16Variants[] = {
    {4, 8, 64, {&launch_bf16<false, 4, 8, 64>, &launch_bf16<true, 4, 8, 64>}},
    {8, 8, 256, {&launch_bf16<false, 8, 8, 256>, &launch_bf16<true, 8, 8, 256>}},
    {4, 16, 256, {&launch_bf16<false, 4, 16, 256>, &launch_bf16<true, 4, 16, 256>}},
    {8, 4, 256, {&launch_bf16<false, 8, 4, 256>, &launch_bf16<true, 8, 4, 256>}},
    {4, 8, 256, {&launch_bf16<false, 4, 8, 256>, &launch_bf16<true, 4, 8, 256>}},  // the rounds 2-4 default
    {8, 8, 64, {&launch_bf16<false, 8, 8, 64>, &launch_bf16<true, 8, 8, 64>}},
};
#else
const Bf16Variant kBf16Variants[] = {
    {4, 8, 64, {&launch_bf16<false, 4, 8, 64>, &launch_bf16<true, 4, 8, 64>}},
};
#endif
constexpr int kNumBf16Variants = sizeof(kBf16Variants) / sizeof(kBf16Variants[0]);

// ---------------------------------------------------------------------------
// Ceiling probes (tuning only): how fast this chip streams the same bytes with
// no arithmetic dependence.  mode 0: NT read + NT write copy; mode 1: NT read
// only (per-lane xor kept live by a conditional store that never fires).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void stream_probe(const f4* __restrict__ src, f4* __restrict__ dst, uint64_t n4,
                                                    uint32_t unroll) {
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (; i + 7 * stride < n4; i += 8 * stride) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load((gf4*)src + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (MODE == 0) {
        __builtin_nontemporal_store(v[u], (__attribute__((address_space(1))) f4*)dst + i + u * stride);
      } else {
        acc += v[u];
      }
    }
  }
  for (; i < n4; i += stride) {
    f4 v = __builtin_nontemporal_load((gf4*)src + i);
    if constexpr (MODE == 0) {
      __builtin_nontemporal_store(v, (__attribute__((address_space(1))) f4*)dst + i);
    } else {
      acc += v;
    }
  }
  if constexpr (MODE == 1) {
    if (acc.x == 1234.5f && acc.y == -1234.5f) dst[0] = acc;  // keeps the loads live
  }
  (void)unroll;
}

// ---------------------------------------------------------------------------
// Elementwise helpers (off the hot path; grid-stride, f4 where possible)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t gtid() { return uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return uint64_t(gridDim.x) * blockDim.x; }

dim3 grid_for(uint64_t work) {
  uint64_t b = (work + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;  // grid-stride the rest (32 waves/CU x 256 CUs)
  return dim3(uint32_t(b));
}

// x / o (and xi / oi) may be the same arena: the delta arenas convert a staged row in place (x -= b),
// so they carry no __restrict__; each element is read once, then written, by the same lane.
__global__ __launch_bounds__(kBlock) void deltas_kernel(const float* x, const int64_t* xi,
                                                        const float* __restrict__ b, const int64_t* __restrict__ bi,
                                                        float* o, int64_t* oi, uint64_t n_f32, uint64_t n_i64) {
  const uint64_t n4 = n_f32 / 4;
  for (uint64_t k = gtid(); k < n4; k += gstride()) {
    reinterpret_cast<f4*>(o)[k] =
        f4_sub(reinterpret_cast<const f4*>(x)[k], reinterpret_cast<const f4*>(b)[k]);
  }
  const uint64_t tail = n_f32 - 4 * n4;
  for (uint64_t k = gtid(); k < tail + n_i64; k += gstride()) {
    if (k < tail) {
      o[4 * n4 + k] = x[4 * n4 + k] - b[4 * n4 + k];
    } else {
      const uint64_t e = k - tail;
      oi[e] = (int64_t)((uint64_t)xi[e] - (uint64_t)bi[e]);
    }
  }
}

__global__ __launch_bounds__(kBlock) void update_kernel(const float* b, const int64_t* __restrict__ bi,
                                                        const float* avg, const float* __restrict__ avgi,
                                                        float* o, float* __restrict__ oi, uint64_t n_f32,
                                                        uint64_t n_i64) {
  const uint64_t n4 = n_f32 / 4;
  for (uint64_t k = gtid(); k < n4; k += gstride()) {
    reinterpret_cast<f4*>(o)[k] =
        f4_add(reinterpret_cast<const f4*>(b)[k], reinterpret_cast<const f4*>(avg)[k]);
  }
  const uint64_t tail = n_f32 - 4 * n4;
  for (uint64_t k = gtid(); k < tail + n_i64; k += gstride()) {
    if (k < tail) {
      o[4 * n4 + k] = b[4 * n4 + k] + avg[4 * n4 + k];
    } else {
      const uint64_t e = k - tail;
      oi[e] = (float)bi[e] + avgi[e];
    }
  }
}

__device__ __forceinline__ int64_t trunc_f32_i64(float f) {
  // x86-64 cvttss2si semantics: NaN / out of range -> INT64_MIN.
  if (!(f >= -9223372036854775808.0f && f < 9223372036854775808.0f)) return INT64_MIN;
  return (int64_t)f;
}

__global__ __launch_bounds__(kBlock) void cast_kernel(const float* __restrict__ s, int64_t* __restrict__ d,
                                                      uint64_t n) {
  for (uint64_t k = gtid(); k < n; k += gstride()) d[k] = trunc_f32_i64(s[k]);
}

__global__ __launch_bounds__(kBlock) void mix_kernel(const float* __restrict__ x, const int64_t* __restrict__ xi,
                                                     const float* b, const int64_t* __restrict__ bi, float om,
                                                     float m, float* o, float* __restrict__ oi, uint64_t n_f32,
                                                     uint64_t n_i64) {
  const uint64_t n4 = n_f32 / 4;
  for (uint64_t k = gtid(); k < n4; k += gstride()) {
    f4 bb = reinterpret_cast<const f4*>(b)[k];
    f4 xx = reinterpret_cast<const f4*>(x)[k];
    reinterpret_cast<f4*>(o)[k] = f4_add(f4_scale(bb, om), f4_scale(xx, m));
  }
  const uint64_t tail = n_f32 - 4 * n4;
  for (uint64_t k = gtid(); k < tail + n_i64; k += gstride()) {
    if (k < tail) {
      const uint64_t e = 4 * n4 + k;
      o[e] = b[e] * om + x[e] * m;
    } else {
      const uint64_t e = k - tail;
      oi[e] = (float)bi[e] * om + (float)xi[e] * m;
    }
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void synth_f32_kernel(float* o, const float* add, uint64_t n, uint64_t key,
                                                           float scale) {
  for (uint64_t k = gtid(); k < n; k += gstride()) {
    const uint64_t h = splitmix64(key + k);
    const int32_t r = int32_t(h >> 40) - (1 << 23);
    const float v = float(r) * scale;
    o[k] = add ? add[k] + v : v;
  }
}

__global__ __launch_bounds__(kBlock) void synth_i64_kernel(int64_t* o, const int64_t* add, uint64_t n, uint64_t key,
                                                           uint64_t mod) {
  for (uint64_t k = gtid(); k < n; k += gstride()) {
    const int64_t v = int64_t(splitmix64(key + k) % mod);
    o[k] = add ? (int64_t)((uint64_t)add[k] + (uint64_t)v) : v;
  }
}

uint64_t synth_key(uint64_t seed, uint64_t stream_id) {
  uint64_t z = seed ^ (stream_id * 0xD1B54A32D192ED03ull);
  // host copy of splitmix64
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int plato_agg_abi_version(void) { return PLATO_AGG_ABI_VERSION; }

const char* plato_agg_last_error(void) { return g_last_error.c_str(); }

int plato_agg_fedavg_weights(const float* const* d_x_f32, const int64_t* const* d_x_i64, const float* d_w,
                             const float* d_s, int K, const float* d_base_f32, const int64_t* d_base_i64,
                             float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64,
                             hipStream_t stream) {
  return run_agg(0, true, d_x_f32, d_x_i64, d_w, d_s, K, d_base_f32, d_base_i64, d_out_f32, d_out_i64f, n_f32,
                 n_i64, stream);
}

int plato_agg_fedavg_deltas(const float* const* d_d_f32, const int64_t* const* d_d_i64, const float* d_w,
                            const float* d_s, int K, float* d_avg_f32, float* d_avg_i64f, size_t n_f32,
                            size_t n_i64, hipStream_t stream) {
  return run_agg(0, false, d_d_f32, d_d_i64, d_w, d_s, K, nullptr, nullptr, d_avg_f32, d_avg_i64f, n_f32, n_i64,
                 stream);
}

}  // extern "C"

namespace {
// ---------------------------------------------------------------------------
// float64 weights on the fp32 entries (the reference's numpy/torch promotion):
//   acc = fp32( double(acc) + double(d) * w64_i )      d = x - b (fp32) or x
// int64 entries keep the fp32 chain with their own weights w_i64:
//   acc = acc + fp32(fp32(d) * w_i64_i)
// RL server: `delta * self.smart_weighting[i]` with a float64 [K, 1] numpy
// action (rl_server.py:66-71) is a float64 tensor added into the fp32 average
// (in-place add in float64, then cast); its int64 entries use
// smart_weighting[i][0] as a Python scalar.
// Streaming shape of the fp32 kernel: a float4 group per lane, clients in
// order, 4 clients' loads in flight; HBM-bound (fp64 is cheap on MI355X).
// ---------------------------------------------------------------------------
struct W64Args {
  const float* const* xf;
  const int64_t* const* xi;
  const double* w64;
  const float* wi;
  const float* base_f;
  const int64_t* base_i;
  float* out_f;
  float* out_if;
  uint64_t n4, n_f32, n_i64;
  uint32_t nb_vec;
  uint32_t nb_scalar;  // workgroups of scalar items: the FIRST blocks of the grid (see fedavg_kernel)
  int K;
};

template <bool HAS_BASE>
__global__ __launch_bounds__(256) void fedavg_w64_kernel(W64Args a) {
  const uint32_t blk = blockIdx.x - a.nb_scalar;
  if (blockIdx.x >= a.nb_scalar) {
    const uint64_t g = uint64_t(blk) * 256 + threadIdx.x;
    if (g >= a.n4) return;
    const uint32_t off = uint32_t(g * 16u);
    const f4 b = HAS_BASE ? ld4_off<false>(a.base_f, off) : f4_zero();
    f4 acc = f4_zero();
    int i = 0;
    for (; i + 4 <= a.K; i += 4) {
      f4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = ld4_off<true>(sld(a.xf, i + u), off);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double w = sld(a.w64, i + u);
        const f4 d = HAS_BASE ? f4_sub(x[u], b) : x[u];
        acc.x = float(double(acc.x) + double(d.x) * w);
        acc.y = float(double(acc.y) + double(d.y) * w);
        acc.z = float(double(acc.z) + double(d.z) * w);
        acc.w = float(double(acc.w) + double(d.w) * w);
      }
    }
    for (; i < a.K; ++i) {
      const f4 x = ld4_off<true>(sld(a.xf, i), off);
      const double w = sld(a.w64, i);
      const f4 d = HAS_BASE ? f4_sub(x, b) : x;
      acc.x = float(double(acc.x) + double(d.x) * w);
      acc.y = float(double(acc.y) + double(d.y) * w);
      acc.z = float(double(acc.z) + double(d.z) * w);
      acc.w = float(double(acc.w) + double(d.w) * w);
    }
    st4_off<true>(a.out_f, off, HAS_BASE ? f4_add(b, acc) : acc);
    return;
  }
  // scalar items: kSU client loads per round trip, then the in-order adds
  const uint64_t j = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t tail = a.n_f32 - 4 * a.n4;
  const int K = a.K;
  if (j < tail) {
    const uint64_t e = 4 * a.n4 + j;
    const float b = HAS_BASE ? a.base_f[e] : 0.f;
    float acc = 0.f;
    int i = 0;
    for (; i + kSU <= K; i += kSU) {
      float x[kSU];
#pragma unroll
      for (int u = 0; u < kSU; ++u) x[u] = ((gfloat*)sld(a.xf, i + u))[e];
#pragma unroll
      for (int u = 0; u < kSU; ++u) {
        const float d = HAS_BASE ? x[u] - b : x[u];
        acc = float(double(acc) + double(d) * sld(a.w64, i + u));
      }
    }
    for (; i < K; ++i) {
      const float x = sld(a.xf, i)[e];
      const float d = HAS_BASE ? x - b : x;
      acc = float(double(acc) + double(d) * sld(a.w64, i));
    }
    a.out_f[e] = HAS_BASE ? b + acc : acc;
    return;
  }
  const uint64_t e = j - tail;
  if (e >= a.n_i64) return;
  typedef __attribute__((address_space(1))) const int64_t gi64;
  const int64_t b = HAS_BASE ? a.base_i[e] : 0;
  float acc = 0.f;
  int i = 0;
  for (; i + kSU <= K; i += kSU) {
    int64_t x[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) x[u] = ((gi64*)sld(a.xi, i + u))[e];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x[u] - (uint64_t)b) : x[u];
      acc = acc + (float)d * sld(a.wi, i + u);
    }
  }
  for (; i < K; ++i) {
    const int64_t x = sld(a.xi, i)[e];
    const int64_t d = HAS_BASE ? (int64_t)((uint64_t)x - (uint64_t)b) : x;
    acc = acc + (float)d * sld(a.wi, i);
  }
  a.out_if[e] = HAS_BASE ? (float)b + acc : acc;
}
}  // namespace

namespace {
// float64 weighted sum (HE plaintext half): acc = acc + x_i * w_i, float64,
// separately rounded, clients in order; two doubles per lane (16-byte loads).
typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const d2 gd2;

__global__ __launch_bounds__(256) void weighted_sum_f64_kernel(const double* const* xs, const double* w, int K,
                                                               double* out, uint64_t n) {
  const uint64_t g = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t n2 = n / 2;
  if (g < n2) {
    d2 acc = d2{0.0, 0.0};
    int i = 0;
    for (; i + 4 <= K; i += 4) {
      d2 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load((gd2*)(sld(xs, i + u)) + g);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = acc + x[u] * sld(w, i + u);
    }
    for (; i < K; ++i) acc = acc + __builtin_nontemporal_load((gd2*)(sld(xs, i)) + g) * sld(w, i);
    ((__attribute__((address_space(1))) d2*)out)[g] = acc;
  } else if (g == n2 && (n & 1)) {
    double acc = 0.0;
    for (int i = 0; i < K; ++i) acc = acc + sld(xs, i)[n - 1] * sld(w, i);
    out[n - 1] = acc;
  }
}
}  // namespace

extern "C" {

int plato_agg_weighted_sum_f64(const double* const* d_x, const double* d_w, int K, double* d_out, size_t n,
                               hipStream_t stream) {
  if (K <= 0) return fail(PLATO_AGG_EINVAL, "K must be >= 1");
  if (!n) return plato_agg_internal::clear_error();
  if (!d_x || !d_w || !d_out) return fail(PLATO_AGG_EINVAL, "null pointer");
  if (!aligned16(d_out)) return fail(PLATO_AGG_EINVAL, "output must be 16-byte aligned");
  const uint64_t threads = n / 2 + 1;
  hipLaunchKernelGGL(weighted_sum_f64_kernel, dim3(uint32_t((threads + 255) / 256)), dim3(256), 0, stream, d_x,
                     d_w, K, d_out, uint64_t(n));
  return check_launch("weighted_sum_f64 launch");
}

int plato_agg_fedavg_w64(const float* const* d_x_f32, const int64_t* const* d_x_i64, const double* d_w64,
                         const float* d_w_i64, int K, const float* d_base_f32, const int64_t* d_base_i64,
                         float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64, hipStream_t stream) {
  if (K <= 0) return fail(PLATO_AGG_EINVAL, "K must be >= 1");
  if (n_f32 && (!d_x_f32 || !d_w64 || !d_out_f32)) return fail(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_i64 && (!d_x_i64 || !d_w_i64 || !d_out_i64f)) return fail(PLATO_AGG_EINVAL, "null int64 pointer");
  const bool has_base = d_base_f32 != nullptr || d_base_i64 != nullptr;
  if (has_base && ((n_f32 && !d_base_f32) || (n_i64 && !d_base_i64)))
    return fail(PLATO_AGG_EINVAL, "baseline given for one region only");
  if (n_f32 && (!aligned16(d_out_f32) || (has_base && !aligned16(d_base_f32))))
    return fail(PLATO_AGG_EINVAL, "fp32 baseline/output must be 16-byte aligned");
  if (n_f32 + n_i64 == 0) return plato_agg_internal::clear_error();
  W64Args a{};
  a.xf = d_x_f32;
  a.xi = d_x_i64;
  a.w64 = d_w64;
  a.wi = d_w_i64;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.out_f = d_out_f32;
  a.out_if = d_out_i64f;
  a.n4 = n_f32 / 4;
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.K = K;
  if (a.n4 * 16ull > 0xffffffffull) return fail(PLATO_AGG_EINVAL, "fp32 arena must be < 4 GiB for float64 weights");
  const uint64_t nb_vec = (a.n4 + 255) / 256;
  const uint64_t nb_scalar = ((n_f32 - 4 * a.n4) + n_i64 + 255) / 256;
  a.nb_vec = uint32_t(nb_vec);
  a.nb_scalar = uint32_t(nb_scalar);
  const dim3 grid(uint32_t(nb_vec + nb_scalar));
  if (has_base) {
    hipLaunchKernelGGL(fedavg_w64_kernel<true>, grid, dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL(fedavg_w64_kernel<false>, grid, dim3(256), 0, stream, a);
  }
  return check_launch("fedavg_w64 launch");
}

namespace {
int run_bf16_range(const Bf16Variant& vr, const uint16_t* const* d_x_bf16, const uint16_t* const* d_x_i64_bf16,
                   const float* d_w, const float* d_s, int K, const float* d_base_f32, const int64_t* d_base_i64,
                   float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64, uint64_t x_off,
                   hipStream_t stream);

int run_bf16(int variant, const uint16_t* const* d_x_bf16, const uint16_t* const* d_x_i64_bf16, const float* d_w,
             const float* d_s, int K, const float* d_base_f32, const int64_t* d_base_i64, float* d_out_f32,
             float* d_out_i64f, size_t n_f32, size_t n_i64, hipStream_t stream) {
  if (variant < 0 || variant >= kNumBf16Variants) return fail(PLATO_AGG_EINVAL, "bad bf16 variant");
  if (K <= 0) return fail(PLATO_AGG_EINVAL, "K must be >= 1");
  if (!d_w) return fail(PLATO_AGG_EINVAL, "null weight array");
  if (n_f32 && (!d_x_bf16 || !d_base_f32 || !d_out_f32)) return fail(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_i64 && (!d_x_i64_bf16 || !d_base_i64 || !d_out_i64f)) return fail(PLATO_AGG_EINVAL, "null int64 pointer");
  if (n_f32 && (!aligned16(d_base_f32) || !aligned16(d_out_f32)))
    return fail(PLATO_AGG_EINVAL, "fp32 baseline/output must be 16-byte aligned");
  if (n_f32 + n_i64 == 0) return plato_agg_internal::clear_error();
  const Bf16Variant& vr = kBf16Variants[variant];
  // < 4 GiB of fp32 output per launch (32-bit lane offsets): larger arenas run
  // as consecutive whole-block ranges, as in run_agg.
  const uint64_t n8_all = n_f32 / 8;
  const uint64_t range8 = g_launch_groups ? (g_launch_groups / 2 + 255) / 256 * 256
                                          : ((0xffffffffull / 32) / 256) * 256;
  uint64_t g0 = 0;
  for (; n8_all - g0 > range8; g0 += range8) {
    const int rc = run_bf16_range(vr, d_x_bf16, nullptr, d_w, d_s, K, d_base_f32 + 8 * g0, nullptr,
                                  d_out_f32 + 8 * g0, nullptr, 8 * range8, 0, 8 * g0, stream);
    if (rc != PLATO_AGG_OK) return rc;
  }
  return run_bf16_range(vr, d_x_bf16, d_x_i64_bf16, d_w, d_s, K, n_f32 ? d_base_f32 + 8 * g0 : d_base_f32,
                        d_base_i64, n_f32 ? d_out_f32 + 8 * g0 : d_out_f32, d_out_i64f, n_f32 - 8 * g0, n_i64,
                        8 * g0, stream);
}

int run_bf16_range(const Bf16Variant& vr, const uint16_t* const* d_x_bf16, const uint16_t* const* d_x_i64_bf16,
                   const float* d_w, const float* d_s, int K, const float* d_base_f32, const int64_t* d_base_i64,
                   float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64, uint64_t x_off,
                   hipStream_t stream) {
  if (n_f32 + n_i64 == 0) return plato_agg_internal::clear_error();
  Bf16Args a{};
  a.x_off = x_off;
  a.xf = d_x_bf16;
  a.xi = d_x_i64_bf16;
  a.w = d_w;
  a.s = d_s;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.out_f = d_out_f32;
  a.out_if = d_out_i64f;
  a.n8 = n_f32 / 8;  // the vector bodies cover 8 * n8 elements (LANE 4: 2 * n8 groups of 4)
  a.n_f32 = n_f32;
  a.n_i64 = n_i64;
  a.K = K;
  const uint64_t groups = vr.lane == 8 ? a.n8 : 2 * a.n8;
  const uint64_t nb_vec = (groups + vr.block - 1) / vr.block;
  const uint64_t n_scalar = (n_f32 - 8 * a.n8) + n_i64;
  const uint64_t nb_scalar = (n_scalar + vr.block - 1) / vr.block;
  if (nb_vec + nb_scalar > 0x7fffffffull || a.n8 * 32ull > 0xffffffffull)
    return fail(PLATO_AGG_EINVAL, "launch range exceeds 4 GiB (internal split error)");
  a.nb_vec = uint32_t(nb_vec);
  a.nb_vec_full = uint32_t(groups / vr.block);
  a.nb_scalar = uint32_t(nb_scalar);
  vr.fn[d_s ? 1 : 0](a, dim3(uint32_t(nb_vec + nb_scalar)), stream);
  return check_launch("fedavg_bf16 kernel launch");
}
}  // namespace

int plato_agg_fedavg_weights_bf16(const uint16_t* const* d_x_bf16, const uint16_t* const* d_x_i64_bf16,
                                  const float* d_w, const float* d_s, int K, const float* d_base_f32,
                                  const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                                  size_t n_i64, hipStream_t stream) {
  return run_bf16(0, d_x_bf16, d_x_i64_bf16, d_w, d_s, K, d_base_f32, d_base_i64, d_out_f32, d_out_i64f, n_f32,
                  n_i64, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h: libplato_agg_tune.so only
int plato_agg_tune_num_bf16_variants(void) { return kNumBf16Variants; }

int plato_agg_tune_fedavg_bf16(int variant, const uint16_t* const* d_x_bf16, const uint16_t* const* d_x_i64_bf16,
                               const float* d_w, const float* d_s, int K, const float* d_base_f32,
                               const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                               size_t n_i64, hipStream_t stream) {
  return run_bf16(variant, d_x_bf16, d_x_i64_bf16, d_w, d_s, K, d_base_f32, d_base_i64, d_out_f32, d_out_i64f,
                  n_f32, n_i64, stream);
}

int plato_agg_tune_num_variants(void) { return kNumVariants; }

void plato_agg_tune_set_launch_groups(uint64_t groups) { g_launch_groups = groups; }

int plato_agg_tune_describe(int variant, int* block, int* v, int* u, int* flags) {
  if (variant < 0 || variant >= kNumVariants) return fail(PLATO_AGG_EINVAL, "bad variant");
  const Variant& vr = kVariants[variant];
  *block = vr.B;
  *v = vr.V;
  *u = vr.U;
  *flags = (vr.NTL ? 1 : 0) | (vr.NTS ? 2 : 0) | (vr.PIPE ? 4 : 0) | (vr.BUF ? 8 : 0) | (vr.PERSIST << 4) |
           (vr.XCD ? 1 << 12 : 0) | (vr.BAL ? 1 << 13 : 0);
  return PLATO_AGG_OK;
}

int plato_agg_tune_fedavg(int variant, int has_base, const float* const* d_x_f32, const int64_t* const* d_x_i64,
                          const float* d_w, const float* d_s, int K, const float* d_base_f32,
                          const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                          size_t n_i64, hipStream_t stream) {
  return run_agg(variant, has_base != 0, d_x_f32, d_x_i64, d_w, d_s, K, d_base_f32, d_base_i64, d_out_f32,
                 d_out_i64f, n_f32, n_i64, stream);
}

int plato_agg_tune_stream(int mode, const float* d_src, float* d_dst, size_t n, int blocks, hipStream_t stream) {
  if (!d_src || !d_dst || (n & 3)) return fail(PLATO_AGG_EINVAL, "stream probe: null pointer or n % 4 != 0");
  if (blocks <= 0) blocks = 2048;
  const uint64_t n4 = n / 4;
  if (mode == 0) {
    hipLaunchKernelGGL(stream_probe<0>, dim3(blocks), dim3(256), 0, stream, (const f4*)d_src, (f4*)d_dst, n4, 8u);
  } else {
    hipLaunchKernelGGL(stream_probe<1>, dim3(blocks), dim3(256), 0, stream, (const f4*)d_src, (f4*)d_dst, n4, 8u);
  }
  return check_launch("stream probe launch");
}
#endif  // PLATO_AGG_TUNE

int plato_agg_compute_deltas(const float* d_x_f32, const int64_t* d_x_i64, const float* d_base_f32,
                             const int64_t* d_base_i64, float* d_out_f32, int64_t* d_out_i64, size_t n_f32,
                             size_t n_i64, hipStream_t stream) {
  if (n_f32 && (!d_x_f32 || !d_base_f32 || !d_out_f32)) return fail(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_i64 && (!d_x_i64 || !d_base_i64 || !d_out_i64)) return fail(PLATO_AGG_EINVAL, "null int64 pointer");
  if (n_f32 && !(aligned16(d_x_f32) && aligned16(d_base_f32) && aligned16(d_out_f32)))
    return fail(PLATO_AGG_EINVAL, "fp32 pointers must be 16-byte aligned");
  if (n_f32 + n_i64 == 0) return PLATO_AGG_OK;
  hipLaunchKernelGGL(deltas_kernel, grid_for(n_f32 / 4 + n_i64 + 4), dim3(kBlock), 0, stream, d_x_f32, d_x_i64,
                     d_base_f32, d_base_i64, d_out_f32, d_out_i64, n_f32, n_i64);
  return check_launch("compute_deltas launch");
}

int plato_agg_update_weights(const float* d_base_f32, const int64_t* d_base_i64, const float* d_avg_f32,
                             const float* d_avg_i64f, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                             size_t n_i64, hipStream_t stream) {
  if (n_f32 && (!d_base_f32 || !d_avg_f32 || !d_out_f32)) return fail(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_i64 && (!d_base_i64 || !d_avg_i64f || !d_out_i64f)) return fail(PLATO_AGG_EINVAL, "null int64 pointer");
  if (n_f32 && !(aligned16(d_base_f32) && aligned16(d_avg_f32) && aligned16(d_out_f32)))
    return fail(PLATO_AGG_EINVAL, "fp32 pointers must be 16-byte aligned");
  if (n_f32 + n_i64 == 0) return PLATO_AGG_OK;
  hipLaunchKernelGGL(update_kernel, grid_for(n_f32 / 4 + n_i64 + 4), dim3(kBlock), 0, stream, d_base_f32,
                     d_base_i64, d_avg_f32, d_avg_i64f, d_out_f32, d_out_i64f, n_f32, n_i64);
  return check_launch("update_weights launch");
}

int plato_agg_cast_f32_i64(const float* d_src, int64_t* d_dst, size_t n, hipStream_t stream) {
  if (n == 0) return PLATO_AGG_OK;
  if (!d_src || !d_dst) return fail(PLATO_AGG_EINVAL, "null pointer");
  hipLaunchKernelGGL(cast_kernel, grid_for(n), dim3(kBlock), 0, stream, d_src, d_dst, (uint64_t)n);
  return check_launch("cast launch");
}

int plato_agg_mix_weights(const float* d_x_f32, const int64_t* d_x_i64, const float* d_base_f32,
                          const int64_t* d_base_i64, float one_minus_m, float m, float* d_out_f32,
                          float* d_out_i64f, size_t n_f32, size_t n_i64, hipStream_t stream) {
  if (n_f32 && (!d_x_f32 || !d_base_f32 || !d_out_f32)) return fail(PLATO_AGG_EINVAL, "null fp32 pointer");
  if (n_i64 && (!d_x_i64 || !d_base_i64 || !d_out_i64f)) return fail(PLATO_AGG_EINVAL, "null int64 pointer");
  if (n_f32 && !(aligned16(d_x_f32) && aligned16(d_base_f32) && aligned16(d_out_f32)))
    return fail(PLATO_AGG_EINVAL, "fp32 pointers must be 16-byte aligned");
  if (n_f32 + n_i64 == 0) return PLATO_AGG_OK;
  hipLaunchKernelGGL(mix_kernel, grid_for(n_f32 / 4 + n_i64 + 4), dim3(kBlock), 0, stream, d_x_f32, d_x_i64,
                     d_base_f32, d_base_i64, one_minus_m, m, d_out_f32, d_out_i64f, n_f32, n_i64);
  return check_launch("mix launch");
}

int plato_agg_fill_synth_f32_at(float* d_out, const float* d_add, size_t n, uint64_t seed, uint64_t stream_id,
                                uint64_t first, int scale_log2, hipStream_t stream) {
  if (n == 0) return PLATO_AGG_OK;
  if (!d_out) return fail(PLATO_AGG_EINVAL, "null output");
  if (scale_log2 < -126 || scale_log2 > 100) return fail(PLATO_AGG_EINVAL, "scale_log2 out of range");
  const float scale = ldexpf(1.0f, scale_log2);
  // element e of the slice is element first + e of the stream: h = splitmix64(key + first + e)
  hipLaunchKernelGGL(synth_f32_kernel, grid_for(n), dim3(kBlock), 0, stream, d_out, d_add, (uint64_t)n,
                     synth_key(seed, stream_id) + first, scale);
  return check_launch("synth_f32 launch");
}

int plato_agg_fill_synth_f32(float* d_out, const float* d_add, size_t n, uint64_t seed, uint64_t stream_id,
                             int scale_log2, hipStream_t stream) {
  return plato_agg_fill_synth_f32_at(d_out, d_add, n, seed, stream_id, 0, scale_log2, stream);
}

int plato_agg_fill_synth_i64_at(int64_t* d_out, const int64_t* d_add, size_t n, uint64_t seed, uint64_t stream_id,
                                uint64_t first, uint64_t modulus, hipStream_t stream) {
  if (n == 0) return PLATO_AGG_OK;
  if (!d_out) return fail(PLATO_AGG_EINVAL, "null output");
  if (modulus == 0) return fail(PLATO_AGG_EINVAL, "modulus must be >= 1");
  hipLaunchKernelGGL(synth_i64_kernel, grid_for(n), dim3(kBlock), 0, stream, d_out, d_add, (uint64_t)n,
                     synth_key(seed, stream_id) + first, modulus);
  return check_launch("synth_i64 launch");
}

int plato_agg_fill_synth_i64(int64_t* d_out, const int64_t* d_add, size_t n, uint64_t seed, uint64_t stream_id,
                             uint64_t modulus, hipStream_t stream) {
  return plato_agg_fill_synth_i64_at(d_out, d_add, n, seed, stream_id, 0, modulus, stream);
}

}  // extern "C"
