// fedadp.hip — FedAdp's float32 dots straight from the staged client arenas, for gfx950.
// C ABI: include/plato_agg.h (plato_agg_fedadp_dots).  CPU restatement: oracle/reductions.c (sdot).
//
// The reference (examples/server_aggregation/fedadp/fedadp_server.py:91-99, 122-133) flattens
// every client delta with process_grad — entries sorted by name.lower(), all but the first
// divided by -lr — and takes numpy's float32 np.inner(g, loc_k) and np.linalg.norm(loc_k)
// (sqrt of loc_k . loc_k), i.e. cblas_sdot of numpy's OpenBLAS: on AVX-512 hosts
// sdot_k_SKYLAKEX, 64 fma chains (chain j sums positions = j mod 64, serially over the
// 64-element blocks), a fold, one 32-element block, a fixed horizontal sum and a float64 tail.
//
// plato_agg_flatten + plato_agg_sdot_shared (flat.hip) materialise the K flattened deltas
// (5.7 GB for 128 ResNet-18 clients written and read again).  Here the flattening is folded
// into the dot kernel: producer waves gather positions from the staged arenas through the
// segment map, form loc = (x - b) or -(x - b) / lr in registers and write them transposed
// into an LDS tile; chain waves only run the fma chains out of LDS.
//
// Shape (the product default, kAdpDefault; one workgroup per CU for 128 clients):
//   * 1 pair (client) x 32 of the 64 chains per workgroup: a gather iteration reads whole
//     128-byte lines (16 bytes per lane, buffer_load_dwordx4) of the client arena, of b and of g;
//     the two chain groups of a pair run on one XCD, so x and b are served from its L2.
//   * chain wave: lane = kind * 32 + chain, kind 0 = g . loc, kind 1 = loc . loc: ONE dependent
//     fma per step per lane (the dots are split over lanes, not interleaved), 4 steps per
//     ds_read_b128 of a transposed row (row pitch kS + 16 floats, rows 4m .. 4m + 3 shifted by
//     4m floats: conflict-free ds_read_b128 and ds_write_b32).
//   * 8 producer waves, 2 gather iterations each per 128-block stage; their global loads run
//     kD = 2 stages ahead of the tile being written (kD register sets), the tile ring has two
//     slots, one s_barrier per stage.  A wave's current entry is cached in SGPRs: the segment
//     map in LDS is read only at entry boundaries.
//   * g . g: an extra chain wave in the workgroups of pair 0 (x . x over the same tile).
// The other shapes (8 / 4 / 2 pairs per workgroup, 4-byte gathers, deeper pipelines, chain waves
// isolated on a SIMD) and the timing probes are tuning variants (PLATO_AGG_TUNE); DESIGN.md §13.
// Compiled with -ffp-contract=off; the chain fma is an explicit v_fma_f32.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <type_traits>

#include "common.h"
#include "plato_agg.h"

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;

namespace {

int check_launch(const char* what) {
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string(what) + ": " + hipGetErrorString(err));
  return clear_error();
}

template <class T>
__device__ __forceinline__ T sld(const T* p, int i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

__device__ __forceinline__ float chain_fma(float a, float b, float c) {
  asm("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  return c;
}

typedef __attribute__((address_space(1))) const float gfloat;
typedef float f4v __attribute__((ext_vector_type(4)));

// Segment map entry in LDS: positions [flat, end) read element src + (p - flat) of the region.
struct AdpSeg {
  uint32_t flat;
  uint32_t end;
  uint32_t src;
  uint32_t info;  // bit 0: int64 region, bit 1: NEG_DIV
};
constexpr uint32_t kSegI64 = 1u, kSegNeg = 2u;
constexpr int kMaxSegs = 2048;

struct AdpArgs {
  const float* x;                // flattened global gradient (process_grad(g)), >= nsteps * 64 floats
  const float* const* xf;        // client fp32 arenas
  const int64_t* const* xi;      // client int64 arenas
  const float* base_f;
  const int64_t* base_i;
  const plato_agg_segment* segs;
  uint32_t n_segs;
  uint64_t n;                    // flat length
  uint64_t nsteps;               // whole 64-element blocks before sdot's 32-block and tail
  float lr;
  float* ws;                     // [n_pairs + with_xx][128]: chain sums of x.y, then of y.y
  float* y64;                    // [n_pairs][n_i64]: process_grad's value of every int64 element
  uint64_t n_i64;
  uint64_t n_f32;                // fp32 arena length (buffer bounds)
  int n_pairs;
  int with_xx;
};

// process_grad's value at one position, from the client's staged arena (flat.hip flat_value, DELTA)
__device__ __forceinline__ float adp_f32(float x, float b, bool neg, float lr) {
  float v = x - b;
  if (neg) v = (-v) / lr;
  return v;
}
__device__ __forceinline__ float adp_i64(int64_t x, int64_t b, bool neg, float lr) {
  // int64 delta, exact (wrapping) in int64; -delta too, then the cast and the division
  const uint64_t d = uint64_t(x) - uint64_t(b);
  return neg ? float(int64_t(uint64_t(0) - d)) / lr : float(int64_t(d));
}

// The last segment with flat <= p, walking forward from `from` (segments are in flat order).
__device__ __forceinline__ int seg_walk(const AdpSeg* S, int n_segs, uint32_t p, int from) {
  int s = from;
  while (s + 1 < n_segs && S[s + 1].flat <= p) ++s;
  return s;
}

// kP pairs x kC chains per workgroup (kP * kC = 32: one chain wave of 2 kinds); kS steps per
// stage; kW producer waves, kIt gather iterations of 64 positions each per stage; kVRpad floats
// between vectors (chosen with the row pitch kS + 4 so that the chain wave's ds_read_b128 pairs
// are conflict-free for the lane map kind * 32 + chain * kP + pair: DESIGN.md §12)
template <int kP, int kC, int kS, int kW, int kIt, int kVRpad = 0, int kV = 1, int kSw = 0>
struct AdpShape {
  static_assert(kP * kC == 32, "one chain wave: kind * 32 + chain * kP + pair");
  static_assert(kV == 1 || kV == 4, "one or four consecutive positions per lane and gather iteration");
  static_assert(kC % kV == 0, "a lane's positions lie in one 64-block");
  static_assert(kS * kC == 64 * kV * kW * kIt, "a stage is kW x kIt gather iterations of 64 * kV positions");
  static_assert(kS % 16 == 0, "the chain wave reads 16 steps per block");
  // transposed row pitch (floats).  kSw = 2 (kC = 32, 4-position producer lanes): pitch kS + 16
  // and rows 4m .. 4m + 3 shifted by 4m floats.  A ds_write_b32 half-wave (banks (a/4) mod 32) of
  // the producers then writes rows 4m + j, m = 0..7, on 8 different 4-bank slots (4-way conflicted
  // with pitch kS + 4: 268 M extra LDS cycles per launch, all of them these writes), and every
  // 16-lane group of the chain's ds_read_b128 (banks mod 64) still covers 16 different slots.
  static constexpr int kR = kSw == 2 ? kS + 16 : kS + 4;
  static_assert(kSw != 2 || (kC == 32 && kS % 64 == 0), "swizzled rows: one chain wave of 32 chains");
  // kSw = 1 (measured no better): the upper half of a vector's rows sits 32 floats further on
  static constexpr int kGap = kSw == 1 ? 32 : kSw == 2 ? 4 * (kC / 4) : 0;
  static constexpr int kVR = kC * kR + kVRpad + kGap;  // rows of one vector (x, loc_0 .. loc_{kP-1})
  __device__ static constexpr int row(int r) {
    return r * kR + (kSw == 2 ? 4 * (r >> 2) : (r >= kC / 2 ? kGap : 0));
  }
  static constexpr int kSlot = (1 + kP) * kVR;
  static constexpr int kBlkPerIt = 64 * kV / kC;  // 64-blocks per gather iteration
  static constexpr int kLpB = kC / kV;             // lanes per 64-block in a gather iteration
};

// One producer wave's loads for one stage: x, b and the kP arenas at kIt positions per lane.
template <int kP, int kIt>
struct AdpRegs {
  float x[kIt];
  float b[kIt];
  float y[kIt][kP];
  uint32_t code[kIt];  // per lane: kSegNeg; kSegI64 (+ element << 8): an int64 position, fetched at write time
  uint32_t fast;       // bit i: iteration i lies in one fp32 entry (wave-uniform)
};

// Buffer resources of a producer wave: raw buffer loads take a 32-bit byte offset per lane against
// a descriptor in SGPRs, so a gathered load costs no 64-bit address arithmetic (and an offset past
// num_records reads 0 instead of faulting).
template <int kP>
struct AdpSrc {
  __amdgpu_buffer_rsrc_t x, b, y[kP];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t adp_rsrc(const void* base, uint64_t bytes) {
  const uint64_t n = bytes < 0xffffffffull ? bytes : 0xffffffffull;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)uint32_t(n), 0x00020000);
}

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// A producer wave's current segment, wave-uniform (SGPRs): the positions a wave gathers only move
// forward, so the segment map in LDS is read only when an iteration crosses into the next entry
struct AdpCursor {
  int idx;
  uint32_t flat, end, src, info;
};

__device__ __forceinline__ void adp_cursor_load(const AdpSeg* S, int idx, AdpCursor& c) {
  c.idx = idx;
  c.flat = __builtin_amdgcn_readfirstlane(S[idx].flat);
  c.end = __builtin_amdgcn_readfirstlane(S[idx].end);
  c.src = __builtin_amdgcn_readfirstlane(S[idx].src);
  c.info = __builtin_amdgcn_readfirstlane(S[idx].info);
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe>
__device__ __forceinline__ void adp_issue(const AdpArgs& a, const AdpSeg* S, int n_segs, AdpCursor& cur,
                                          const AdpSrc<kP>& src, uint32_t t, int cg, int w, int lane,
                                          AdpRegs<kP, kIt>& r) {
  using Sh = AdpShape<kP, kC, kS, kW, kIt, kVRpad>;
  const uint32_t last = uint32_t(a.nsteps - 1);
  r.fast = 0;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int g = i * kW + w;
    const uint32_t s0 = t * kS + uint32_t(g * Sh::kBlkPerIt);  // nsteps < 2^26: 32-bit block indices
    const uint32_t s = min(s0 + uint32_t(lane / kC), last);     // a ragged last stage re-reads a valid block
    const uint32_t p = s * 64 + uint32_t(cg * kC + lane % kC);
    const uint32_t pf = min(s0, last) * 64 + uint32_t(cg * kC);
    const uint32_t pl = min(s0 + uint32_t(Sh::kBlkPerIt - 1), last) * 64 + uint32_t(cg * kC + kC - 1);
    while (pf >= cur.end && cur.idx + 1 < n_segs) adp_cursor_load(S, cur.idx + 1, cur);  // rare: next entry
    uint32_t e, code;
    // the loads below are the same on both paths (no branch around them): every trip issues
    // kIt * (kP + 2) loads and the compiler's vmcnt bookkeeping covers exactly one stage
    if (!(cur.info & kSegI64) && pl < cur.end) {
      r.fast |= 1u << i;  // the whole iteration inside one fp32 entry: one shift for every lane
      e = p - cur.flat + cur.src;
      code = cur.info;
    } else {  // an entry boundary inside the iteration: per-lane entries
      const AdpSeg ls = S[seg_walk(S, n_segs, p, cur.idx)];
      const uint32_t el = p - ls.flat + ls.src;
      const bool i64 = ls.info & kSegI64;
      e = i64 ? 0u : el;
      code = i64 ? (ls.info | (el << 8)) : ls.info;
    }
    r.code[i] = code;
    if (kProbe == 3) {  // timing probe: no loads (wrong results)
      r.x[i] = float(p);
      r.b[i] = float(e);
#pragma unroll
      for (int k = 0; k < kP; ++k) r.y[i][k] = float(e + k);
      continue;
    }
    r.x[i] = bload(src.x, p * 4u);
    r.b[i] = bload(src.b, e * 4u);
#pragma unroll
    for (int k = 0; k < kP; ++k) r.y[i][k] = bload(src.y[k], e * 4u);
  }
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe>
__device__ __forceinline__ void adp_write(const AdpArgs& a, float* slot, int pair0, int w, int lane,
                                          AdpRegs<kP, kIt>& r) {
  using Sh = AdpShape<kP, kC, kS, kW, kIt, kVRpad>;
  const float lr = a.lr;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int g = i * kW + w;
    const int col = g * Sh::kBlkPerIt + lane / kC;  // step within the stage
    float* dst = slot + (lane % kC) * Sh::kR + col;
    dst[0] = r.x[i];
    const uint32_t code = r.code[i];
    if (r.fast & (1u << i)) {  // wave-uniform: one entry, one sign/divide mode
      if (kProbe != 1 && (__builtin_amdgcn_readfirstlane(int(code)) & kSegNeg)) {  // probe 1: no division
#pragma unroll
        for (int k = 0; k < kP; ++k) dst[(1 + k) * Sh::kVR] = (-(r.y[i][k] - r.b[i])) / lr;
      } else {
#pragma unroll
        for (int k = 0; k < kP; ++k) dst[(1 + k) * Sh::kVR] = r.y[i][k] - r.b[i];
      }
    } else {
      const bool neg = code & kSegNeg;
      if (code & kSegI64) {
        // rare (one per int64 entry and chain group): the finished value from fedadp_i64_kernel's table
#pragma unroll
        for (int k = 0; k < kP; ++k) {
          const int pair = pair0 + k < a.n_pairs ? pair0 + k : a.n_pairs - 1;
          r.y[i][k] = a.y64[uint64_t(pair) * a.n_i64 + (code >> 8)];
        }
      }
#pragma unroll
      for (int k = 0; k < kP; ++k)
        dst[(1 + k) * Sh::kVR] = (code & kSegI64) ? r.y[i][k] : adp_f32(r.y[i][k], r.b[i], neg, lr);
    }
  }
}

// Four consecutive positions per lane (kV = 4): a lane's x, b and loc_k come from one 16-byte
// buffer load each (an arena position is 4-byte aligned only: dword-aligned dwordx4 loads are
// legal, MI355X_MICROARCH.md), so a gather iteration of 256 positions costs kP + 2 load
// instructions instead of 4 x (kP + 2).  An iteration that crosses an entry keeps the loads
// (their values are unused) and its lanes fetch their four positions one by one at write time.
template <int kP, int kIt>
struct AdpRegs4 {
  f4v x[kIt];
  f4v b[kIt];
  f4v y[kIt][kP];
  uint32_t code[kIt];  // fast iterations: the entry's info; otherwise the segment index of pos[i]
  uint32_t pos[kIt];   // first position of the lane
  uint32_t fast;       // bit i: iteration i lies in one fp32 entry (wave-uniform)
};

// kAux: the load's cache policy (2 = nt: a streaming read, kept out of the way of the re-read x and b)
template <int kAux = 0>
__device__ __forceinline__ f4v bload4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAux));
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kNt = 0>
__device__ __forceinline__ void adp_issue4(const AdpArgs& a, const AdpSeg* S, int n_segs, AdpCursor& cur,
                                           const AdpSrc<kP>& src, uint32_t t, int cg, int w, int lane,
                                           AdpRegs4<kP, kIt>& r) {
  using Sh = AdpShape<kP, kC, kS, kW, kIt, kVRpad, 4>;
  const uint32_t last = uint32_t(a.nsteps - 1);
  r.fast = 0;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int g = i * kW + w;
    const uint32_t s0 = t * kS + uint32_t(g * Sh::kBlkPerIt);
    const uint32_t s = min(s0 + uint32_t(lane / Sh::kLpB), last);
    const uint32_t p = s * 64 + uint32_t(cg * kC + (lane % Sh::kLpB) * 4);
    const uint32_t pf = min(s0, last) * 64 + uint32_t(cg * kC);
    const uint32_t pl = min(s0 + uint32_t(Sh::kBlkPerIt - 1), last) * 64 + uint32_t(cg * kC + kC - 1);
    while (pf >= cur.end && cur.idx + 1 < n_segs) adp_cursor_load(S, cur.idx + 1, cur);  // rare: next entry
    uint32_t e, code;
    if (!(cur.info & kSegI64) && pl < cur.end) {
      r.fast |= 1u << i;
      e = p - cur.flat + cur.src;
      code = cur.info;
    } else {
      const int idx = seg_walk(S, n_segs, p, cur.idx);
      e = 0u;  // the loads still go out (same count on every path); the write fetches the values
      code = uint32_t(idx);
    }
    r.code[i] = code;
    r.pos[i] = p;
    // kNt & 3: 1 = the client arenas (read once) as nt loads, 2 = every load nt
    r.x[i] = bload4<(kNt & 3) == 2 ? 2 : 0>(src.x, p * 4u);
    r.b[i] = bload4<(kNt & 3) == 2 ? 2 : 0>(src.b, e * 4u);
#pragma unroll
    for (int k = 0; k < kP; ++k) r.y[i][k] = bload4<(kNt & 3) ? 2 : 0>(src.y[k], e * 4u);
  }
}

// process_grad's value at flat position p of pair `pair`, walking the segment map from `idx`
// (the slow path of an iteration that crosses an entry)
__device__ __forceinline__ float adp_value_at(const AdpArgs& a, const AdpSeg* S, int n_segs, int& idx, uint32_t p,
                                              int pair) {
  idx = seg_walk(S, n_segs, p, idx);
  const AdpSeg sg = S[idx];
  const uint32_t el = p - sg.flat + sg.src;
  if (sg.info & kSegI64) return a.y64[uint64_t(pair) * a.n_i64 + el];
  return adp_f32(a.xf[pair][el], a.base_f[el], sg.info & kSegNeg, a.lr);
}

// (-d) / lr, correctly rounded, as RN32(RN64(-d * RN64(1 / lr))) (kNt & 4): the float64 product is
// within 2^-52 (relative) of the quotient, while a quotient of two floats that is not a float lies
// at least 2^-49 (relative) from every midpoint of the float grid (and is never on one), so the one
// rounding to float gives the float32 division's bits — 3 instructions instead of the division's ~10
__device__ __forceinline__ float adp_div_lr_f64(float v, double inv_lr) { return float(double(v) * inv_lr); }

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kSw, int kNt = 0>
__device__ __forceinline__ void adp_write4(const AdpArgs& a, const AdpSeg* S, int n_segs, float* slot, int pair0,
                                           int w, int lane, AdpRegs4<kP, kIt>& r) {
  using Sh = AdpShape<kP, kC, kS, kW, kIt, kVRpad, 4, kSw>;
  const float lr = a.lr;
  const double inv_lr = (kNt & 4) ? 1.0 / double(lr) : 0.0;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int g = i * kW + w;
    const int col = g * Sh::kBlkPerIt + lane / Sh::kLpB;  // step within the stage
    float* dst = slot + Sh::row((lane % Sh::kLpB) * 4) + col;  // chain c0 = 4 * (lane % kLpB), rows c0 .. c0 + 3
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j * Sh::kR] = r.x[i][j];
    if (r.fast & (1u << i)) {  // wave-uniform: one entry, one sign/divide mode
      if (__builtin_amdgcn_readfirstlane(int(r.code[i])) & kSegNeg) {
#pragma unroll
        for (int k = 0; k < kP; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float nv = -(r.y[i][k][j] - r.b[i][j]);
            dst[(1 + k) * Sh::kVR + j * Sh::kR] = (kNt & 4) ? adp_div_lr_f64(nv, inv_lr) : nv / lr;
          }
      } else {
#pragma unroll
        for (int k = 0; k < kP; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[(1 + k) * Sh::kVR + j * Sh::kR] = r.y[i][k][j] - r.b[i][j];
      }
    } else {  // rare: an entry boundary (or an int64 entry) inside the iteration
      for (int k = 0; k < kP; ++k) {
        const int pair = pair0 + k < a.n_pairs ? pair0 + k : a.n_pairs - 1;
        int idx = int(r.code[i]);
        for (int j = 0; j < 4; ++j) dst[(1 + k) * Sh::kVR + j * Sh::kR] = adp_value_at(a, S, n_segs, idx, r.pos[i] + j, pair);
      }
    }
  }
}

// Waves per workgroup: kW producers + 2 chain waves, or with kIso 12 waves placed so that the chain
// waves share a SIMD with no producer (waves are dealt to the CU's 4 SIMDs round-robin, so waves 0, 4
// and 8 share one: wave 0 runs the pairs' chains, wave 4 g . g, wave 8 idles; producers are the other 9
// waves, the last of them idle when kW = 8).  A producer's VALU instruction (the division sequence, the
// 64-bit address arithmetic) holds its SIMD for several cycles, and on a shared SIMD the serial fma
// chain waits for it at every step (timing probes).
template <int kW, int kIso>
constexpr int adp_waves() { return kIso ? 12 : kW + 2; }

template <int kP, int kIt, int kV>
using AdpRegsV = std::conditional_t<kV == 4, AdpRegs4<kP, kIt>, AdpRegs<kP, kIt>>;

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe, int kV, int kNt = 0>
__device__ __forceinline__ void adp_issue_v(const AdpArgs& a, const AdpSeg* S, int n_segs, AdpCursor& cur,
                                            const AdpSrc<kP>& src, uint32_t t, int cg, int w, int lane,
                                            AdpRegsV<kP, kIt, kV>& r) {
  if constexpr (kV == 4) adp_issue4<kP, kC, kS, kW, kIt, kVRpad, kNt>(a, S, n_segs, cur, src, t, cg, w, lane, r);
  else adp_issue<kP, kC, kS, kW, kIt, kVRpad, kProbe>(a, S, n_segs, cur, src, t, cg, w, lane, r);
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe, int kV, int kSw, int kNt = 0>
__device__ __forceinline__ void adp_write_v(const AdpArgs& a, const AdpSeg* S, int n_segs, float* slot, int pair0,
                                            int w, int lane, AdpRegsV<kP, kIt, kV>& r) {
  static_assert(!kSw || kV == 4, "the row gap is laid out for 4-position producer lanes");
  if constexpr (kV == 4) adp_write4<kP, kC, kS, kW, kIt, kVRpad, kSw, kNt>(a, S, n_segs, slot, pair0, w, lane, r);
  else adp_write<kP, kC, kS, kW, kIt, kVRpad, kProbe>(a, slot, pair0, w, lane, r);
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe = 0, int kIso = 0, int kV = 1, int kD = 2,
          int kCP = 1, int kPrio = 3, int kSw = 0, int kNt = 0>
__global__ __launch_bounds__((64 * adp_waves<kW, kIso>())) void fedadp_dots_kernel(AdpArgs a) {
  using Sh = AdpShape<kP, kC, kS, kW, kIt, kVRpad, kV, kSw>;
  static_assert(!kIso || kW <= 9, "kIso: at most 9 producer waves");
  __shared__ __attribute__((aligned(16))) float ring[2 * Sh::kSlot];
  __shared__ AdpSeg S[kMaxSegs];
  constexpr int kGroups = 64 / kC;
  // workgroups are dealt to the 8 XCDs round-robin: the kGroups chain groups of a pair group
  // get ids that agree mod 8, so they share one XCD and its L2
  const int b = int(blockIdx.x), lo = b & 7;
  const int cg = (b / 8) % kGroups;
  const int pg = (b / (8 * kGroups)) * 8 + lo;
  if (pg * kP >= a.n_pairs) return;  // padding workgroup (before any barrier)
  const int n_segs = int(a.n_segs);
  for (int j = int(threadIdx.x); j < n_segs; j += int(blockDim.x)) {
    const plato_agg_segment sg = a.segs[j];
    S[j] = AdpSeg{uint32_t(sg.flat_offset), uint32_t(sg.flat_offset + sg.numel), uint32_t(sg.src_offset),
                  (sg.region ? kSegI64 : 0u) | ((sg.flags & PLATO_AGG_SEG_NEG_DIV) ? kSegNeg : 0u)};
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = int(threadIdx.x & 63);
  const uint64_t nsteps = a.nsteps;
  const uint64_t nst = (nsteps + kS - 1) / kS;
  static_assert(kD >= 2 && kD <= 4, "2-4 stages of loads in flight per producer wave");
  const uint64_t nst2 = (nst + kD - 1) / kD * kD;  // barriers: one per stage, in whole trips of kD stages
  // role: chain wave 0 (pairs) / 1 (g . g), or producer w; idle waves end here (a wave that has ended
  // is no longer counted by s_barrier)
  int chain_role = -1, w = -1;
  if (kIso) {
    if ((wave & 3) == 0) chain_role = wave >> 2;
    else w = (wave >> 2) * 3 + (wave & 3) - 1;
    if (chain_role > 1 || w >= kW) return;
  } else {
    if (wave >= 2) w = wave - 2;
    else chain_role = wave;
  }
  if (w >= 0) {  // producer
    if (kProbe == 4) {  // timing probe: the chains alone (producers only keep the barrier count)
      for (uint64_t t = 0; t < nst2; ++t) __builtin_amdgcn_s_barrier();
      return;
    }
    const int pair0 = pg * kP;
    AdpSrc<kP> src;
    src.x = adp_rsrc(a.x, a.nsteps * 256);
    src.b = adp_rsrc(a.base_f, a.n_f32 * 4);
#pragma unroll
    for (int k = 0; k < kP; ++k)
      src.y[k] = adp_rsrc(sld(a.xf, pair0 + k < a.n_pairs ? pair0 + k : a.n_pairs - 1), a.n_f32 * 4);
    AdpCursor cursor;
    adp_cursor_load(S, 0, cursor);
    // kD register sets: the loads of stage t + kD go out right after stage t is written, so every
    // producer wave keeps kD stages of loads in flight; the tile ring in LDS has two slots
    AdpRegsV<kP, kIt, kV> regs[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j)
      adp_issue_v<kP, kC, kS, kW, kIt, kVRpad, kProbe, kV, kNt>(a, S, n_segs, cursor, src, uint32_t(j), cg, w, lane, regs[j]);
    uint64_t t_start = 0, t_wait = 0, t_write = 0, c0 = 0;  // probe 6: cycle counts
    if (kProbe == 6) t_start = __builtin_readcyclecounter();
    // whole trips of kD stages (the last trip may run idle stages): no branch inside the loop, so the
    // compiler's vmcnt bookkeeping sees the same kD stages in flight on every trip
    for (uint32_t t = 0; t < uint32_t(nst2); t += kD) {
#pragma unroll
      for (int j = 0; j < kD; ++j) {
        if (kProbe == 6) c0 = __builtin_readcyclecounter();
        adp_write_v<kP, kC, kS, kW, kIt, kVRpad, kProbe, kV, kSw, kNt>(a, S, n_segs, ring + ((t + j) & 1) * Sh::kSlot, pair0, w,
                                                             lane, regs[j]);
        if (kProbe == 6) t_write += __builtin_readcyclecounter() - c0;
        // past the last stage (t = nst) every position clamps to the last block: valid addresses,
        // never consumed, and every trip issues the same loads
        const uint32_t nxt = t + j + kD;
        adp_issue_v<kP, kC, kS, kW, kIt, kVRpad, kProbe, kV, kNt>(a, S, n_segs, cursor, src, nxt < nst ? nxt : uint32_t(nst),
                                                             cg, w, lane, regs[j]);
        if (kProbe == 6) c0 = __builtin_readcyclecounter();
        __builtin_amdgcn_s_barrier();  // stage t + j published in slot (t + j) & 1
        if (kProbe == 6) t_wait += __builtin_readcyclecounter() - c0;
      }
    }
    if (kProbe == 6 && lane == 0) {  // probe 6: [total, barrier wait, write, HW_ID] of every producer
      uint32_t* o = reinterpret_cast<uint32_t*>(a.ws) + blockIdx.x * 48 + 8 + 4 * w;
      o[0] = uint32_t(__builtin_readcyclecounter() - t_start);
      o[1] = uint32_t(t_wait);
      o[2] = uint32_t(t_write);
      o[3] = uint32_t(__builtin_amdgcn_s_getreg((31 << 11) | 4));  // hwreg(HW_REG_HW_ID): wave, SIMD, CU ...
    }
    return;
  }
  // chain waves: wave 0 the kP pairs' dots, wave 1 g . g (pair group 0 only; elsewhere it only
  // keeps the barrier count)
  if (kPrio) __builtin_amdgcn_s_setprio(kPrio);  // the chain wave issues first
  const bool xx = chain_role == 1;
  const bool active = !xx || (pg == 0 && a.with_xx);
  const int kind = xx ? 0 : lane >> 5, c = xx ? lane % kC : (lane & 31) / kP, p = lane % kP;
  const int arow = (xx || kind == 0 ? 0 : (1 + p) * Sh::kVR) + Sh::row(c);
  const int brow = (xx ? 0 : (1 + p) * Sh::kVR) + Sh::row(c);
  float acc = 0.f;
  uint64_t t_start = 0, t_wait = 0, c0 = 0;  // probe 6: cycle counts
  if (kProbe == 6) t_start = __builtin_readcyclecounter();
  for (uint64_t t = 0; t < nst2; ++t) {
    if (kProbe == 6) c0 = __builtin_readcyclecounter();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (kProbe == 6) t_wait += __builtin_readcyclecounter() - c0;
    if (!active || t >= nst || kProbe == 2) continue;  // probe 2: no chains
    const float* slot = ring + (t & 1) * Sh::kSlot;
    const float* A = slot + arow;
    const float* B = slot + brow;
    if (kProbe == 7) {  // probe 7: the producers alone — one LDS read per stage keeps their stores live
      acc += A[t & 15] * B[t & 15];
      continue;
    }
    const uint64_t left = nsteps - t * kS;
    typedef float f4 __attribute__((ext_vector_type(4)));
    if (left >= uint64_t(kS)) {
      // 16 steps per block of 4 ds_read_b128 pairs; the reads of the next kCP blocks in flight
      constexpr int kNB = kS / 16, kRS = kCP + 1;
      f4 av[kRS][4], bv[kRS][4];
#pragma unroll
      for (int d = 0; d < kCP; ++d) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          av[d][q] = *reinterpret_cast<const f4*>(A + 16 * d + 4 * q);
          bv[d][q] = *reinterpret_cast<const f4*>(B + 16 * d + 4 * q);
        }
      }
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        const int nb = blk + kCP;
        if (kProbe != 5 && nb < kNB) {  // probe 5: no LDS reads after the first blocks
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            av[nb % kRS][q] = *reinterpret_cast<const f4*>(A + 16 * nb + 4 * q);
            bv[nb % kRS][q] = *reinterpret_cast<const f4*>(B + 16 * nb + 4 * q);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        const int cb = kProbe == 5 ? 0 : blk % kRS;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc = chain_fma(av[cb][q].x, bv[cb][q].x, acc);
          acc = chain_fma(av[cb][q].y, bv[cb][q].y, acc);
          acc = chain_fma(av[cb][q].z, bv[cb][q].z, acc);
          acc = chain_fma(av[cb][q].w, bv[cb][q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      for (int s = 0; s < int(left); ++s) acc = chain_fma(A[s], B[s], acc);
    }
  }
  const int chain = cg * kC + c;
  if (kProbe == 6) {  // probe 6: [total, barrier wait, HW_ID] of the pairs' chain wave, HW_ID of g . g (no results)
    uint32_t* o = reinterpret_cast<uint32_t*>(a.ws) + blockIdx.x * 48;
    if (!xx && lane == 0) {
      o[0] = uint32_t(__builtin_readcyclecounter() - t_start);
      o[1] = uint32_t(t_wait);
      o[2] = uint32_t(__builtin_amdgcn_s_getreg((31 << 11) | 4));
    }
    if (xx && lane == 0) o[3] = uint32_t(__builtin_amdgcn_s_getreg((31 << 11) | 4));
    if (acc == 12345.f) a.ws[blockIdx.x] = acc;  // keep the chains
    return;
  }
  if (!xx) {
    const int pair = pg * kP + p;
    if (pair < a.n_pairs) a.ws[uint64_t(pair) * 128 + uint64_t(kind) * 64 + chain] = acc;
  } else if (active && lane < kC) {  // the virtual pair (g, g): its x.y and y.y chains are both g.g
    a.ws[uint64_t(a.n_pairs) * 128 + chain] = acc;
    a.ws[uint64_t(a.n_pairs) * 128 + 64 + chain] = acc;
  }
}

// process_grad's value of every int64 element (num_batches_tracked deltas), per pair: the gather
// reads these finished values instead of doing int64 arithmetic in the stream
__global__ __launch_bounds__(64) void fedadp_i64_kernel(AdpArgs a) {
  const int pair = blockIdx.x;
  const int64_t* xi = a.xi[pair];
  for (uint32_t j = 0; j < a.n_segs; ++j) {
    const plato_agg_segment sg = a.segs[j];
    if (!sg.region) continue;
    const bool neg = sg.flags & PLATO_AGG_SEG_NEG_DIV;
    for (uint64_t q = threadIdx.x; q < sg.numel; q += 64) {
      const uint64_t e = sg.src_offset + q;
      a.y64[uint64_t(pair) * a.n_i64 + e] = adp_i64(xi[e], a.base_i[e], neg, a.lr);
    }
  }
}

// process_grad's value at any position (binary search of the segment map; the epilogue's few positions)
__device__ float adp_y_at(const AdpArgs& a, int pair, uint64_t p) {
  uint32_t lo = 0, hi = a.n_segs;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.segs[mid].flat_offset <= p) lo = mid; else hi = mid;
  }
  const plato_agg_segment sg = a.segs[lo];
  const uint64_t e = sg.src_offset + (p - sg.flat_offset);
  const bool neg = sg.flags & PLATO_AGG_SEG_NEG_DIV;
  if (sg.region) return adp_i64(a.xi[pair][e], a.base_i[e], neg, a.lr);
  return adp_f32(a.xf[pair][e], a.base_f[e], neg, a.lr);
}

// The rest of sdot_k_SKYLAKEX per pair from the 64 chain sums (flat.hip sdot_finish_kernel), with
// the 32-element block and the float64 tail gathered from the arenas.
__global__ __launch_bounds__(64) void fedadp_finish_kernel(AdpArgs a, float* out_xy, float* out_yy) {
  const int pair = blockIdx.x, lane = threadIdx.x & 63;
  const bool virt = pair >= a.n_pairs;  // (g, g)
  const uint64_t n = a.n;
  const uint64_t n1 = n & ~uint64_t(31);
  const uint64_t n64 = n1 & ~uint64_t(63);
  auto yv_at = [&](uint64_t p) { return virt ? a.x[p] : adp_y_at(a, pair, p); };
  const float axy = a.ws[uint64_t(pair) * 128 + lane];
  const float ayy = a.ws[uint64_t(pair) * 128 + 64 + lane];
  const float hxy = __shfl(axy, (lane + 8) & 63, 64);
  const float hyy = __shfl(ayy, (lane + 8) & 63, 64);
  const int r = lane >> 4, l = lane & 15;
  float bxy = 0.f, byy = 0.f;
  if (l < 8) {
    bxy = axy + hxy;
    byy = ayy + hyy;
    if (n1 > n64) {
      const float xv = a.x[n64 + 8 * r + l];
      const float yv = yv_at(n64 + 8 * r + l);
      bxy = __builtin_fmaf(xv, yv, bxy);
      byy = __builtin_fmaf(yv, yv, byy);
    }
  }
  const float xy1 = __shfl(bxy, 16 + l, 64), xy2 = __shfl(bxy, 32 + l, 64), xy3 = __shfl(bxy, 48 + l, 64);
  const float yy1 = __shfl(byy, 16 + l, 64), yy2 = __shfl(byy, 32 + l, 64), yy3 = __shfl(byy, 48 + l, 64);
  const float sxy = ((bxy + xy1) + xy2) + xy3;
  const float syy = ((byy + yy1) + yy2) + yy3;
  const float sxy4 = __shfl(sxy, (lane + 4) & 63, 64);
  const float syy4 = __shfl(syy, (lane + 4) & 63, 64);
  const float hx = sxy + sxy4, hy = syy + syy4;
  const float hx1 = __shfl(hx, 1, 64), hx2 = __shfl(hx, 2, 64), hx3 = __shfl(hx, 3, 64);
  const float hy1 = __shfl(hy, 1, 64), hy2 = __shfl(hy, 2, 64), hy3 = __shfl(hy, 3, 64);
  // the < 32 tail positions: gathered by one lane each, then summed by lane 0 in order
  __shared__ float txy_s[32], tyy_s[32];
  if (uint64_t(lane) < n - n1) {
    const float xv = a.x[n1 + lane], yv = yv_at(n1 + lane);
    txy_s[lane] = yv * xv;
    tyy_s[lane] = yv * yv;
  }
  __syncthreads();
  if (lane != 0) return;
  double kxy = 0.0, kyy = 0.0;
  if (n1) {
    kxy = double((hx + hx1) + (hx2 + hx3));
    kyy = double((hy + hy1) + (hy2 + hy3));
  }
  double txy = 0.0, tyy = 0.0;  // the scalar tail in float64, products rounded to fp32 first
  for (int i = 0; i < int(n - n1); ++i) {
    txy += double(txy_s[i]);
    tyy += double(tyy_s[i]);
  }
  out_xy[pair] = float(txy + kxy);
  out_yy[pair] = float(tyy + kyy);
}

// Flag-synchronised form (tuning; one pair per workgroup, 4-position lanes): no s_barrier between
// producers and chains.  Each producer wave adds 1 to full[slot] (an LDS counter) after writing its
// part of a stage, the chain waves wait for kW arrivals, run the stage and add 1 to `done`; a
// producer waits for the chains to have finished stage t - kRing before overwriting its slot.  So a
// slow stage on one side no longer stalls the other at every tile (the barrier form pays the max of
// both per tile).  Every wait is bounded: a wave that spins past kSpinMax raises `abort` in LDS and
// every wait then returns at once, so the grid always drains (results of such a launch are garbage
// and flagged in ws[0] as NaN by the finish kernel's inputs).
constexpr uint32_t kSpinMax = 1u << 20;

__device__ __forceinline__ bool adp_wait_geq(const uint32_t* ctr, uint32_t target, uint32_t* abort_flag) {
  for (uint32_t spin = 0;; ++spin) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (spin > kSpinMax) {
      __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int kC, int kS, int kW, int kIt, int kD, int kRing>
__global__ __launch_bounds__(64 * (kW + 2)) void fedadp_dots_flag_kernel(AdpArgs a) {
  using Sh = AdpShape<1, kC, kS, kW, kIt, 0, 4>;
  static_assert(kRing >= 2 && kRing <= 3, "2-3 tile slots");
  __shared__ __attribute__((aligned(16))) float ring[kRing * Sh::kSlot];
  __shared__ AdpSeg S[kMaxSegs];
  __shared__ uint32_t full[kRing], done, abort_flag;
  constexpr int kGroups = 64 / kC;
  const int b = int(blockIdx.x), lo = b & 7;
  const int cg = (b / 8) % kGroups;
  const int pg = (b / (8 * kGroups)) * 8 + lo;
  if (pg >= a.n_pairs) return;  // padding workgroup (before the barrier)
  const int n_segs = int(a.n_segs);
  for (int j = int(threadIdx.x); j < n_segs; j += int(blockDim.x)) {
    const plato_agg_segment sg = a.segs[j];
    S[j] = AdpSeg{uint32_t(sg.flat_offset), uint32_t(sg.flat_offset + sg.numel), uint32_t(sg.src_offset),
                  (sg.region ? kSegI64 : 0u) | ((sg.flags & PLATO_AGG_SEG_NEG_DIV) ? kSegNeg : 0u)};
  }
  if (threadIdx.x < kRing) full[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    done = 0;
    abort_flag = 0;
  }
  __syncthreads();  // the only workgroup barrier
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = int(threadIdx.x & 63);
  const uint32_t nst = uint32_t((a.nsteps + kS - 1) / kS);
  const bool xx_active = pg == 0 && a.with_xx;
  const uint32_t nchain = xx_active ? 2u : 1u;
  if (wave >= 2) {  // producer
    const int w = wave - 2;
    AdpSrc<1> src;
    src.x = adp_rsrc(a.x, a.nsteps * 256);
    src.b = adp_rsrc(a.base_f, a.n_f32 * 4);
    src.y[0] = adp_rsrc(sld(a.xf, pg), a.n_f32 * 4);
    AdpCursor cursor;
    adp_cursor_load(S, 0, cursor);
    AdpRegs4<1, kIt> regs[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j)
      adp_issue4<1, kC, kS, kW, kIt, 0>(a, S, n_segs, cursor, src, uint32_t(j) < nst ? uint32_t(j) : nst, cg, w, lane,
                                        regs[j]);
    for (uint32_t t0 = 0; t0 < nst; t0 += kD) {
#pragma unroll
      for (int j = 0; j < kD; ++j) {
        const uint32_t t = t0 + j;
        if (t < nst) {  // wave-uniform
          if (t >= uint32_t(kRing)) adp_wait_geq(&done, nchain * (t + 1 - kRing), &abort_flag);
          adp_write4<1, kC, kS, kW, kIt, 0, 0>(a, S, n_segs, ring + (t % kRing) * Sh::kSlot, pg, w, lane, regs[j]);
          const uint32_t nxt = t + kD;
          adp_issue4<1, kC, kS, kW, kIt, 0>(a, S, n_segs, cursor, src, nxt < nst ? nxt : nst, cg, w, lane, regs[j]);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this wave's part of stage t is in LDS
          if (lane == 0) atomicAdd(&full[t % kRing], 1u);
        }
      }
    }
    return;
  }
  const bool xx = wave == 1;
  if (xx && !xx_active) return;
  __builtin_amdgcn_s_setprio(3);
  const int kind = xx ? 0 : lane >> 5, c = xx ? lane % kC : (lane & 31);
  const int arow = (xx || kind == 0 ? 0 : Sh::kVR) + Sh::row(c);
  const int brow = (xx ? 0 : Sh::kVR) + Sh::row(c);
  float acc = 0.f;
  for (uint32_t t = 0; t < nst; ++t) {
    adp_wait_geq(&full[t % kRing], uint32_t(kW) * (t / kRing + 1), &abort_flag);
    const float* slot = ring + (t % kRing) * Sh::kSlot;
    const float* A = slot + arow;
    const float* B = slot + brow;
    const uint64_t left = a.nsteps - uint64_t(t) * kS;
    if (left >= uint64_t(kS)) {
      f4v av[4], bv[4], an[4], bn[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[q] = *reinterpret_cast<const f4v*>(A + 4 * q);
        bv[q] = *reinterpret_cast<const f4v*>(B + 4 * q);
      }
#pragma unroll
      for (int blk = 0; blk < kS / 16; ++blk) {
        if (blk + 1 < kS / 16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            an[q] = *reinterpret_cast<const f4v*>(A + 16 * (blk + 1) + 4 * q);
            bn[q] = *reinterpret_cast<const f4v*>(B + 16 * (blk + 1) + 4 * q);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc = chain_fma(av[q].x, bv[q].x, acc);
          acc = chain_fma(av[q].y, bv[q].y, acc);
          acc = chain_fma(av[q].z, bv[q].z, acc);
          acc = chain_fma(av[q].w, bv[q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          av[q] = an[q];
          bv[q] = bn[q];
        }
      }
    } else {
      for (int s = 0; s < int(left); ++s) acc = chain_fma(A[s], B[s], acc);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this stage's reads are consumed
    if (lane == 0) atomicAdd(&done, 1u);
  }
  if (__hip_atomic_load(&abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) acc = __builtin_nanf("");
  const int chain = cg * kC + c;
  if (!xx) {
    a.ws[uint64_t(pg) * 128 + uint64_t(kind) * 64 + chain] = acc;
  } else if (lane < kC) {  // the virtual pair (g, g)
    a.ws[uint64_t(a.n_pairs) * 128 + chain] = acc;
    a.ws[uint64_t(a.n_pairs) * 128 + 64 + chain] = acc;
  }
}

template <int kC, int kS, int kW, int kIt, int kD, int kRing>
void launch_adp_flag(const AdpArgs& a, hipStream_t st) {
  constexpr int kGroups = 64 / kC;
  const uint32_t pgs = uint32_t((a.n_pairs + 7) / 8 * 8);
  hipLaunchKernelGGL((fedadp_dots_flag_kernel<kC, kS, kW, kIt, kD, kRing>), dim3(pgs * kGroups), dim3(64 * (kW + 2)), 0,
                     st, a);
}

template <int kP, int kC, int kS, int kW, int kIt, int kVRpad, int kProbe = 0, int kIso = 0, int kV = 1, int kD = 2,
          int kCP = 1, int kPrio = 3, int kSw = 0, int kNt = 0>
void launch_adp(const AdpArgs& a, hipStream_t st) {
  constexpr int kGroups = 64 / kC;
  uint32_t pgs = uint32_t((a.n_pairs + kP - 1) / kP);
  pgs = (pgs + 7) / 8 * 8;  // whole XCD rounds (padding workgroups return at once)
  hipLaunchKernelGGL((fedadp_dots_kernel<kP, kC, kS, kW, kIt, kVRpad, kProbe, kIso, kV, kD, kCP, kPrio, kSw, kNt>), dim3(pgs * kGroups),
                     dim3((64 * adp_waves<kW, kIso>())), 0, st, a);
}
using AdpFn = void (*)(const AdpArgs&, hipStream_t);
// pairs x chains per workgroup, steps per stage, producer waves, iterations, vector pad
// The product's shape (tuning variant 23): one pair and 32 of its 64 chains per workgroup, so a
// gather reads whole 128-byte lines, 16 bytes per lane (x and b come once per pair, from L2);
// 1.94 ms for 128 ResNet-18 clients against 5.4 ms for variant 0 (profiles/r03i_fedadp.log); with
// the swizzled rows (variant 51: no LDS bank conflicts, LDS-array cycles 450 M -> 181 M) 1.90 ms
// (profiles/r03w_fedadp.log)
constexpr AdpFn kAdpDefault = &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2>;
#ifdef PLATO_AGG_TUNE
const AdpFn kAdpVariants[] = {
    &launch_adp<8, 4, 256, 8, 2, 0>,     // 0: 16 B per block per vector, x and b shared by 8 pairs
    &launch_adp<4, 8, 256, 8, 4, 16>,    // 1: 32 B
    &launch_adp<2, 16, 256, 8, 8, 32>,   // 2: 64 B
    &launch_adp<1, 32, 128, 8, 8, 0>,    // 3: whole 128-byte lines, x and b per pair (from L2)
    &launch_adp<2, 16, 192, 12, 4, 32>,  // 4: variant 2 with 12 producer waves
    &launch_adp<2, 16, 128, 8, 4, 32>,   // 5: variant 2, half stages
    &launch_adp<2, 16, 256, 8, 8, 32, 1>,  // 6: probe of 2 without the division (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 2>,  // 7: probe of 2 without the chains (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 3>,  // 8: probe of 2 without the loads (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 4>,  // 9: probe of 2: the chains alone (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 5>,  // 10: probe of 2: chains without LDS reads (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 0, 1>,  // 11: variant 2, chain waves on a SIMD of their own
    &launch_adp<2, 16, 128, 8, 4, 32, 0, 1>,  // 12: variant 5, chain waves on a SIMD of their own
    &launch_adp<4, 8, 256, 8, 4, 16, 0, 1>,   // 13: variant 1, chain waves on a SIMD of their own
    &launch_adp<1, 32, 128, 8, 8, 0, 0, 1>,   // 14: variant 3, chain waves on a SIMD of their own
    &launch_adp<2, 16, 256, 8, 8, 32, 4, 1>,  // 15: probe of 11: the chains alone (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 2, 1>,  // 16: probe of 11: no chains (wrong results)
    &launch_adp<2, 16, 256, 8, 8, 32, 6>,     // 17: probe of 2: cycle counts per wave into the workspace
    &launch_adp<2, 16, 128, 8, 4, 32, 6, 1>,  // 18: probe of 12: cycle counts per wave into the workspace
    &launch_adp<2, 16, 256, 8, 2, 32, 0, 0, 4>,  // 19: variant 2, 16-byte gathers
    &launch_adp<2, 16, 128, 8, 1, 32, 0, 0, 4>,  // 20: variant 5, 16-byte gathers
    &launch_adp<2, 16, 256, 8, 2, 32, 0, 1, 4>,  // 21: variant 19, chain waves on a SIMD of their own
    &launch_adp<4, 8, 256, 8, 1, 16, 0, 0, 4>,   // 22: variant 1, 16-byte gathers
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4>,   // 23: variant 3, 16-byte gathers
    &launch_adp<8, 4, 256, 4, 1, 0, 0, 0, 4>,    // 24: variant 0, 16-byte gathers (4 producer waves)
    &launch_adp<2, 16, 256, 8, 2, 32, 6, 0, 4>,  // 25: probe of 19: cycle counts per wave into the workspace
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 3>,   // 26: variant 23, 3 stages of loads in flight
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 4>,   // 27: variant 23, 4 stages of loads in flight
    &launch_adp<2, 16, 128, 8, 1, 32, 0, 0, 4, 4>,  // 28: variant 20, 4 stages of loads in flight
    &launch_adp<1, 32, 128, 8, 2, 0, 6, 0, 4, 3>,   // 29: probe of 26: cycle counts per wave into the workspace
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 1, 4, 3>,   // 30: variant 26, chain waves on a SIMD of their own
    &launch_adp<1, 32, 128, 8, 8, 0, 0, 0, 1, 3>,   // 31: variant 3, 3 stages of loads in flight
    &launch_adp<1, 32, 192, 8, 3, 0, 0, 0, 4>,      // 32: variant 23 with 192-step stages
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 2>,  // 33: variant 23, chain reads 2 blocks ahead
    &launch_adp<1, 32, 192, 8, 3, 0, 0, 0, 4, 2, 2>,  // 34: variant 32, chain reads 2 blocks ahead
    &launch_adp<1, 32, 128, 8, 2, 0, 4, 0, 4>,      // 35: probe of 23: the chains alone (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 2, 0, 4>,      // 36: probe of 23: no chains (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 6, 0, 4>,      // 37: probe of 23: cycle counts per wave
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 3>,  // 38: variant 23, chain reads 3 blocks ahead
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 0>,  // 39: variant 23, chain wave at priority 0
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 1>,  // 40: variant 23, chain wave at priority 1
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 1, 4, 2, 1, 0>,  // 41: variant 30 (isolated chain SIMD), priority 0
    &launch_adp<1, 32, 128, 4, 4, 0, 0, 0, 4, 2>,        // 42: variant 23 with 4 producer waves
    &launch_adp<1, 32, 192, 12, 2, 0, 0, 0, 4, 2>,       // 43: variant 32 with 12 producer waves
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 1>,  // 44: variant 23 with the row gap (conflict-free writes)
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 1, 4, 2, 1, 3, 1>,  // 45: variant 30 with the row gap
    &launch_adp<1, 32, 192, 8, 3, 0, 0, 0, 4, 2, 1, 3, 1>,  // 46: variant 32 with the row gap
    &launch_adp<2, 16, 128, 8, 1, 32, 0, 0, 4, 2, 1, 3, 1>, // 47: variant 20 with the row gap
    &launch_adp_flag<32, 128, 8, 2, 2, 2>,  // 48: variant 23 synchronised by LDS counters, 2 tile slots
    &launch_adp_flag<32, 128, 8, 2, 2, 3>,  // 49: the same, 3 tile slots
    &launch_adp_flag<32, 128, 8, 2, 3, 3>,  // 50: 3 tile slots, 3 stages of loads in flight
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2>,  // 51: variant 23 with swizzled rows (conflict-free writes)
    &launch_adp<1, 32, 128, 8, 2, 0, 4, 0, 4, 2, 1, 3, 2>,  // 52: probe of 51: the chains alone (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 3, 1, 3, 2>,  // 53: variant 51, 3 stages of loads in flight
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 2, 3, 2>,  // 54: variant 51, chain reads 2 blocks ahead
    &launch_adp<1, 32, 128, 8, 2, 0, 7, 0, 4, 2, 1, 3, 2>,  // 55: probe of 51: the producers alone (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2, 1>,  // 56: variant 51, client arenas read nt
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2, 2>,  // 57: variant 51, every load nt
    &launch_adp<1, 32, 128, 8, 2, 0, 7, 0, 4, 2, 1, 3, 2, 1>,  // 58: probe of 56: the producers alone (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 3, 1, 3, 2, 1>,  // 59: variant 56, 3 stages of loads in flight
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2, 4>,  // 60: variant 51, division as a float64 product
    &launch_adp<1, 32, 128, 8, 2, 0, 7, 0, 4, 2, 1, 3, 2, 4>,  // 61: probe of 60: the producers alone (wrong results)
    &launch_adp<1, 32, 128, 8, 2, 0, 0, 0, 4, 2, 1, 3, 2, 5>,  // 62: variant 60, client arenas read nt
};
constexpr int kNumAdpVariants = sizeof(kAdpVariants) / sizeof(kAdpVariants[0]);
// timing probes of the table above: wrong results by design (tests skip them)
constexpr int kAdpProbes[] = {6, 7, 8, 9, 10, 15, 16, 17, 18, 25, 29, 35, 36, 37, 52, 55, 58, 61};
#endif

int run_fedadp(AdpFn fn, const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64, int n_pairs,
               const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs, uint32_t n_segs,
               size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy,
               float* d_out_yy, hipStream_t stream);

}  // namespace

extern "C" {

size_t plato_agg_fedadp_dots_workspace(int n_pairs, int with_xx, size_t n_i64) {
  const size_t k = size_t(n_pairs > 0 ? n_pairs : 0);
  return ((k + (with_xx ? 1 : 0)) * 128 + k * n_i64) * sizeof(float);
}

int plato_agg_fedadp_dots(const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64, int n_pairs,
                          const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
                          uint32_t n_segs, size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace,
                          float* d_out_xy, float* d_out_yy, hipStream_t stream) {
  return run_fedadp(kAdpDefault, d_x, d_src_f32, d_src_i64, n_pairs, d_base_f32, d_base_i64, d_segs, n_segs, n_flat, n_f32,
                    n_i64, lr, with_xx, d_workspace, d_out_xy, d_out_yy, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_fedadp_variants(void) { return kNumAdpVariants; }

int plato_agg_tune_fedadp_is_probe(int variant) {
  for (int v : kAdpProbes)
    if (v == variant) return 1;
  return 0;
}

int plato_agg_tune_fedadp_dots(int variant, const float* d_x, const void* const* d_src_f32,
                               const void* const* d_src_i64, int n_pairs, const float* d_base_f32,
                               const int64_t* d_base_i64, const plato_agg_segment* d_segs, uint32_t n_segs,
                               size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy,
                               float* d_out_yy, hipStream_t stream) {
  if (variant < 0 || variant >= kNumAdpVariants) return set_error(PLATO_AGG_EINVAL, "bad fedadp_dots variant");
  return run_fedadp(kAdpVariants[variant], d_x, d_src_f32, d_src_i64, n_pairs, d_base_f32, d_base_i64, d_segs, n_segs, n_flat,
                    n_f32, n_i64, lr, with_xx, d_workspace, d_out_xy, d_out_yy, stream);
}
#endif  // PLATO_AGG_TUNE

}  // extern "C"

namespace {
int run_fedadp(AdpFn fn, const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64, int n_pairs,
               const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs, uint32_t n_segs,
               size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy,
               float* d_out_yy, hipStream_t stream) {
  if (n_pairs <= 0 || n_pairs > (1 << 20)) return set_error(PLATO_AGG_EINVAL, "n_pairs must be in [1, 2^20]");
  if (with_xx != 0 && with_xx != 1) return set_error(PLATO_AGG_EINVAL, "with_xx must be 0 or 1");
  if (!d_x || !d_src_f32 || !d_src_i64 || !d_base_f32 || !d_segs || !d_workspace || !d_out_xy || !d_out_yy ||
      (n_i64 && !d_base_i64))
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (reinterpret_cast<uintptr_t>(d_x) & 15u) return set_error(PLATO_AGG_EINVAL, "x must be 16-byte aligned");
  if (n_segs == 0 || n_segs > uint32_t(kMaxSegs))
    return set_error(PLATO_AGG_EINVAL, "segment count must be in [1, 2048]");
  if (n_flat == 0 || n_flat >= (size_t(1) << 32)) return set_error(PLATO_AGG_EINVAL, "flat length must be in [1, 2^32)");
  if (n_f32 >= (size_t(1) << 30)) return set_error(PLATO_AGG_EINVAL, "fp32 arena must be < 2^30 elements");
  AdpArgs a{};
  a.x = d_x;
  a.xf = reinterpret_cast<const float* const*>(d_src_f32);
  a.xi = reinterpret_cast<const int64_t* const*>(d_src_i64);
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.segs = d_segs;
  a.n_segs = n_segs;
  a.n = n_flat;
  a.nsteps = (uint64_t(n_flat) & ~uint64_t(31)) / 64;
  a.lr = lr;
  a.ws = static_cast<float*>(d_workspace);
  a.y64 = a.ws + (uint64_t(n_pairs) + (with_xx ? 1 : 0)) * 128;
  a.n_i64 = n_i64;
  a.n_f32 = n_f32;
  a.n_pairs = n_pairs;
  a.with_xx = with_xx;
  if (n_i64) {
    hipLaunchKernelGGL(fedadp_i64_kernel, dim3(uint32_t(n_pairs)), dim3(64), 0, stream, a);
    if (int rc = check_launch("fedadp_i64 launch")) return rc;
  }
  if (a.nsteps) {
    fn(a, stream);
    if (int rc = check_launch("fedadp_dots launch")) return rc;
  } else {
    (void)hipMemsetAsync(d_workspace, 0, (size_t(n_pairs) + (with_xx ? 1 : 0)) * 128 * sizeof(float), stream);
  }
  hipLaunchKernelGGL(fedadp_finish_kernel, dim3(uint32_t(n_pairs + with_xx)), dim3(64), 0, stream, a, d_out_xy,
                     d_out_yy);
  return check_launch("fedadp_finish launch");
}
}  // namespace
