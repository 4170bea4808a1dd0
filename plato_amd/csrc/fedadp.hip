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
// The flattening is folded into the dot kernel: producer waves gather positions from the staged
// client arenas, form loc = (y - b) or -(y - b) / lr in registers and write them transposed into
// an LDS tile; a chain wave only runs the fma chains out of LDS.
//
// Shape (one workgroup per CU for 128 clients):
//   * 1 pair (client) x 32 of the 64 chains per workgroup (chain group cg = half of every
//     64-block); a gather iteration of a producer wave covers the cg halves of 8 consecutive
//     blocks (a "group", 256 positions): 16 bytes per lane, whole 128-byte lines of the client
//     arena; the two chain groups of a pair run on one XCD.
//   * per (cg, group) one 8-byte descriptor (fedadp_desc_kernel, read by a scalar load): a group
//     inside one fp32 entry ("fast") reads the client arena at position + (arena offset - flat
//     offset) and divides by -lr or not; a group that crosses an entry boundary or holds int64
//     positions ("boundary", at most two per entry) reads its 256 finished values from a table
//     fedadp_boundary_kernel fills per pair before the launch — the same one 16-byte load per
//     lane, so the stream never waits on a per-position lookup.
//   * x (the flattened global gradient) and b (the baseline, flattened once per round by
//     fedadp_prep_span) come from one chain-group-major buffer: per (cg, group) the 256 x values
//     then the 256 b values — every x or b load of a wave is 1 KiB contiguous and 16-byte aligned.
//     (Gathered from the arena, b's 16-byte loads start 4-12 bytes off a 16-byte boundary wherever
//     an entry's arena offset and flat position differ mod 4, half of ResNet-18's elements;
//     scripts/micro/adp_stream.hip, profiles/r04*_adp_stream.log.)
//   * chain wave: lane = kind * 32 + chain, kind 0 = g . loc, kind 1 = loc . loc: ONE dependent
//     fma per step per lane, 4 steps per ds_read_b128 of a transposed row (row pitch kS + 16
//     floats, rows 4m .. 4m + 3 shifted by 4m floats: conflict-free ds_read_b128 and
//     ds_write_b32).
//   * kW producer waves, kIt gather iterations each per stage; their global loads run kD stages
//     ahead of the tile being written, the tile ring has two slots, one s_barrier per stage.
//   * g . g: an extra chain wave in the workgroups of pair 0 (x . x over the same tile).
// No segment map in the stream: any entry count.  Compiled with -ffp-contract=off; the chain fma
// is an explicit v_fma_f32.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

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
__device__ __forceinline__ T sld(const T* p, uint64_t i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

__device__ __forceinline__ float chain_fma(float a, float b, float c) {
  asm("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  return c;
}

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr uint32_t kDescBoundary = 1u, kDescNeg = 2u;

// Per (chain group, 8-block group): fast groups: `off` = arena offset - flat offset (mod 2^32) of
// the one fp32 entry the group lies in, flags kDescNeg if it is divided by -lr; boundary groups:
// flags kDescBoundary, `off` = the group's row of the boundary table
struct AdpDesc {
  uint32_t off;
  uint32_t flags;
};

struct AdpArgs {
  const float* x;                // flattened global gradient (process_grad(g)), >= nsteps * 64 floats
  const float* xb;               // [2][ngroups][512]: chain-group-major x and b (fedadp_prep_span)
  const float* const* xf;        // client fp32 arenas
  const int64_t* const* xi;      // client int64 arenas
  const float* base_f;
  const int64_t* base_i;
  const plato_agg_segment* segs;
  AdpDesc* desc;                 // [2][ngroups]
  uint32_t* bnd_at;              // [max_bnd]: (cg, group) of each boundary row
  uint32_t* n_bnd;               // number of boundary rows
  uint32_t* cnt;                 // [ceil(2 ngroups / 256)]: boundary groups per descriptor block
  float* bnd;                    // [n_pairs][max_bnd][256]: process_grad's values of the boundary groups
  uint32_t* bsrc;                // [max_bnd][256]: the source word of each boundary value (fedadp_bndsrc_kernel)
  uint32_t n_segs;
  uint32_t ngroups;              // 8-block groups: ceil(nsteps / 8)
  uint32_t max_bnd;              // >= boundary groups (adp_max_bnd)
  uint64_t n;                    // flat length
  uint64_t nsteps;               // whole 64-element blocks before sdot's 32-block and tail
  float lr;
  double inv_lr;                 // 1 / double(lr)
  float* ws;                     // [n_pairs + with_xx][128]: chain sums of x.y, then of y.y
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

// (-d) / lr, correctly rounded, as RN32(RN64(-d * RN64(1 / lr))): the float64 product is within
// 2^-52 (relative) of the quotient, while a quotient of two floats that is not a float lies at
// least 2^-49 (relative) from every midpoint of the float grid (and is never on one), so the one
// rounding to float gives the float32 division's bits (tests/test_division.py) — 3 instructions
// instead of the division's ~10
__device__ __forceinline__ float adp_div_lr_f64(float v, double inv_lr) { return float(double(v) * inv_lr); }

// The last segment with flat_offset <= p (segments are in flat order).
__device__ __forceinline__ uint32_t adp_find(const plato_agg_segment* segs, uint32_t n, uint64_t p) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].flat_offset <= p) lo = mid; else hi = mid;
  }
  return lo;
}

// process_grad's value at position p of pair `pair`, in segment sidx (the boundary groups and the epilogue)
__device__ float adp_y_in(const AdpArgs& a, int pair, uint64_t p, uint32_t sidx) {
  const plato_agg_segment sg = a.segs[sidx];
  const uint64_t e = sg.src_offset + (p - sg.flat_offset);
  const bool neg = sg.flags & PLATO_AGG_SEG_NEG_DIV;
  if (sg.region) return adp_i64(a.xi[pair][e], a.base_i ? a.base_i[e] : int64_t(0), neg, a.lr);
  return adp_f32(a.xf[pair][e], a.base_f ? a.base_f[e] : 0.f, neg, a.lr);
}
__device__ float adp_y_at(const AdpArgs& a, int pair, uint64_t p) {
  return adp_y_in(a, pair, p, adp_find(a.segs, a.n_segs, p));
}

// Tuning flags (kF): client arenas read non-temporally, the division as a float64 product, x and
// b from the chain-group-major buffer (else x from the flat vector and b from the baseline arena);
// kFDelta: the client arenas hold deltas (y - b, formed when each payload was staged), so the
// producers load no b at all: y - 0 is y bit for bit (also -0, NaN), the same values as y - b formed
// here, and each (cg, group) stage streams x and the client only
constexpr int kFYnt = 1, kFDiv64 = 4, kFXB = 8, kFDelta = 16;

// 32 of the 64 chains per workgroup; kS steps per stage; kW producer waves, kIt gather iterations
// of one group (8 half-blocks x 32 positions) each per stage
template <int kS, int kW, int kIt>
struct AdpShape {
  static constexpr int kC = 32;
  static_assert(kS * kC == 256 * kW * kIt, "a stage is kW x kIt gather iterations of 256 positions");
  static_assert(kS % 64 == 0, "swizzled rows: whole 64-step row groups");
  // transposed row pitch (floats) kS + 16 and rows 4m .. 4m + 3 shifted by 4m floats: a
  // ds_write_b32 half-wave (banks (a/4) mod 32) of the producers writes rows 4m + j, m = 0..7, on
  // 8 different 4-bank slots, and every 16-lane group of the chain's ds_read_b128 (banks mod 64)
  // covers 16 different slots (pitch = 16 mod 64)
  static constexpr int kR = kS + 16;
  static constexpr int kVR = kC * kR + 4 * (kC / 4);  // rows of one vector (x or loc)
  __device__ static constexpr int row(int r) { return r * kR + 4 * (r >> 2); }
  static constexpr int kSlot = 2 * kVR;
  static constexpr int kBlkPerIt = 8;  // 64-blocks per gather iteration (one group)
  static constexpr int kLpB = 8;       // lanes per half-block
};

// One producer wave's loads for kIt iterations: 4 consecutive positions per lane, 16-byte loads
template <int kIt>
struct AdpRegs {
  f4v x[kIt];
  f4v b[kIt];
  f4v y[kIt];
  uint32_t flags[kIt];  // the group's descriptor flags (wave-uniform)
};

struct AdpSrc {
  __amdgpu_buffer_rsrc_t x, b, y, bnd;
};

// Buffer resources: raw buffer loads take a 32-bit byte offset per lane against a descriptor in
// SGPRs, so a gathered load costs no 64-bit address arithmetic (an offset past num_records reads 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t adp_rsrc(const void* base, uint64_t bytes) {
  const uint64_t n = bytes < 0xffffffffull ? bytes : 0xffffffffull;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)uint32_t(n), 0x00020000);
}

// kAux: the load's cache policy (2 = nt: a streaming read, kept out of the way of the re-read x and b)
template <int kAux = 0>
__device__ __forceinline__ f4v bload4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAux));
}

template <int kS, int kW, int kIt, int kF>
__device__ __forceinline__ void adp_issue(const AdpArgs& a, const AdpDesc* desc, const AdpSrc& src, uint32_t t, int cg,
                                          int w, int lane, AdpRegs<kIt>& r) {
  using Sh = AdpShape<kS, kW, kIt>;
  const uint32_t last = uint32_t(a.nsteps - 1);
  const uint32_t glast = a.ngroups - 1;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const uint32_t grp = min(t * uint32_t(kS / 8) + uint32_t(i * kW + w), glast);  // past the end: re-read a valid group
    const uint32_t s = min(grp * 8u + uint32_t(lane / Sh::kLpB), last);  // a ragged last group re-reads a valid block
    const uint32_t p = s * 64 + uint32_t(cg * Sh::kC + (lane % Sh::kLpB) * 4);
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(desc);  // wave-uniform: one scalar load
    const AdpDesc d{sld(dw, 2 * uint64_t(grp)), sld(dw, 2 * uint64_t(grp) + 1)};
    r.flags[i] = d.flags;
    // one load of the client's values per lane on both paths (the compiler's vmcnt bookkeeping
    // covers exactly one stage): the arena for a fast group, the boundary table otherwise
    const bool bnd = d.flags & kDescBoundary;
    const __amdgpu_buffer_rsrc_t ry = bnd ? src.bnd : src.y;
    const uint32_t yo = bnd ? (d.off * 256u + uint32_t(lane) * 4u) * 4u : (p + d.off) * 4u;
    r.y[i] = bload4<(kF & kFYnt) ? 2 : 0>(ry, yo);
    if constexpr ((kF & kFDelta) != 0) {
      // delta arenas: no b; x from the chain-group-major buffer, or (round 6) straight from the flat
      // gradient: 8 lanes read one 128-byte run of a half-block, whole lines, 16-byte aligned (p = 0 mod 4)
      r.x[i] = (kF & kFXB) ? bload4<0>(src.x, (grp * 512u + uint32_t(lane) * 4u) * 4u) : bload4<0>(src.x, p * 4u);
      r.b[i] = f4v{0.f, 0.f, 0.f, 0.f};
    } else if constexpr ((kF & kFXB) != 0) {  // [cg][group][x: 256 | b: 256], lane l at 4 l
      const uint32_t q = (grp * 512u + uint32_t(lane) * 4u) * 4u;
      r.x[i] = bload4<0>(src.x, q);
      r.b[i] = bload4<0>(src.x, q + 1024u);
    } else {
      r.x[i] = bload4<0>(src.x, p * 4u);
      r.b[i] = bload4<0>(src.b, bnd ? 0u : (p + d.off) * 4u);
    }
  }
}

template <int kS, int kW, int kIt, int kF>
__device__ __forceinline__ void adp_write(const AdpArgs& a, float* slot, int w, int lane, AdpRegs<kIt>& r) {
  using Sh = AdpShape<kS, kW, kIt>;
  const float lr = a.lr;
  const double inv_lr = a.inv_lr;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const int g = i * kW + w;
    const int col = g * Sh::kBlkPerIt + lane / Sh::kLpB;  // step within the stage
    float* dst = slot + Sh::row((lane % Sh::kLpB) * 4) + col;  // chain c0 = 4 * (lane % kLpB), rows c0 .. c0 + 3
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j * Sh::kR] = r.x[i][j];
    const uint32_t flags = __builtin_amdgcn_readfirstlane(r.flags[i]);
    if (flags & kDescBoundary) {  // the finished values
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[Sh::kVR + j * Sh::kR] = r.y[i][j];
    } else if (flags & kDescNeg) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float nv = -(r.y[i][j] - r.b[i][j]);
        dst[Sh::kVR + j * Sh::kR] = (kF & kFDiv64) ? adp_div_lr_f64(nv, inv_lr) : nv / lr;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[Sh::kVR + j * Sh::kR] = r.y[i][j] - r.b[i][j];
    }
  }
}

// kProbe (tuning only, wrong results by design): 1 = the chains alone (producers keep only the
// barrier count), 2 = the producers alone (the chain wave reads one value per stage, which keeps
// the producers' stores and loads live)
template <int kS, int kW, int kIt, int kD, int kF, int kProbe = 0>
__global__ __launch_bounds__(64 * (kW + 2)) void fedadp_dots_kernel(AdpArgs a) {
  using Sh = AdpShape<kS, kW, kIt>;
  static_assert(kD >= 2 && kD <= 4, "2-4 stages of loads in flight per producer wave");
  __shared__ __attribute__((aligned(16))) float ring[2 * Sh::kSlot];
  // workgroups are dealt to the 8 XCDs round-robin: the 2 chain groups of a pair get ids that
  // agree mod 8, so they share one XCD and its L2
  const int b = int(blockIdx.x), lo = b & 7;
  const int cg = (b / 8) % 2;
  const int pg = (b / 16) * 8 + lo;
  if (pg >= a.n_pairs) return;  // padding workgroup (before any barrier)
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = int(threadIdx.x & 63);
  const uint64_t nsteps = a.nsteps;
  const uint64_t nst = (nsteps + kS - 1) / kS;
  const uint64_t nst2 = (nst + kD - 1) / kD * kD;  // barriers: one per stage, in whole trips of kD stages
  if (wave >= 2) {  // producer w
    const int w = wave - 2;
    if (kProbe == 1) {
      for (uint64_t t = 0; t < nst2; ++t) __builtin_amdgcn_s_barrier();
      return;
    }
    AdpSrc src;
    if (kF & kFXB) {
      src.x = adp_rsrc(a.xb + uint64_t(cg) * a.ngroups * 512, uint64_t(a.ngroups) * 512 * 4);
      src.b = src.x;
    } else {
      src.x = adp_rsrc(a.x, a.nsteps * 256);
      src.b = adp_rsrc(a.base_f, a.n_f32 * 4);
    }
    src.y = adp_rsrc(sld(a.xf, uint64_t(pg)), a.n_f32 * 4);
    src.bnd = adp_rsrc(a.bnd + uint64_t(pg) * a.max_bnd * 256, uint64_t(a.max_bnd) * 256 * 4);
    const AdpDesc* desc = a.desc + uint64_t(cg) * a.ngroups;
    // kD register sets: the loads of stage t + kD go out right after stage t is written, so every
    // producer wave keeps kD stages of loads in flight; the tile ring in LDS has two slots
    AdpRegs<kIt> regs[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j) adp_issue<kS, kW, kIt, kF>(a, desc, src, uint32_t(j), cg, w, lane, regs[j]);
    // whole trips of kD stages (the last trip may run idle stages): no branch inside the loop, so the
    // compiler's vmcnt bookkeeping sees the same kD stages in flight on every trip
    for (uint32_t t = 0; t < uint32_t(nst2); t += kD) {
#pragma unroll
      for (int j = 0; j < kD; ++j) {
        adp_write<kS, kW, kIt, kF>(a, ring + ((t + j) & 1) * Sh::kSlot, w, lane, regs[j]);
        // past the last stage every group clamps to the last one: valid addresses, never consumed
        const uint32_t nxt = t + j + kD;
        adp_issue<kS, kW, kIt, kF>(a, desc, src, nxt < nst ? nxt : uint32_t(nst), cg, w, lane, regs[j]);
        __builtin_amdgcn_s_barrier();  // stage t + j published in slot (t + j) & 1
      }
    }
    return;
  }
  // chain waves: wave 0 the pair's dots, wave 1 g . g (pair group 0 only; elsewhere it only keeps
  // the barrier count)
  __builtin_amdgcn_s_setprio(3);  // the chain wave issues first
  const bool xx = wave == 1;
  const bool active = !xx || (pg == 0 && a.with_xx);
  const int kind = xx ? 0 : lane >> 5, c = lane & 31;
  const int arow = (xx || kind == 0 ? 0 : Sh::kVR) + Sh::row(c);
  const int brow = (xx ? 0 : Sh::kVR) + Sh::row(c);
  float acc = 0.f;
  for (uint64_t t = 0; t < nst2; ++t) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (!active || t >= nst) continue;
    const float* slot = ring + (t & 1) * Sh::kSlot;
    const float* A = slot + arow;
    const float* B = slot + brow;
    if (kProbe == 2) {
      acc += A[t & 15] * B[t & 15];
      continue;
    }
    const uint64_t left = nsteps - t * kS;
    if (left >= uint64_t(kS)) {
      // 16 steps per block of 4 ds_read_b128 pairs; the next block's reads in flight
      constexpr int kNB = kS / 16;
      f4v av[2][4], bv[2][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[0][q] = *reinterpret_cast<const f4v*>(A + 4 * q);
        bv[0][q] = *reinterpret_cast<const f4v*>(B + 4 * q);
      }
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        const int nb = blk + 1;
        if (nb < kNB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            av[nb % 2][q] = *reinterpret_cast<const f4v*>(A + 16 * nb + 4 * q);
            bv[nb % 2][q] = *reinterpret_cast<const f4v*>(B + 16 * nb + 4 * q);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        const int cb = blk % 2;
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
  const int chain = cg * Sh::kC + c;
  if (!xx) {
    a.ws[uint64_t(pg) * 128 + uint64_t(kind) * 64 + chain] = acc;
  } else if (active && lane < Sh::kC) {  // the virtual pair (g, g): its x.y and y.y chains are both g.g
    a.ws[uint64_t(a.n_pairs) * 128 + chain] = acc;
    a.ws[uint64_t(a.n_pairs) * 128 + 64 + chain] = acc;
  }
}

// The descriptor of every (cg, group): fast if all its positions (whole blocks only) lie in one
// fp32 entry, else a boundary group (its row in the table comes from fedadp_rows_kernel); and the
// boundary groups of each 256-descriptor block, for the rows' scan
__global__ __launch_bounds__(256) void fedadp_desc_kernel(AdpArgs a) {
  __shared__ uint32_t wave_cnt[4];
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  bool bnd = false;
  if (j < 2 * a.ngroups) {
    const uint32_t cg = j / a.ngroups, grp = j % a.ngroups;
    const uint64_t s_last = min(uint64_t(grp) * 8 + 7, a.nsteps - 1);
    const uint64_t pf = uint64_t(grp) * 8 * 64 + cg * 32, pl = s_last * 64 + cg * 32 + 31;
    const plato_agg_segment sg = a.segs[adp_find(a.segs, a.n_segs, pf)];
    AdpDesc d;
    if (!sg.region && pl < sg.flat_offset + sg.numel) {
      d.off = uint32_t(sg.src_offset - sg.flat_offset);  // mod 2^32: position + off = arena element
      d.flags = (sg.flags & PLATO_AGG_SEG_NEG_DIV) ? kDescNeg : 0u;
    } else {
      d.off = 0;
      d.flags = kDescBoundary;
      bnd = true;
    }
    a.desc[j] = d;
  }
  const uint64_t m = __ballot(bnd);
  if ((threadIdx.x & 63) == 0) wave_cnt[threadIdx.x >> 6] = uint32_t(__popcll(m));
  __syncthreads();
  if (threadIdx.x == 0) a.cnt[blockIdx.x] = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
}

// Rows of the boundary table, in (cg, group) order: one workgroup per 256-descriptor block; the
// block's first row is the sum of the earlier blocks' counts, each boundary descriptor's row within
// the block its rank among the block's boundary descriptors (ballots); the last block writes the total
__global__ __launch_bounds__(256) void fedadp_rows_kernel(AdpArgs a) {
  __shared__ uint32_t part[4], wave_cnt[4];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t before = 0;
  for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 256) before += a.cnt[b];
  for (int d = 32; d >= 1; d >>= 1) before += __shfl_xor(before, d, 64);
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  const bool bnd = j < 2 * a.ngroups && (a.desc[j].flags & kDescBoundary);
  const uint64_t m = __ballot(bnd);
  if (lane == 0) {
    part[wave] = before;
    wave_cnt[wave] = uint32_t(__popcll(m));
  }
  __syncthreads();
  uint32_t row = part[0] + part[1] + part[2] + part[3];
  for (uint32_t w = 0; w < wave; ++w) row += wave_cnt[w];
  row += uint32_t(__popcll(m & ((uint64_t(1) << lane) - 1)));
  if (bnd) {
    a.desc[j].off = row;
    if (row < a.max_bnd) a.bnd_at[row] = j;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) *a.n_bnd = row + (bnd ? 1u : 0u);
}

// The boundary table: process_grad's values of every boundary group of every pair, in the lane
// order of the stream (index u * 32 + v: block 8 group + u, position cg * 32 + v); 0 past the
// last whole block.  Two launches: the positions' sources depend on the layout only, so one
// workgroup per boundary row finds them once (segment search and walk) and packs each into a
// word; the per-pair launch then costs one source word and one client load per value, R rows per
// workgroup with their loads in flight together.  (Round 5 ran the search per (row, pair), one row
// per workgroup: 25 us for ResNet-18 at K = 128; walking the rows with 16 workgroups per pair made
// the searches serial, 49 us, profiles/r06l_kernel_stats.csv.)
// Source word: the arena element (bits 0-29; both regions are < 2^30 elements, run_fedadp), bit 30
// the int64 region, bit 31 the division by -lr; kBndNone past the last whole block.
constexpr uint32_t kBndI64 = 1u << 30, kBndNeg = 1u << 31, kBndNone = 0xffffffffu;
__global__ __launch_bounds__(256) void fedadp_bndsrc_kernel(AdpArgs a) {
  const uint32_t row = blockIdx.x;
  if (row >= min(*a.n_bnd, a.max_bnd)) return;
  const uint32_t j = a.bnd_at[row];
  const uint32_t cg = j / a.ngroups, grp = j % a.ngroups;
  const uint32_t u = threadIdx.x / 32, v = threadIdx.x % 32;
  const uint64_t s = uint64_t(grp) * 8 + u;
  // one segment search per workgroup (its first position), then short forward walks: the group's
  // 512-position span crosses few segments
  __shared__ uint32_t first;
  if (threadIdx.x == 0) first = adp_find(a.segs, a.n_segs, uint64_t(grp) * 512 + cg * 32);
  __syncthreads();
  uint32_t word = kBndNone;
  if (s < a.nsteps) {
    const uint64_t p = s * 64 + cg * 32 + v;
    uint32_t idx = first;
    while (idx + 1 < a.n_segs && a.segs[idx + 1].flat_offset <= p) ++idx;
    const plato_agg_segment sg = a.segs[idx];
    word = uint32_t(sg.src_offset + (p - sg.flat_offset)) | (sg.region ? kBndI64 : 0u) |
           ((sg.flags & PLATO_AGG_SEG_NEG_DIV) ? kBndNeg : 0u);
  }
  a.bsrc[uint64_t(row) * 256 + threadIdx.x] = word;
}

constexpr uint32_t kBndRows = 4;  // boundary rows per workgroup of the per-pair launch
__device__ __forceinline__ void fedadp_boundary_rows(const AdpArgs& a, int pair, uint32_t bx) {
  const uint32_t nrows = min(*a.n_bnd, a.max_bnd);
  const uint32_t row0 = bx * kBndRows;
  if (row0 >= nrows) return;
  const float* xf = sld(a.xf, pair);
  const int64_t* xi = sld(a.xi, pair);
  uint32_t word[kBndRows];
#pragma unroll
  for (uint32_t r = 0; r < kBndRows; ++r)
    word[r] = row0 + r < nrows ? a.bsrc[uint64_t(row0 + r) * 256 + threadIdx.x] : kBndNone;
#pragma unroll
  for (uint32_t r = 0; r < kBndRows; ++r) {
    if (row0 + r >= nrows) break;
    float val = 0.f;
    const uint32_t w = word[r];
    if (w != kBndNone) {
      const uint32_t e = w & (kBndI64 - 1u);
      const bool neg = (w & kBndNeg) != 0;
      val = (w & kBndI64) ? adp_i64(xi[e], a.base_i ? a.base_i[e] : int64_t(0), neg, a.lr)
                          : adp_f32(xf[e], a.base_f ? a.base_f[e] : 0.f, neg, a.lr);
    }
    a.bnd[(uint64_t(pair) * a.max_bnd + row0 + r) * 256 + threadIdx.x] = val;
  }
}
__global__ __launch_bounds__(256) void fedadp_boundary_kernel(AdpArgs a) {
  fedadp_boundary_rows(a, int(blockIdx.y), blockIdx.x);
}

// The chain-group-major x / b buffer: xb[cg][grp][0..255] = x at the group's half-block positions
// (block 8 grp + u, position cg * 32 + v at index u * 32 + v), xb[cg][grp][256..511] = b at the
// same positions (the baseline through the segment map; 0 at int64 positions, whose values come
// from the boundary table).  A workgroup takes 2,048 consecutive flat positions and walks the
// segments overlapping them (workgroup-uniform), consecutive positions on consecutive lanes:
// coalesced reads of x and of each entry's baseline run, 128-byte runs of writes.
constexpr int kPrepSpan = 2048;
__device__ __forceinline__ void fedadp_prep_span(const AdpArgs& a, float* xb, uint32_t span) {
  const uint64_t np = a.nsteps * 64;  // whole blocks only
  const uint64_t b0 = uint64_t(span) * kPrepSpan;
  const uint64_t b1 = min(b0 + kPrepSpan, np);
  for (uint32_t sidx = adp_find(a.segs, a.n_segs, b0); sidx < a.n_segs; ++sidx) {
    const plato_agg_segment sg = a.segs[sidx];
    if (sg.flat_offset >= b1) break;
    const uint64_t lo = max(uint64_t(sg.flat_offset), b0), hi = min(uint64_t(sg.flat_offset + sg.numel), b1);
    const bool i64 = sg.region;
    for (uint64_t p = lo + threadIdx.x; p < hi; p += 256) {
      const uint64_t s = p / 64, c = p % 64;
      float* o = xb + ((c / 32) * a.ngroups + s / 8) * 512 + (s % 8) * 32 + (c % 32);
      o[0] = a.x[p];
      if (a.base_f) o[256] = i64 ? 0.f : a.base_f[p - sg.flat_offset + sg.src_offset];  // (delta arenas: no b)
    }
  }
}
// The prep spans and the per-pair boundary rows in one launch (they are independent): the boundary
// table's ~11 us of dependent loads run beside the prep copy instead of after it (round 6).
__global__ __launch_bounds__(256) void fedadp_prep_boundary_kernel(AdpArgs a, float* xb, uint32_t n_spans,
                                                                   uint32_t nbx) {
  if (blockIdx.x < n_spans) {
    fedadp_prep_span(a, xb, blockIdx.x);
  } else {
    const uint32_t b = blockIdx.x - n_spans;
    fedadp_boundary_rows(a, int(b / nbx), b % nbx);
  }
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

struct AdpLaunch {
  void (*fn)(const AdpArgs&, hipStream_t);
  bool uses_xb;
  bool delta;  // kFDelta: for delta arenas (null baseline)
};

template <int kS, int kW, int kIt, int kD, int kF, int kProbe>
void launch_adp_impl(const AdpArgs& a, hipStream_t st) {
  const uint32_t pgs = uint32_t((a.n_pairs + 7) / 8 * 8);  // whole XCD rounds (padding workgroups return at once)
  hipLaunchKernelGGL((fedadp_dots_kernel<kS, kW, kIt, kD, kF, kProbe>), dim3(pgs * 2), dim3(64 * (kW + 2)), 0, st, a);
}

template <int kS, int kW, int kIt, int kD, int kF, int kProbe = 0>
constexpr AdpLaunch adp_launch() {
  return AdpLaunch{&launch_adp_impl<kS, kW, kIt, kD, kF, kProbe>, (kF & kFXB) != 0, (kF & kFDelta) != 0};
}

// The product's shape: 192-step stages of 12 producer waves x 2 iterations, x and b from the
// chain-group-major buffer, the client arenas read non-temporally (once-read, kept out of the L2
// the re-read x and b live in), the division as a float64 product.  On aligned
// arenas the buffer still pays for its prep launch: without it (x from the flat gradient, b from
// the baseline arena) the whole call took 1.381 ms against 1.355 (profiles/r04v_fedadp.log).
constexpr AdpLaunch kAdpDefault = adp_launch<192, 12, 2, 2, kFYnt | kFDiv64 | kFXB>();
// Delta arenas (null baseline): the same shape without the b loads, three stages of loads in flight (the
// registers the b loads held): 1.077 / 1.080 against 1.088 / 1.092 ms with two, interleaved on two leases
// (profiles/r05zzu_delta_probe_shapes.log, r05zzm_delta_probe.log; 1.054 by rocprof with two, r05zzo)
constexpr AdpLaunch kAdpDefaultDelta = adp_launch<192, 12, 2, 3, kFYnt | kFDiv64 | kFXB | kFDelta>();
#ifdef PLATO_AGG_TUNE
const AdpLaunch kAdpVariants[] = {
    kAdpDefault,                                            // 0: the default
    adp_launch<128, 8, 2, 2, kFDiv64>(),                    // 1: round 3's stream (x flat, b from the arena), 128-step stages
    adp_launch<128, 8, 2, 2, kFDiv64 | kFXB>(),             // 2: x and b chain-group-major, 128-step stages
    adp_launch<192, 12, 2, 2, kFDiv64 | kFXB>(),            // 3: the default with plain (not nt) client loads
    adp_launch<256, 8, 4, 2, kFYnt | kFDiv64 | kFXB>(),     // 4: 256-step stages of 8 waves x 4 iterations
    adp_launch<128, 8, 2, 3, kFYnt | kFDiv64 | kFXB>(),     // 5: 128-step stages, 3 stages of loads in flight
    adp_launch<192, 12, 2, 2, kFYnt | kFXB>(),              // 6: the default with the IEEE division
    adp_launch<192, 12, 2, 2, kFYnt | kFDiv64 | kFXB, 1>(), // 7: probe: the default's chains alone
    adp_launch<192, 12, 2, 2, kFYnt | kFDiv64 | kFXB, 2>(), // 8: probe: the default's producers alone
    adp_launch<192, 12, 2, 2, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 9: the default's shape on delta arenas
                                                                     //    (null baseline), two stages in flight
    adp_launch<128, 8, 2, 2, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 10: delta arenas, 128-step stages
    adp_launch<256, 8, 4, 2, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 11: delta arenas, 256-step stages
    adp_launch<128, 8, 2, 3, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 12: delta arenas, 3 stages in flight
    kAdpDefaultDelta,                                        // 13: the default for delta arenas, 3 stages in flight
    adp_launch<192, 6, 4, 2, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 14: delta arenas, 6 producer waves x 4
    adp_launch<192, 8, 3, 2, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 15: delta arenas, 8 producer waves x 3
    adp_launch<192, 8, 3, 3, kFYnt | kFDiv64 | kFXB | kFDelta>(),  // 16: the same, 3 stages in flight
    adp_launch<192, 12, 2, 4, kFYnt | kFDiv64 | kFXB | kFDelta>(), // 17: 12 waves x 2, 4 stages in flight
    // round 6: delta arenas with x read straight from the flat gradient (no chain-group-major buffer, no prep launch)
    adp_launch<192, 12, 2, 3, kFYnt | kFDiv64 | kFDelta>(),        // 18: the delta default's shape
    adp_launch<192, 12, 2, 4, kFYnt | kFDiv64 | kFDelta>(),        // 19: 4 stages in flight
    adp_launch<192, 12, 2, 2, kFYnt | kFDiv64 | kFDelta>(),        // 20: 2 stages in flight
};
constexpr int kNumAdpVariants = sizeof(kAdpVariants) / sizeof(kAdpVariants[0]);
// timing probes of the table above: wrong results by design (tests skip them)
constexpr int kAdpProbes[] = {7, 8};
#endif

int run_fedadp(const AdpLaunch& fn, const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64,
               int n_pairs, const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
               uint32_t n_segs, size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace,
               float* d_out_xy, float* d_out_yy, hipStream_t stream, int flags);

// workspace: [chain sums][descriptors][boundary rows + count][block counts][boundary table][xb][boundary sources],
// 256-byte aligned parts
size_t align256(size_t v) { return (v + 255) / 256 * 256; }
// Boundary groups per chain group: one ends at (and so holds) each segment start — at most n_segs
// — plus the groups that lie wholly inside int64 entries, each holding 256 of the chain group's
// int64 positions: at most n_i64 / 256
size_t adp_max_bnd(uint32_t n_segs, size_t n_i64) { return 2 * (size_t(n_segs) + n_i64 / 256 + 1); }
struct AdpWs {
  size_t chains, desc, bnd_at, cnt, bnd, xb, bsrc, total;
};
AdpWs adp_ws(int n_pairs, int with_xx, size_t n_i64, size_t n_flat, uint32_t n_segs) {
  const size_t k = size_t(n_pairs > 0 ? n_pairs : 0);
  const size_t nsteps = (n_flat & ~size_t(31)) / 64, ngroups = (nsteps + 7) / 8;
  const size_t max_bnd = adp_max_bnd(n_segs, n_i64);
  AdpWs w{};
  w.chains = 0;
  w.desc = align256((k + (with_xx ? 1 : 0)) * 128 * sizeof(float));
  w.bnd_at = align256(w.desc + 2 * ngroups * sizeof(AdpDesc));
  w.cnt = align256(w.bnd_at + (max_bnd + 1) * sizeof(uint32_t));
  w.bnd = align256(w.cnt + (2 * ngroups + 255) / 256 * sizeof(uint32_t));
  w.xb = align256(w.bnd + k * max_bnd * 256 * sizeof(float));
  w.bsrc = align256(w.xb + 2 * ngroups * 512 * sizeof(float));
  w.total = w.bsrc + max_bnd * 256 * sizeof(uint32_t);
  return w;
}

}  // namespace

extern "C" {

size_t plato_agg_fedadp_dots_workspace(int n_pairs, int with_xx, size_t n_i64, size_t n_flat, uint32_t n_segs) {
  return adp_ws(n_pairs, with_xx, n_i64, n_flat, n_segs).total;
}

int plato_agg_fedadp_dots(const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64, int n_pairs,
                          const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
                          uint32_t n_segs, size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace,
                          float* d_out_xy, float* d_out_yy, hipStream_t stream) {
  return run_fedadp(d_base_f32 ? kAdpDefault : kAdpDefaultDelta, d_x, d_src_f32, d_src_i64, n_pairs, d_base_f32,
                    d_base_i64, d_segs, n_segs, n_flat, n_f32, n_i64, lr, with_xx, d_workspace, d_out_xy, d_out_yy,
                    stream, 0);
}

int plato_agg_fedadp_dots_ex(const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64,
                             int n_pairs, const float* d_base_f32, const int64_t* d_base_i64,
                             const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat, size_t n_f32,
                             size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy, float* d_out_yy,
                             hipStream_t stream, int flags) {
  if (flags & ~PLATO_AGG_FEDADP_TABLES_READY) return set_error(PLATO_AGG_EINVAL, "unknown fedadp_dots flags");
  return run_fedadp(d_base_f32 ? kAdpDefault : kAdpDefaultDelta, d_x, d_src_f32, d_src_i64, n_pairs, d_base_f32,
                    d_base_i64, d_segs, n_segs, n_flat, n_f32, n_i64, lr, with_xx, d_workspace, d_out_xy, d_out_yy,
                    stream, flags);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_fedadp_variants(void) { return kNumAdpVariants; }

int plato_agg_tune_fedadp_is_probe(int variant) {
  for (int v : kAdpProbes)
    if (v == variant) return 1;
  return 0;
}

int plato_agg_tune_fedadp_is_delta(int variant) {
  return (variant >= 0 && variant < kNumAdpVariants && kAdpVariants[variant].delta) ? 1 : 0;
}

int plato_agg_tune_fedadp_dots(int variant, const float* d_x, const void* const* d_src_f32,
                               const void* const* d_src_i64, int n_pairs, const float* d_base_f32,
                               const int64_t* d_base_i64, const plato_agg_segment* d_segs, uint32_t n_segs,
                               size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy,
                               float* d_out_yy, hipStream_t stream) {
  if (variant < 0 || variant >= kNumAdpVariants) return set_error(PLATO_AGG_EINVAL, "bad fedadp_dots variant");
  return run_fedadp(kAdpVariants[variant], d_x, d_src_f32, d_src_i64, n_pairs, d_base_f32, d_base_i64, d_segs, n_segs, n_flat,
                    n_f32, n_i64, lr, with_xx, d_workspace, d_out_xy, d_out_yy, stream, 0);
}
#endif  // PLATO_AGG_TUNE

}  // extern "C"

namespace {
int run_fedadp(const AdpLaunch& fn, const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64,
               int n_pairs, const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
               uint32_t n_segs, size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace,
               float* d_out_xy, float* d_out_yy, hipStream_t stream, int flags) {
  if (n_pairs <= 0 || n_pairs > 65535) return set_error(PLATO_AGG_EINVAL, "n_pairs must be in [1, 65535]");
  if (with_xx != 0 && with_xx != 1) return set_error(PLATO_AGG_EINVAL, "with_xx must be 0 or 1");
  if (!d_x || !d_src_f32 || !d_src_i64 || !d_segs || !d_workspace || !d_out_xy || !d_out_yy ||
      (d_base_f32 && n_i64 && !d_base_i64))
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (!d_base_f32 && d_base_i64) return set_error(PLATO_AGG_EINVAL, "int64 baseline without an fp32 baseline");
  // a null baseline means the arenas hold deltas: only the delta shapes run on them, and only on them
  if (fn.delta != (d_base_f32 == nullptr))
    return set_error(PLATO_AGG_EINVAL, fn.delta ? "this variant takes delta arenas (null baseline)"
                                                : "delta arenas (null baseline) need a delta variant");
  if ((reinterpret_cast<uintptr_t>(d_x) & 15u) || (reinterpret_cast<uintptr_t>(d_workspace) & 255u))
    return set_error(PLATO_AGG_EINVAL, "x must be 16-byte and the workspace 256-byte aligned");
  if (n_segs == 0 || n_segs >= (1u << 22)) return set_error(PLATO_AGG_EINVAL, "segment count must be in [1, 2^22)");
  if (n_flat == 0 || n_flat >= (size_t(1) << 30)) return set_error(PLATO_AGG_EINVAL, "flat length must be in [1, 2^30)");
  if (n_f32 >= (size_t(1) << 30)) return set_error(PLATO_AGG_EINVAL, "fp32 arena must be < 2^30 elements");
  if (n_i64 >= (size_t(1) << 30)) return set_error(PLATO_AGG_EINVAL, "int64 region must be < 2^30 elements");
  // boundary-table rows are 1 KiB, addressed by 32-bit byte offsets within a pair's table (adp_issue)
  if (adp_max_bnd(n_segs, n_i64) >= (size_t(1) << 22))
    return set_error(PLATO_AGG_EINVAL, "boundary table needs >= 2^22 rows (too many segments / int64 entries)");
  const AdpWs w = adp_ws(n_pairs, with_xx, n_i64, n_flat, n_segs);
  char* ws = static_cast<char*>(d_workspace);
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
  a.ngroups = uint32_t((a.nsteps + 7) / 8);
  a.max_bnd = uint32_t(adp_max_bnd(n_segs, n_i64));
  a.lr = lr;
  a.inv_lr = 1.0 / double(lr);
  a.ws = reinterpret_cast<float*>(ws + w.chains);
  a.desc = reinterpret_cast<AdpDesc*>(ws + w.desc);
  a.bnd_at = reinterpret_cast<uint32_t*>(ws + w.bnd_at);
  a.n_bnd = a.bnd_at + a.max_bnd;
  a.cnt = reinterpret_cast<uint32_t*>(ws + w.cnt);
  a.bnd = reinterpret_cast<float*>(ws + w.bnd);
  a.xb = reinterpret_cast<const float*>(ws + w.xb);
  a.bsrc = reinterpret_cast<uint32_t*>(ws + w.bsrc);
  a.n_i64 = n_i64;
  a.n_f32 = n_f32;
  a.n_pairs = n_pairs;
  a.with_xx = with_xx;
  if (a.nsteps) {
    if (!(flags & PLATO_AGG_FEDADP_TABLES_READY)) {  // the layout-only tables (descriptors, rows, sources)
      hipLaunchKernelGGL(fedadp_desc_kernel, dim3((2 * a.ngroups + 255) / 256), dim3(256), 0, stream, a);
      if (int rc = check_launch("fedadp_desc launch")) return rc;
      hipLaunchKernelGGL(fedadp_rows_kernel, dim3((2 * a.ngroups + 255) / 256), dim3(256), 0, stream, a);
      if (int rc = check_launch("fedadp_rows launch")) return rc;
      hipLaunchKernelGGL(fedadp_bndsrc_kernel, dim3(a.max_bnd), dim3(256), 0, stream, a);
      if (int rc = check_launch("fedadp_bndsrc launch")) return rc;
    }
    const uint32_t nbx = (a.max_bnd + kBndRows - 1) / kBndRows;
    if (fn.uses_xb) {  // the chain-group-major x (and b) and the boundary table, one launch
      const uint32_t n_spans = uint32_t((a.nsteps * 64 + kPrepSpan - 1) / kPrepSpan);
      hipLaunchKernelGGL(fedadp_prep_boundary_kernel, dim3(n_spans + nbx * uint32_t(n_pairs)), dim3(256), 0, stream,
                         a, reinterpret_cast<float*>(ws + w.xb), n_spans, nbx);
      if (int rc = check_launch("fedadp_prep_boundary launch")) return rc;
    } else {
      hipLaunchKernelGGL(fedadp_boundary_kernel, dim3(nbx, uint32_t(n_pairs)), dim3(256), 0, stream, a);
      if (int rc = check_launch("fedadp_boundary launch")) return rc;
    }
    fn.fn(a, stream);
    if (int rc = check_launch("fedadp_dots launch")) return rc;
  } else {
    (void)hipMemsetAsync(a.ws, 0, (size_t(n_pairs) + (with_xx ? 1 : 0)) * 128 * sizeof(float), stream);
  }
  hipLaunchKernelGGL(fedadp_finish_kernel, dim3(uint32_t(n_pairs + with_xx)), dim3(64), 0, stream, a, d_out_xy,
                     d_out_yy);
  return check_launch("fedadp_finish launch");
}
}  // namespace
