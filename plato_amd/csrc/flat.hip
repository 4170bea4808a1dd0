// flat.hip — the reductions Plato's variant servers run over flattened models,
// in the reference's own float32 evaluation order (bit-exact), for gfx950.
// C ABI: include/plato_agg.h (plato_agg_flatten, plato_agg_sdot_pairs,
// plato_agg_torch_cosine_sum).  CPU restatements: oracle/reductions.c.
//
// * plato_agg_flatten gathers a model (or a client delta) into the flat
//   float32 vector the reference builds: Port concatenates every entry in
//   state_dict order (port_server.py:36-48); FedAdp sorts the entries by
//   name.lower() and divides all but the first by -lr (fedadp_server.py:
//   122-133).  One launch covers K vectors.
// * plato_agg_sdot_pairs is numpy's float32 np.inner / dot on x86-64 AVX-512
//   hosts (OpenBLAS 0.3.29 sdot_k_SKYLAKEX): 64 fma chains (4 x 16 lanes) over
//   the 64-element blocks, folded to 4 x 8, one more 32-block, a fixed
//   horizontal sum, and a float64 tail.  One 64-lane wavefront holds exactly
//   the 64 chains; the other waves of the workgroup stream the two vectors
//   into a double-buffered LDS tile.
// * plato_agg_torch_cosine_sum is the sum in F.cosine_similarity
//   (port_server.py:50): q = (a/|a|)*(b/|b|) summed by PyTorch's CPU
//   two-pass reduction over T OpenMP chunks, each a 4-level cascade of 8-wide
//   vectors x 4 rows of ILP (ATen SumKernel.cpp).  A workgroup computes two
//   clients of one chunk (a staged once in LDS for both; one client per
//   workgroup for chunks past 2^24 elements): the level-0 groups in parallel,
//   the higher levels in order; a second launch combines the T partials.  (The norms |a|, |b| are
//   plato_agg_entry_norms_f32 over the flattened vectors.)
// Compiled with -ffp-contract=off: fmaf where the reference fuses, separate
// roundings everywhere else; divisions are IEEE (correctly rounded).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <string>

#include "common.h"
#include "plato_agg.h"

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;
using plato_agg_internal::side_stream;
using plato_agg_internal::SideStream;

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

// ------------------------------------------------------------------ flatten
struct FlatArgs {
  const void* const* src_f;   // K pointers: fp32 region
  const void* const* src_i;   // K pointers: int64 region (fp32 values in RAW mode)
  const float* base_f;
  const int64_t* base_i;
  const plato_agg_segment* segs;
  uint32_t n_segs;
  uint64_t n_flat;
  float lr;
  float* const* out;
  int mode;
  int K;
};

__device__ __forceinline__ uint32_t find_segment(const plato_agg_segment* segs, uint32_t n, uint64_t p) {
  uint32_t lo = 0, hi = n;  // last segment with flat_offset <= p
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].flat_offset <= p) lo = mid; else hi = mid;
  }
  return lo;
}

constexpr int kFlatPer = 8;  // positions per thread
constexpr int kFlatK = 8;    // clients per workgroup: the baseline is read once for all of them

// The baseline element of a position (what the delta modes subtract), read once per workgroup.
struct FlatBase {
  float f;
  int64_t i;
};

template <int MODE, bool I64>
__device__ __forceinline__ FlatBase flat_base(const FlatArgs& a, uint64_t e) {
  FlatBase b{0.f, 0};
  if (MODE != PLATO_AGG_FLAT_RAW) {
    if (!I64) b.f = a.base_f[e];
    else b.i = a.base_i[e];
  }
  return b;
}

// One element of a segment (the segment's region / flags and the mode are workgroup-uniform).
template <int MODE, bool I64, bool NEG>
__device__ __forceinline__ float flat_value(const FlatArgs& a, const void* xf, const void* xi, uint64_t e,
                                            FlatBase b) {
  float v;
  if (!I64) {
    const float x = __builtin_nontemporal_load(static_cast<const float*>(xf) + e);
    v = MODE == PLATO_AGG_FLAT_RAW ? x : x - b.f;
    if (NEG) v = (-v) / a.lr;
  } else if (MODE == PLATO_AGG_FLAT_RAW) {
    v = static_cast<const float*>(xi)[e];
    if (NEG) v = (-v) / a.lr;
  } else if (MODE == PLATO_AGG_FLAT_CAST_DIFF) {
    // torch.cat casts each int64 entry to fp32 before the subtraction
    v = float(static_cast<const int64_t*>(xi)[e]) - float(b.i);
    if (NEG) v = (-v) / a.lr;
  } else {
    // int64 delta, exact (wrapping) in int64; -delta too, then the cast
    uint64_t d = uint64_t(static_cast<const int64_t*>(xi)[e]) - uint64_t(b.i);
    v = NEG ? float(int64_t(uint64_t(0) - d)) / a.lr : float(int64_t(d));
  }
  return v;
}

template <int MODE, bool I64, bool NEG>
__device__ __forceinline__ void flat_range(const FlatArgs& a, int k0, int nk, uint64_t lo, uint64_t hi,
                                           uint64_t shift) {
  // positions lo..hi-1 of one segment, consecutive positions on consecutive lanes (coalesced),
  // kFlatPer positions per lane loaded before any is stored (loads in flight, not one at a time);
  // the baseline values once, then each of the workgroup's nk clients
  for (uint64_t p0 = lo; p0 < hi; p0 += 256 * kFlatPer) {
    FlatBase b[kFlatPer];
#pragma unroll
    for (int u = 0; u < kFlatPer; ++u) {
      const uint64_t p = p0 + uint64_t(u) * 256 + threadIdx.x;
      b[u] = p < hi ? flat_base<MODE, I64>(a, p - shift) : FlatBase{0.f, 0};
    }
    for (int kk = 0; kk < nk; ++kk) {
      const void* xf = sld(a.src_f, k0 + kk);
      const void* xi = sld(a.src_i, k0 + kk);
      float* out = sld(a.out, k0 + kk);
      float v[kFlatPer];
#pragma unroll
      for (int u = 0; u < kFlatPer; ++u) {
        const uint64_t p = p0 + uint64_t(u) * 256 + threadIdx.x;
        v[u] = p < hi ? flat_value<MODE, I64, NEG>(a, xf, xi, p - shift, b[u]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kFlatPer; ++u) {
        const uint64_t p = p0 + uint64_t(u) * 256 + threadIdx.x;
        if (p < hi) __builtin_nontemporal_store(v[u], out + p);
      }
    }
  }
}

template <int MODE>
__device__ __forceinline__ void flat_block(const FlatArgs& a, int k0, int nk, uint64_t b0, uint64_t b1) {
  // the segments overlapping [b0, b1), one after the other; every branch is workgroup-uniform
  for (uint32_t s = find_segment(a.segs, a.n_segs, b0); s < a.n_segs; ++s) {
    const uint64_t fo = a.segs[s].flat_offset;
    if (fo >= b1) break;
    const uint64_t so = a.segs[s].src_offset, n = a.segs[s].numel;
    const uint32_t region = a.segs[s].region, flags = a.segs[s].flags;
    const uint64_t lo = fo > b0 ? fo : b0, hi = fo + n < b1 ? fo + n : b1;
    if (lo >= hi) continue;
    const uint64_t shift = fo - so;  // position p reads source element p - shift (mod 2^64)
    const bool neg = flags & PLATO_AGG_SEG_NEG_DIV;
    if (region == 0) {
      if (neg) flat_range<MODE, false, true>(a, k0, nk, lo, hi, shift);
      else flat_range<MODE, false, false>(a, k0, nk, lo, hi, shift);
    } else {
      if (neg) flat_range<MODE, true, true>(a, k0, nk, lo, hi, shift);
      else flat_range<MODE, true, false>(a, k0, nk, lo, hi, shift);
    }
  }
}

__global__ __launch_bounds__(256) void flatten_kernel(FlatArgs a) {
  const int k0 = int(blockIdx.y) * kFlatK;
  const int nk = a.K - k0 < kFlatK ? a.K - k0 : kFlatK;
  const uint64_t b0 = uint64_t(blockIdx.x) * (256 * kFlatPer);
  const uint64_t b1 = b0 + 256 * kFlatPer < a.n_flat ? b0 + 256 * kFlatPer : a.n_flat;
  if (a.mode == PLATO_AGG_FLAT_RAW) {
    flat_block<PLATO_AGG_FLAT_RAW>(a, k0, nk, b0, b1);
  } else if (a.mode == PLATO_AGG_FLAT_CAST_DIFF) {
    flat_block<PLATO_AGG_FLAT_CAST_DIFF>(a, k0, nk, b0, b1);
  } else {
    flat_block<PLATO_AGG_FLAT_DELTA>(a, k0, nk, b0, b1);
  }
}

// ------------------------------------------------------------- sdot (SKX)
constexpr int kSdotThreads = 512;        // wave 0: the 64 chains; waves 1..7: the tile stream
constexpr int kSdotTS = 64;              // steps (64-element blocks) per tile
constexpr int kSdotTile = kSdotTS * 64;  // floats per tile per vector

struct SdotArgs {
  const float* const* x;
  const float* const* y;
  uint64_t n;
  float* out_xy;
  float* out_yy;
};

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void sdot_load_tile(const float* x, const float* y, uint64_t base, uint32_t cnt,
                                               float* lx, float* ly, int ptid, int nprod) {
  // cnt is a multiple of 64; base a multiple of kSdotTile (16-byte aligned vectors)
  for (uint32_t e = uint32_t(ptid) * 4; e < cnt; e += uint32_t(nprod) * 4) {
    const f4 vx = *reinterpret_cast<const f4*>(x + base + e);
    const f4 vy = *reinterpret_cast<const f4*>(y + base + e);
    *reinterpret_cast<f4*>(lx + e) = vx;
    *reinterpret_cast<f4*>(ly + e) = vy;
  }
}

__global__ __launch_bounds__(kSdotThreads) void sdot_skx_kernel(SdotArgs a) {
  __shared__ __attribute__((aligned(16))) float tx[2][kSdotTile];
  __shared__ __attribute__((aligned(16))) float ty[2][kSdotTile];
  const int pair = blockIdx.x;
  const float* x = sld(a.x, pair);
  const float* y = sld(a.y, pair);
  const uint64_t n = a.n;
  const uint64_t n1 = n & ~uint64_t(31);
  const uint64_t n64 = n1 & ~uint64_t(63);
  const uint64_t ntiles = (n64 + kSdotTile - 1) / kSdotTile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nprod = kSdotThreads - 64, ptid = tid - 64;
  float axy = 0.f, ayy = 0.f;  // chain `lane` = 16 r + l of the 512-bit accumulators
  if (wave != 0 && ntiles) {
    sdot_load_tile(x, y, 0, uint32_t(n64 < kSdotTile ? n64 : kSdotTile), tx[0], ty[0], ptid, nprod);
  }
  __syncthreads();
  for (uint64_t t = 0; t < ntiles; ++t) {
    const int cur = int(t & 1);
    if (wave != 0) {
      if (t + 1 < ntiles) {
        const uint64_t base = (t + 1) * kSdotTile;
        const uint64_t left = n64 - base;
        sdot_load_tile(x, y, base, uint32_t(left < kSdotTile ? left : kSdotTile), tx[cur ^ 1], ty[cur ^ 1],
                       ptid, nprod);
      }
    } else {
      const uint64_t base = t * kSdotTile;
      const uint64_t left = n64 - base;
      const int steps = int((left < kSdotTile ? left : kSdotTile) / 64);
      const float* lx = tx[cur];
      const float* ly = ty[cur];
      for (int s = 0; s < steps; ++s) {
        const float xv = lx[s * 64 + lane];
        const float yv = ly[s * 64 + lane];
        axy = __builtin_fmaf(xv, yv, axy);
        ayy = __builtin_fmaf(yv, yv, ayy);
      }
    }
    __syncthreads();
  }
  if (wave != 0) return;
  // fold the 4 x 16 accumulators to 4 x 8: a[r][l] = acc[r][l] + acc[r][l+8]
  const float hxy = __shfl(axy, (lane + 8) & 63, 64);
  const float hyy = __shfl(ayy, (lane + 8) & 63, 64);
  const int r = lane >> 4, l = lane & 15;
  float bxy = 0.f, byy = 0.f;
  if (l < 8) {
    bxy = axy + hxy;
    byy = ayy + hyy;
    if (n1 > n64) {  // one 32-element block left: 4 x 8 lanes
      const float xv = x[n64 + 8 * r + l];
      const float yv = y[n64 + 8 * r + l];
      bxy = __builtin_fmaf(xv, yv, bxy);
      byy = __builtin_fmaf(yv, yv, byy);
    }
  }
  // s[l] = ((a0 + a1) + a2) + a3 over r, then h[l] = s[l] + s[l+4], (h0 + h1) + (h2 + h3)
  const float xy1 = __shfl(bxy, 16 + l, 64), xy2 = __shfl(bxy, 32 + l, 64), xy3 = __shfl(bxy, 48 + l, 64);
  const float yy1 = __shfl(byy, 16 + l, 64), yy2 = __shfl(byy, 32 + l, 64), yy3 = __shfl(byy, 48 + l, 64);
  const float sxy = ((bxy + xy1) + xy2) + xy3;
  const float syy = ((byy + yy1) + yy2) + yy3;
  const float sxy4 = __shfl(sxy, (lane + 4) & 63, 64);
  const float syy4 = __shfl(syy, (lane + 4) & 63, 64);
  const float hx = sxy + sxy4, hy = syy + syy4;  // valid on lanes 0..3
  const float hx1 = __shfl(hx, 1, 64), hx2 = __shfl(hx, 2, 64), hx3 = __shfl(hx, 3, 64);
  const float hy1 = __shfl(hy, 1, 64), hy2 = __shfl(hy, 2, 64), hy3 = __shfl(hy, 3, 64);
  if (lane != 0) return;
  double kxy = 0.0, kyy = 0.0;
  if (n1) {
    kxy = double((hx + hx1) + (hx2 + hx3));
    kyy = double((hy + hy1) + (hy2 + hy3));
  }
  double txy = 0.0, tyy = 0.0;  // the scalar tail in float64, products rounded to fp32 first
  for (uint64_t i = n1; i < n; ++i) {
    const float xv = x[i], yv = y[i];
    txy += double(yv * xv);
    tyy += double(yv * yv);
  }
  a.out_xy[pair] = float(txy + kxy);
  if (a.out_yy) a.out_yy[pair] = float(tyy + kyy);
}

// ------------------------------------------- sdot, shared x, chains split
// FedAdp's dots all share one vector (x = the flattened global gradient,
// fedadp_server.py:95-99): np.inner(g, loc_k) and loc_k . loc_k for every
// client, g . g once.  sdot_skx_kernel above gives each pair one workgroup,
// and its tile stream keeps ~32 KiB in flight per CU, so 129 pairs of 45 MB
// vectors ran at ~21 GB/s per CU (4.2 ms for 128 ResNet-18 clients).
// Here the 64 chains of sdot_k_SKYLAKEX (chain j sums positions j mod 64,
// serially over the 64-element blocks) are split over 64 / kC workgroups, and
// each workgroup runs kC chains for kP pairs that share x: its chain wave holds
// kP x kC chains (every lane useful), x is read once per workgroup instead of
// once per pair, and kW producer waves keep kPS - 1 stages of kS blocks in
// flight by LDS-DMA (global_load_lds_dwordx4, no VGPRs) — ~100 KiB per CU.
// Measured: 129 pairs of ResNet-18-sized vectors 4.23 -> 2.10 ms; the
// default keeps a pair group's chain groups on one XCD, since with the groups on
// different XCDs every 128-byte line was fetched twice (PMC: 12.2 vs 6.2 GB).
// The chains' partial sums go to a workspace; sdot_finish_kernel applies the
// fold, the 32-element block, the horizontal sum and the float64 tail exactly
// as sdot_skx_kernel does, so results are bitwise identical to it.
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;

template <int N>
__device__ __forceinline__ void sd_wait_vmcnt() {  // s_waitcnt vmcnt(N) only (gfx9 encoding)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// One v_fma_f32 (the same instruction __builtin_fmaf selects).  Opaque to the
// SLP vectorizer, which otherwise packs the x.y and y.y chains into a
// v_pk_fma_f32 fed by two v_mov per step (~30 cycles per step measured).
__device__ __forceinline__ float chain_fma(float a, float b, float c) {
  asm("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
  return c;
}

struct SdotSArgs {
  const float* x;
  const float* const* y;
  uint64_t nsteps;  // whole 64-element blocks
  float* ws;        // [n_pairs + with_xx][128]: chain partials of x.y, then of y.y
  int n_pairs;
  int with_xx;      // also x.x, as a virtual pair (x, x) after the last pair
};

template <int kP, int kC, int kS>
struct SdotShape {
  static constexpr int kV = 1 + kP;                // vectors per stage: x, y_0 .. y_{kP-1}
  static constexpr int kRegion = kS * kC + kC;     // floats per vector region; the pad puts
                                                   // y_p's lanes in distinct banks
  static constexpr int kStage = kV * kRegion;
  static constexpr int kStepsPerLd = 256 / kC;     // blocks per 1 KiB LDS-DMA (64 lanes x 16 B)
  static constexpr int kLdPerVec = kS / kStepsPerLd;
  static constexpr int kLd = kV * kLdPerVec;       // LDS-DMAs per stage
  static constexpr int kL = kP * kC;              // chain lanes used (the rest duplicate them)
  static_assert(kL == 64 || kL == 32 || kL == 16, "one chain wave: kP pairs x kC chains");
  static_assert(kS % kStepsPerLd == 0 && kS % 16 == 0, "stage shape");
};

template <int kP, int kC, int kS, int kPS, int kW, bool kXcd = false, bool kXX = false>
__global__ __launch_bounds__(64 * (1 + kW)) void sdot_shared_kernel(SdotSArgs a) {
  using Sh = SdotShape<kP, kC, kS>;
  constexpr int kPer = Sh::kLd / kW;  // LDS-DMAs per producer wave per stage
  static_assert(Sh::kLd % kW == 0, "stage must split evenly over the producer waves");
  static_assert((kPS - 2) * kPer < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) float ring[kPS * Sh::kStage];
  constexpr int kGroups = 64 / kC;
  // kXcd: workgroups are dealt to the 8 XCDs round-robin by blockIdx, so the kGroups chain
  // groups of a pair group get ids that agree mod 8 — one XCD, one L2 — and each 128-byte
  // line of y (and x) is fetched from HBM once for all of them, not once per XCD
  int pg, cg;
  if (kXcd) {
    const int b = int(blockIdx.x), lo = b & 7, hi = b / (8 * kGroups);
    cg = (b / 8) % kGroups;
    pg = hi * 8 + lo;
    if (pg * kP >= a.n_pairs) return;  // padding workgroup (before any barrier)
  } else {
    pg = int(blockIdx.x) / kGroups;
    cg = int(blockIdx.x) % kGroups;
  }
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const uint64_t nsteps = a.nsteps;
  const uint64_t nst = (nsteps + kS - 1) / kS;
  if (wave > 0) {  // producer
    const int w = wave - 1;
    const float* src[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int v = (w + kW * r) / Sh::kLdPerVec;
      const int pair = pg * kP + v - 1;
      src[r] = v == 0 ? a.x : sld(a.y, pair < a.n_pairs ? pair : a.n_pairs - 1);
    }
    const uint32_t lofs = uint32_t(cg * kC + (lane % (kC / 4)) * 4);  // float offset inside a block
    const int lstep = lane / (kC / 4);
    auto issue = [&](uint64_t st, int slot) {
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const int q = w + kW * r;
        const int v = q / Sh::kLdPerVec, j = q % Sh::kLdPerVec;
        uint64_t step = st * kS + uint64_t(j * Sh::kStepsPerLd + lstep);
        step = step < nsteps ? step : nsteps - 1;  // a ragged last stage re-reads a valid block
        float* dst = ring + slot * Sh::kStage + v * Sh::kRegion + j * Sh::kStepsPerLd * kC;
        __builtin_amdgcn_global_load_lds((gvoid*)(src[r] + step * 64 + lofs), (lvoid*)dst, 16, 0, 0);
      }
    };
#pragma unroll
    for (int p = 0; p < kPS - 1; ++p)
      if (uint64_t(p) < nst) issue(uint64_t(p), p);
    int slot = 0;  // t mod kPS
    for (uint64_t t = 0; t < nst; ++t, slot = slot + 1 == kPS ? 0 : slot + 1) {
      if (t + kPS - 2 < nst) sd_wait_vmcnt<(kPS - 2) * kPer>();  // stage t landed
      else sd_wait_vmcnt<0>();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __builtin_amdgcn_s_barrier();  // stage t published; the chain wave is done with stage t - 1
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (t + kPS - 1 < nst) issue(t + kPS - 1, slot == 0 ? kPS - 1 : slot - 1);  // into stage t - 1's slot
    }
    sd_wait_vmcnt<0>();
    return;
  }
  // chain wave: lane = (pair p of the group, chain c of the workgroup's kC); lanes >= kL
  // duplicate lane mod kL (fewer chains per workgroup = more workgroups = more CUs streaming:
  // a CU's LDS-DMA stream tops out near 12 B/clk, MI355X_MICROARCH.md)
  __builtin_amdgcn_s_setprio(3);
  const int p = (lane % Sh::kL) / kC, c = lane % kC;
  float axy = 0.f, ayy = 0.f, axx = 0.f;  // kXX: every chain wave also runs x.x (x is in LDS anyway)
  int slot = 0;
  for (uint64_t t = 0; t < nst; ++t, slot = slot + 1 == kPS ? 0 : slot + 1) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const float* X = ring + slot * Sh::kStage + c;
    const float* Y = ring + slot * Sh::kStage + (1 + p) * Sh::kRegion + c;
    const uint64_t left = nsteps - t * kS;
    if (left >= uint64_t(kS)) {
      // blocks of 16 steps, the next block's reads in flight
      float xv[16], yv[16], xn[16], yn[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        xv[q] = X[q * kC];
        yv[q] = Y[q * kC];
      }
#pragma unroll
      for (int blk = 0; blk < kS / 16; ++blk) {
        if (blk + 1 < kS / 16) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            xn[q] = X[(16 * (blk + 1) + q) * kC];
            yn[q] = Y[(16 * (blk + 1) + q) * kC];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          axy = chain_fma(xv[q], yv[q], axy);
          ayy = chain_fma(yv[q], yv[q], ayy);
          if (kXX) axx = chain_fma(xv[q], xv[q], axx);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          xv[q] = xn[q];
          yv[q] = yn[q];
        }
      }
    } else {
      for (int s = 0; s < int(left); ++s) {
        const float xs = X[s * kC], ys = Y[s * kC];
        axy = chain_fma(xs, ys, axy);
        ayy = chain_fma(ys, ys, ayy);
        if (kXX) axx = chain_fma(xs, xs, axx);
      }
    }
  }
  const int pair = pg * kP + p, chain = cg * kC + c;
  if (pair < a.n_pairs && lane < Sh::kL) {
    a.ws[uint64_t(pair) * 128 + chain] = axy;
    a.ws[uint64_t(pair) * 128 + 64 + chain] = ayy;
  }
  if (kXX && pg == 0 && lane < kC) {  // the virtual pair (x, x): its x.y and y.y chains are both x.x
    a.ws[uint64_t(a.n_pairs) * 128 + chain] = axx;
    a.ws[uint64_t(a.n_pairs) * 128 + 64 + chain] = axx;
  }
}

// The rest of sdot_k_SKYLAKEX per pair from the 64 chain sums (sdot_skx_kernel's epilogue).
__global__ __launch_bounds__(64) void sdot_finish_kernel(const float* x, const float* const* ys, int n_pairs,
                                                         uint64_t n, const float* ws, float* out_xy, float* out_yy) {
  const int pair = blockIdx.x, lane = threadIdx.x & 63;
  const float* y = pair < n_pairs ? sld(ys, pair) : x;  // pair n_pairs: the virtual (x, x)
  const uint64_t n1 = n & ~uint64_t(31);
  const uint64_t n64 = n1 & ~uint64_t(63);
  const float axy = ws[uint64_t(pair) * 128 + lane];
  const float ayy = ws[uint64_t(pair) * 128 + 64 + lane];
  const float hxy = __shfl(axy, (lane + 8) & 63, 64);
  const float hyy = __shfl(ayy, (lane + 8) & 63, 64);
  const int r = lane >> 4, l = lane & 15;
  float bxy = 0.f, byy = 0.f;
  if (l < 8) {
    bxy = axy + hxy;
    byy = ayy + hyy;
    if (n1 > n64) {
      const float xv = x[n64 + 8 * r + l];
      const float yv = y[n64 + 8 * r + l];
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
  if (lane != 0) return;
  double kxy = 0.0, kyy = 0.0;
  if (n1) {
    kxy = double((hx + hx1) + (hx2 + hx3));
    kyy = double((hy + hy1) + (hy2 + hy3));
  }
  double txy = 0.0, tyy = 0.0;
  for (uint64_t i = n1; i < n; ++i) {
    const float xv = x[i], yv = y[i];
    txy += double(yv * xv);
    tyy += double(yv * yv);
  }
  out_xy[pair] = float(txy + kxy);
  if (out_yy) out_yy[pair] = float(tyy + kyy);
}

using SdotSFn = void (*)(const SdotSArgs&, hipStream_t);
template <int kP, int kC, int kS, int kPS, int kW, bool kXcd = false>
void launch_sdot_shared(const SdotSArgs& a, hipStream_t st) {
  uint32_t pgs = uint32_t((a.n_pairs + kP - 1) / kP);
  if (kXcd) pgs = (pgs + 7) / 8 * 8;
  const uint32_t groups = pgs * uint32_t(64 / kC);
  if (a.with_xx)
    hipLaunchKernelGGL((sdot_shared_kernel<kP, kC, kS, kPS, kW, kXcd, true>), dim3(groups), dim3(64 * (1 + kW)), 0,
                       st, a);
  else
    hipLaunchKernelGGL((sdot_shared_kernel<kP, kC, kS, kPS, kW, kXcd, false>), dim3(groups), dim3(64 * (1 + kW)), 0,
                       st, a);
}
// pairs per workgroup x chains per workgroup x blocks per stage x stages x producer waves.  The
// round-2 sweep (12 shapes, profiles/r02*_sdot*) is in DESIGN.md §12; the tuning library keeps the
// three size-picked defaults and variant 0's shape without the XCD grouping.
#ifdef PLATO_AGG_TUNE  // libplato_agg_tune.so
const SdotSFn kSdotSVariants[] = {
    &launch_sdot_shared<4, 16, 64, 6, 4, true>,  // 0: 64 B of each block per vector, a pair group on one XCD
    &launch_sdot_shared<2, 16, 64, 6, 4, true>,  // 1: half chain waves (twice the workgroups)
    &launch_sdot_shared<1, 16, 64, 4, 2, true>,  // 2: quarter chain waves, 2 producers
    &launch_sdot_shared<4, 16, 64, 6, 4>,        // 3: variant 0 without the XCD grouping
};
#else  // libplato_agg.so: the three defaults of default_sdot_variant
const SdotSFn kSdotSVariants[] = {
    &launch_sdot_shared<4, 16, 64, 6, 4, true>,
    &launch_sdot_shared<2, 16, 64, 6, 4, true>,
    &launch_sdot_shared<1, 16, 64, 4, 2, true>,
};
#endif
constexpr int kSdotV5 = 0, kSdotV8 = 1, kSdotV11 = 2;
constexpr int kNumSdotSVariants = sizeof(kSdotSVariants) / sizeof(kSdotSVariants[0]);

// The default by size: with x.x folded in, as many workgroups as CUs when the pairs allow it (a CU's
// stream, ~24 GB/s, is what bounds a workgroup): 128 pairs -> 2 pairs x 16 chains per workgroup,
// 64 x 4 = 256 workgroups; otherwise 4 pairs per workgroup.
int default_sdot_variant(int n_pairs, int with_xx) {
  if (with_xx && n_pairs <= 64) return kSdotV11;
  if (with_xx && n_pairs <= 128) return kSdotV8;
  return kSdotV5;
}

int run_sdot_shared(int variant, const float* d_x, const float* const* d_y, int n_pairs, size_t n, int with_xx,
                    float* d_ws, float* d_out_xy, float* d_out_yy, hipStream_t stream) {
  if (variant < 0) variant = default_sdot_variant(n_pairs, with_xx);
  if (variant >= kNumSdotSVariants) return set_error(PLATO_AGG_EINVAL, "bad sdot_shared variant");
  if (n_pairs <= 0) return set_error(PLATO_AGG_EINVAL, "no pairs");
  if (with_xx != 0 && with_xx != 1) return set_error(PLATO_AGG_EINVAL, "with_xx must be 0 or 1");
  if (!d_x || !d_y || !d_out_xy || !d_ws) return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (reinterpret_cast<uintptr_t>(d_x) & 15u) return set_error(PLATO_AGG_EINVAL, "x must be 16-byte aligned");
  const uint64_t nsteps = (uint64_t(n) & ~uint64_t(31)) / 64;
  if (nsteps) {
    SdotSArgs a{d_x, d_y, nsteps, d_ws, n_pairs, with_xx};
    kSdotSVariants[variant](a, stream);
  } else {
    (void)hipMemsetAsync(d_ws, 0, size_t(n_pairs + with_xx) * 128 * sizeof(float), stream);
  }
  hipLaunchKernelGGL(sdot_finish_kernel, dim3(uint32_t(n_pairs + with_xx)), dim3(64), 0, stream, d_x, d_y, n_pairs,
                     uint64_t(n), d_ws, d_out_xy, d_out_yy);
  return check_launch("sdot_shared launch");
}

// ------------------------------------------------- torch cascade sum (cos)
constexpr int kSumThreads = 256;

struct CosArgs {
  const float* av;            // shared vector a (Port: current - previous)
  const float* const* bv;     // K vectors b
  const float* norm_a;        // |a| (1 float)
  const float* norm_b;        // |b_k| (K floats)
  float eps;
  uint64_t n;
  uint64_t chunk;             // elements per thread chunk
  int nt;                     // chunks (<= T)
  int T;                      // torch threads: partial-buffer length
  int single;                 // one pass (n < grain or T == 1): partial[0] is the result
  float* partial;             // [K][T]
  float* out;                 // [K]
};

__device__ __forceinline__ int ceil_log2_u64(uint64_t x) {
  int r = 0;
  while ((uint64_t(1) << r) < x) ++r;
  return r;
}

// q = (a / |a|) * (b / |b|); kScaled: a already divided by its (clamped) norm, once for all K clients
// (plato_agg_scale_by_norm) — the same fp32 quotient, one division per element instead of two
template <bool kScaled>
struct QSrcT {
  const float* a;
  const float* b;
  float na, nb;
  __device__ __forceinline__ float av(float x) const { return kScaled ? x : x / na; }
  __device__ __forceinline__ float operator()(uint64_t p) const { return av(a[p]) * (b[p] / nb); }
};
using QSrc = QSrcT<false>;

// One chunk [b0, b0+size0) -> final_acc of vectorized_inner_sum (size0 >= 8).
// Level-0 groups (L rows of 32 values: 4 ILP rows x 8 lanes) are summed in
// parallel by the workgroup, the higher levels in order by lanes 0..31 of wave 0.
// kDB: common-case level-0 sums into two alternating LDS buffers, one barrier per level-1 group (the
// buffer a pass writes was last read two passes ago, before the barrier between); else one buffer
// and a second barrier after lanes 0..31 have read it
template <class Q, bool kDB = true>
__device__ float chunk_cascade(const Q& q, uint64_t b0, uint64_t size0, float* lds_s0) {
  const uint64_t vec_size = size0 / 8;
  const uint64_t size_ilp = vec_size / 4;
  int lp = ceil_log2_u64(size_ilp) / 4;
  if (lp < 4) lp = 4;
  const uint64_t L = uint64_t(1) << lp;
  const uint64_t G0 = size_ilp / L;  // full level-0 groups
  const uint64_t G1 = G0 / L;        // full level-1 groups
  const int tid = threadIdx.x;
  const int acc_id = tid & 31;       // (ILP row k, lane l) = (acc_id / 8, acc_id % 8)
  const int gslot = tid >> 5;        // 8 level-0 groups per pass
  float acc2 = 0.f, acc3 = 0.f;      // running on lanes 0..31 of wave 0
  auto s0_of = [&](uint64_t g0) {
    float s = 0.f;
    const uint64_t row0 = g0 * L;
    for (uint64_t i = 0; i < L; ++i) s += q(b0 + (row0 + i) * 32 + uint64_t(acc_id));
    return s;
  };
  for (uint64_t g1 = 0; g1 < G1; ++g1) {
    // L == 16 uses 16 x 32 floats of the 64 x 32: with kDB, passes alternate between the halves
    float* const s0 = (kDB && L == 16) ? lds_s0 + (g1 & 1) * 1024 : lds_s0;
    if (L == 16) {
      // the common case (chunks of 2^14 .. 2^22 elements): both of this thread's level-0 groups with
      // all 64 loads issued before the first add (the generic loop waits on each row's loads in turn)
      constexpr int kL = 16, kJ = 16 / (kSumThreads / 32);
      float av[kJ][kL], bv[kJ][kL];
#pragma unroll
      for (int jj = 0; jj < kJ; ++jj) {
        const uint64_t row0 = (g1 * kL + uint64_t(gslot + jj * (kSumThreads / 32))) * kL;
#pragma unroll
        for (int i = 0; i < kL; ++i) {
          const uint64_t p = b0 + (row0 + uint64_t(i)) * 32 + uint64_t(acc_id);
          av[jj][i] = q.a[p];
          bv[jj][i] = q.b[p];
        }
      }
#pragma unroll
      for (int jj = 0; jj < kJ; ++jj) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < kL; ++i) s += q.av(av[jj][i]) * (bv[jj][i] / q.nb);
        s0[uint64_t(gslot + jj * (kSumThreads / 32)) * 32 + uint64_t(acc_id)] = s;
      }
    } else {
      for (uint64_t j = uint64_t(gslot); j < L; j += kSumThreads / 32)
        lds_s0[j * 32 + uint64_t(acc_id)] = s0_of(g1 * L + j);
    }
    __syncthreads();
    if (tid < 32) {
      float s1 = 0.f;
      for (uint64_t j = 0; j < L; ++j) s1 += s0[j * 32 + uint64_t(tid)];
      acc2 += s1;
      if ((g1 + 1) % L == 0) {
        acc3 += acc2;
        acc2 = 0.f;
      }
    }
    if (!kDB || L != 16) __syncthreads();
  }
  if (kDB && L == 16) __syncthreads();  // lanes 0..31 have read the last pass
  // the partial level-1 group: its complete level-0 groups, in order
  const uint64_t rem0 = G0 - G1 * L;
  for (uint64_t j = uint64_t(gslot); j < rem0; j += kSumThreads / 32)
    lds_s0[j * 32 + uint64_t(acc_id)] = s0_of(G1 * L + j);
  __syncthreads();
  float result = 0.f;
  if (tid < 32) {
    float acc1 = 0.f;
    for (uint64_t j = 0; j < rem0; ++j) acc1 += lds_s0[j * 32 + uint64_t(tid)];
    float acc0 = 0.f;  // the rows after the last complete level-0 group
    for (uint64_t i = G0 * L; i < size_ilp; ++i) acc0 += q(b0 + i * 32 + uint64_t(tid));
    float ps = acc0;
    ps += acc1;
    ps += acc2;
    ps += acc3;
    lds_s0[tid] = ps;  // ps[k][l] at k*8 + l
  }
  __syncthreads();
  if (tid == 0) {
    float ps0[8];
    for (int l = 0; l < 8; ++l) ps0[l] = lds_s0[l];
    for (uint64_t v = size_ilp * 4; v < vec_size; ++v)
      for (int l = 0; l < 8; ++l) ps0[l] += q(b0 + v * 8 + uint64_t(l));
    for (int k = 1; k < 4; ++k)
      for (int l = 0; l < 8; ++l) ps0[l] += lds_s0[k * 8 + l];
    float final_acc = 0.f;
    for (uint64_t e = vec_size * 8; e < size0; ++e) final_acc += q(b0 + e);
    for (int l = 0; l < 8; ++l) final_acc += ps0[l];
    result = final_acc;
  }
  __syncthreads();
  return result;
}

// chunk_cascade for two clients of one chunk (L = 16, chunks of at most 2^24 elements), 512 threads: each
// half (256 threads) runs one client's cascade exactly as chunk_cascade's common case (the same level-0
// groups per thread, the same sums in the same order), and the shared vector a of each level-1 group is
// loaded once for both into LDS (32 KB, 16 coalesced loads per thread) instead of once per client from L2.
// Barriers are the whole workgroup's: both halves walk the same chunk, so they meet every one.
template <int C, class Q>
__device__ float chunk_cascade2(const Q& q, uint64_t b0, uint64_t size0, float* s0, float* a_lds) {
  constexpr int kL = 16, kH = kSumThreads;  // threads per client
  const uint64_t vec_size = size0 / 8;
  const uint64_t size_ilp = vec_size / 4;
  const uint64_t G0 = size_ilp / kL;  // full level-0 groups
  const uint64_t G1 = G0 / kL;        // full level-1 groups
  const int tid = int(threadIdx.x) & (kH - 1), wtid = int(threadIdx.x);
  const int acc_id = tid & 31, gslot = tid >> 5;
  float acc2 = 0.f, acc3 = 0.f;  // lanes 0..31 of the half's first wave
  for (uint64_t g1 = 0; g1 < G1; ++g1) {
    constexpr int kJ = 16 / (kH / 32), kA = kL * kL * 32 / (C * kH);  // 2 groups, 8192 / (C * 256) a values
    const float* ag = q.a + b0 + g1 * (kL * kL * 32);
    float av[kA], bv[kJ][kL];
#pragma unroll
    for (int j = 0; j < kA; ++j) av[j] = ag[j * C * kH + wtid];
#pragma unroll
    for (int jj = 0; jj < kJ; ++jj) {
      const uint64_t row0 = (g1 * kL + uint64_t(gslot + jj * (kH / 32))) * kL;
#pragma unroll
      for (int i = 0; i < kL; ++i) bv[jj][i] = q.b[b0 + (row0 + uint64_t(i)) * 32 + uint64_t(acc_id)];
    }
#pragma unroll
    for (int j = 0; j < kA; ++j) a_lds[j * C * kH + wtid] = av[j];
    __syncthreads();  // the group's a in LDS (and the previous group's level-1 reads of s0 done)
#pragma unroll
    for (int jj = 0; jj < kJ; ++jj) {
      const int g = gslot + jj * (kH / 32);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < kL; ++i) s += q.av(a_lds[(g * kL + i) * 32 + acc_id]) * (bv[jj][i] / q.nb);
      s0[g * 32 + acc_id] = s;
    }
    __syncthreads();  // s0 complete; every a_lds read done
    if (tid < 32) {
      float s1 = 0.f;
      for (int j = 0; j < kL; ++j) s1 += s0[j * 32 + tid];
      acc2 += s1;
      if ((g1 + 1) % kL == 0) {
        acc3 += acc2;
        acc2 = 0.f;
      }
    }
  }
  // the partial level-1 group and the tails: chunk_cascade's code per half (a from global memory)
  auto s0_of = [&](uint64_t g0) {
    float s = 0.f;
    const uint64_t row0 = g0 * kL;
    for (uint64_t i = 0; i < uint64_t(kL); ++i) s += q(b0 + (row0 + i) * 32 + uint64_t(acc_id));
    return s;
  };
  __syncthreads();  // lanes 0..31 have read the last pass's s0
  const uint64_t rem0 = G0 - G1 * kL;
  for (uint64_t j = uint64_t(gslot); j < rem0; j += kH / 32) s0[j * 32 + uint64_t(acc_id)] = s0_of(G1 * kL + j);
  __syncthreads();
  float result = 0.f;
  if (tid < 32) {
    float acc1 = 0.f;
    for (uint64_t j = 0; j < rem0; ++j) acc1 += s0[j * 32 + uint64_t(tid)];
    float acc0 = 0.f;  // the rows after the last complete level-0 group
    for (uint64_t i = G0 * kL; i < size_ilp; ++i) acc0 += q(b0 + i * 32 + uint64_t(tid));
    float ps = acc0;
    ps += acc1;
    ps += acc2;
    ps += acc3;
    s0[tid] = ps;  // ps[k][l] at k*8 + l
  }
  __syncthreads();
  if (tid == 0) {
    float ps0[8];
    for (int l = 0; l < 8; ++l) ps0[l] = s0[l];
    for (uint64_t v = size_ilp * 4; v < vec_size; ++v)
      for (int l = 0; l < 8; ++l) ps0[l] += q(b0 + v * 8 + uint64_t(l));
    for (int k = 1; k < 4; ++k)
      for (int l = 0; l < 8; ++l) ps0[l] += s0[k * 8 + l];
    float final_acc = 0.f;
    for (uint64_t e = vec_size * 8; e < size0; ++e) final_acc += q(b0 + e);
    for (int l = 0; l < 8; ++l) final_acc += ps0[l];
    result = final_acc;
  }
  return result;
}

// scalar_inner_sum / vectorized_inner_sum of a short array (single thread), W = 8 (n >= 8) or 1 lanes;
// every accumulator index is a compile-time constant (unrolled k, l and level loops), so the 4 x 4 x 8
// cascade stays in registers (the runtime-indexed form spilled 656 bytes per lane to scratch and took
// 28 us for the K cosine combines)
template <int W>
__device__ float small_inner_sum_w(const float* in, int n) {
  const int vec_size = n / W;
  const int size_ilp = vec_size / 4;
  int lp = ceil_log2_u64(uint64_t(size_ilp)) / 4;
  if (lp < 4) lp = 4;
  const int L = 1 << lp;
  float acc[4][4][W];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < W; ++l) acc[j][k][l] = 0.f;
  int i = 0;
  for (; i + L <= size_ilp;) {
    for (int jj = 0; jj < L; ++jj, ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < W; ++l) {
          acc[j][k][l] += acc[j - 1][k][l];
          acc[j - 1][k][l] = 0.f;
        }
      if ((uint64_t(i) & (uint64_t(L - 1) << (j * lp))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
#pragma unroll
  for (int j = 1; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < W; ++l) acc[0][k][l] += acc[j][k][l];
  if constexpr (W == 8) {
    float ps0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) ps0[l] = acc[0][0][l];
    for (int v = size_ilp * 4; v < vec_size; ++v)
#pragma unroll
      for (int l = 0; l < 8; ++l) ps0[l] += in[v * 8 + l];
#pragma unroll
    for (int k = 1; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < 8; ++l) ps0[l] += acc[0][k][l];
    float final_acc = 0.f;
    for (int e = vec_size * 8; e < n; ++e) final_acc += in[e];
#pragma unroll
    for (int l = 0; l < 8; ++l) final_acc += ps0[l];
    return final_acc;
  } else {
    float ps0 = acc[0][0][0];
    for (int v = size_ilp * 4; v < n; ++v) ps0 += in[v];
#pragma unroll
    for (int k = 1; k < 4; ++k) ps0 += acc[0][k][0];
    return ps0;
  }
}

__device__ float small_inner_sum_reg(const float* in, int n) {
  return n >= 8 ? small_inner_sum_w<8>(in, n) : small_inner_sum_w<1>(in, n);
}

// the same sum with runtime-indexed accumulators: the cascade chunk kernel's rare < 8-element chunk
// (the register form above would raise that streaming kernel's register count, 62 -> 87 VGPRs)
__device__ float small_inner_sum(const float* in, int n) {
  float ps[4][8];
  for (int k = 0; k < 4; ++k)
    for (int l = 0; l < 8; ++l) ps[k][l] = 0.f;
  const int W = n >= 8 ? 8 : 1;
  const int vec_size = n / W;
  const int size_ilp = vec_size / 4;
  int lp = ceil_log2_u64(uint64_t(size_ilp)) / 4;
  if (lp < 4) lp = 4;
  const int L = 1 << lp;
  float acc[4][4][8];
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < 8; ++l) acc[j][k][l] = 0.f;
  int i = 0;
  for (; i + L <= size_ilp;) {
    for (int j = 0; j < L; ++j, ++i)
      for (int k = 0; k < 4; ++k)
        for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
    for (int j = 1; j < 4; ++j) {
      for (int k = 0; k < 4; ++k)
        for (int l = 0; l < W; ++l) {
          acc[j][k][l] += acc[j - 1][k][l];
          acc[j - 1][k][l] = 0.f;
        }
      if ((uint64_t(i) & (uint64_t(L - 1) << (j * lp))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < W; ++l) acc[0][k][l] += in[(i * 4 + k) * W + l];
  for (int j = 1; j < 4; ++j)
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < W; ++l) acc[0][k][l] += acc[j][k][l];
  for (int k = 0; k < 4; ++k)
    for (int l = 0; l < W; ++l) ps[k][l] = acc[0][k][l];
  if (W == 8) {
    for (int v = size_ilp * 4; v < vec_size; ++v)
      for (int l = 0; l < 8; ++l) ps[0][l] += in[v * 8 + l];
    for (int k = 1; k < 4; ++k)
      for (int l = 0; l < 8; ++l) ps[0][l] += ps[k][l];
    float final_acc = 0.f;
    for (int e = vec_size * 8; e < n; ++e) final_acc += in[e];
    for (int l = 0; l < 8; ++l) final_acc += ps[0][l];
    return final_acc;
  }
  for (int v = size_ilp * 4; v < n; ++v) ps[0][0] += in[v];
  for (int k = 1; k < 4; ++k) ps[0][0] += ps[k][0];
  return ps[0][0];
}

template <bool kScaled, bool kDB = true>
__global__ __launch_bounds__(kSumThreads) void cosine_chunks_kernel(CosArgs a) {
  __shared__ float lds_s0[64 * 32];  // L <= 64 level-0 groups of 32 values
  // the K clients of a chunk are consecutive workgroups (dealt over the 8 XCDs together): the XCD L2s
  // serve the chunk of a to them (chunk-major numbering; DESIGN.md §12, np_sumsq)
  const int k = blockIdx.x, t = blockIdx.y;
  const uint64_t b0 = uint64_t(t) * a.chunk;
  if (b0 >= a.n) return;
  const uint64_t e0 = b0 + a.chunk < a.n ? b0 + a.chunk : a.n;
  QSrcT<kScaled> q;
  q.a = a.av;
  q.b = sld(a.bv, k);
  q.na = kScaled ? 1.f : a.norm_a[0];
  q.nb = a.norm_b[k];
  if (q.na < a.eps) q.na = a.eps;  // clamp_min_: NaN stays NaN
  if (q.nb < a.eps) q.nb = a.eps;
  const uint64_t size0 = e0 - b0;
  float r;
  if (size0 >= 8) {
    r = chunk_cascade<QSrcT<kScaled>, kDB>(q, b0, size0, lds_s0);
  } else {
    r = 0.f;
    if (threadIdx.x == 0) {
      float tmp[8];
      for (uint64_t e = 0; e < size0; ++e) tmp[e] = q(b0 + e);
      r = small_inner_sum(tmp, int(size0));
    }
  }
  if (threadIdx.x == 0) a.partial[uint64_t(k) * a.T + t] = 0.f + r;
}

// Two clients of a chunk per 512-thread workgroup sharing the loads of a through LDS (chunk_cascade2);
// chunks of at most 2^24 elements (L = 16).  A missing second client (K odd) recomputes client K - 1 in
// its half without storing it.
template <bool kScaled, int C = 2>
__global__ __launch_bounds__(C * kSumThreads) void cosine_chunks2_kernel(CosArgs a, int K) {
  __shared__ float s0_all[C][16 * 32];
  __shared__ float a_lds[16 * 16 * 32];
  const int half = int(threadIdx.x) / kSumThreads;
  const int k_raw = int(blockIdx.x) * C + half, k = k_raw < K ? k_raw : K - 1;
  const int t = blockIdx.y;
  const uint64_t b0 = uint64_t(t) * a.chunk;
  if (b0 >= a.n) return;  // workgroup-uniform
  const uint64_t e0 = b0 + a.chunk < a.n ? b0 + a.chunk : a.n;
  QSrcT<kScaled> q;
  q.a = a.av;
  q.b = sld(a.bv, k);
  q.na = kScaled ? 1.f : a.norm_a[0];
  q.nb = a.norm_b[k];
  if (q.na < a.eps) q.na = a.eps;  // clamp_min_: NaN stays NaN
  if (q.nb < a.eps) q.nb = a.eps;
  const uint64_t size0 = e0 - b0;
  const int tid = int(threadIdx.x) % kSumThreads;
  float r;
  if (size0 >= 8) {
    r = chunk_cascade2<C>(q, b0, size0, s0_all[half], a_lds);
  } else {
    r = 0.f;
    if (tid == 0) {
      float tmp[8];
      for (uint64_t e = 0; e < size0; ++e) tmp[e] = q(b0 + e);
      r = small_inner_sum(tmp, int(size0));
    }
  }
  if (tid == 0 && k_raw < K) a.partial[uint64_t(k) * a.T + t] = 0.f + r;
}

// a / max(|a|, eps) (F.cosine_similarity's x1 / x1_norm after clamp_min_), once for the K sums
__global__ __launch_bounds__(256) void scale_by_norm_kernel(const float* a, uint64_t n, const float* norm, float eps,
                                                            float* out) {
  float na = norm[0];
  if (na < eps) na = eps;  // clamp_min_: NaN stays NaN
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) out[i] = a[i] / na;
}

__global__ void cosine_combine_kernel(CosArgs a, int K) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float* buf = a.partial + uint64_t(k) * a.T;
  if (a.single) {
    a.out[k] = buf[0];  // one pass: 0 + inner_sum, already formed
    return;
  }
  for (int t = a.nt; t < a.T; ++t) buf[t] = 0.f;
  a.out[k] = 0.f + small_inner_sum_reg(buf, a.T);
}

// ------------------------------------------------- numpy pairwise sum of squares
// numpy's float32 add.reduce: the inner loop gets at most 8192 elements (the
// ufunc buffer), each loop does out += pairwise_sum(chunk), and pairwise_sum
// (numpy/_core/src/umath/loops_utils.h) is: n < 8 sequential from 0; n <= 128
// eight partial sums r[j] over the multiples of 8, ((r0+r1)+(r2+r3)) +
// ((r4+r5)+(r6+r7)), then the rest; else split at n2 = n/2 - (n/2)%8.
constexpr int kPW = 128;

template <class V>
__device__ float pw_leaf(const V& v, uint64_t off, uint64_t n) {
  if (n < 8) {
    float res = 0.f;
    for (uint64_t i = 0; i < n; ++i) res += v(off + i);
    return res;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = v(off + j);
  uint64_t i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += v(off + i + j);
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += v(off + i);
  return res;
}

// The recursion, post-order, on an explicit stack (depth <= 7 for 8192 elements);
// leaf(off, n) gives the value of a leaf (<= kPW elements), visited left to right.
// The stack lives wherever the caller puts it (registers, or LDS for a single lane).
struct PwStack {
  uint32_t* so;
  uint32_t* sn;
  float* sl;
  uint32_t* stage;
};

template <class Leaf>
__device__ float pw_walk(const Leaf& leaf, uint32_t off, uint32_t n, PwStack st) {
  uint32_t* so = st.so;
  uint32_t* sn = st.sn;
  float* sl = st.sl;
  uint32_t* stage = st.stage;
  int sp = 0;
  so[0] = off;
  sn[0] = n;
  stage[0] = 0;
  float ret = 0.f;
  bool have = false;  // `ret` holds the value of the node just finished
  for (;;) {
    if (!have) {
      if (sn[sp] <= uint32_t(kPW)) {
        ret = leaf(so[sp], sn[sp]);
        have = true;
        --sp;
      } else {  // descend into the left half
        uint32_t n2 = sn[sp] / 2;
        n2 -= n2 % 8;
        so[sp + 1] = so[sp];
        sn[sp + 1] = n2;
        stage[sp + 1] = 0;
        stage[sp] = 1;
        ++sp;
        continue;
      }
    }
    if (sp < 0) return ret;
    if (stage[sp] == 1) {  // left done: remember it, descend right
      uint32_t n2 = sn[sp] / 2;
      n2 -= n2 % 8;
      sl[sp] = ret;
      stage[sp] = 2;
      so[sp + 1] = so[sp] + n2;
      sn[sp + 1] = sn[sp] - n2;
      stage[sp + 1] = 0;
      ++sp;
      have = false;
    } else {  // right done: left + right
      ret = sl[sp] + ret;
      --sp;
    }
  }
}

constexpr uint64_t kNpBuf = 8192;

struct SumsqArgs {
  const float* const* x;
  const float* base;
  const plato_agg_chunk* pieces;  // one per entry: (entry, begin, end)
  const uint32_t* first_chunk;    // per piece: index of its first 8192-chunk (prefix sums)
  uint32_t n_pieces;
  uint32_t n_chunks;
  int K;
  float* chunk_sums;              // [K][n_chunks]
  float* out;                     // [K][n_pieces]
};

// One workgroup per (client, 8192-chunk): the chunk's squared deltas are staged in LDS with
// coalesced loads (one pad float per 128, so that leaves starting 128 apart sit in different
// banks).  A full 8192-element chunk is numpy's balanced case: 64 leaves of 128, summed one per
// lane of wave 0, then combined pairwise by a 6-level xor butterfly (a + b == b + a, so every
// level adds exactly the tree's left and right halves).  A shorter chunk (the last one of an
// entry) is walked serially by one lane over the staged values.
__device__ __forceinline__ uint32_t np_pad(uint64_t e) { return uint32_t(e + e / kPW); }

__global__ __launch_bounds__(256) void np_sumsq_chunks_lds_kernel(SumsqArgs a) {
  __shared__ float sq[kNpBuf + kNpBuf / kPW];
  const uint32_t k = blockIdx.x / a.n_chunks, c = blockIdx.x % a.n_chunks;
  uint32_t lo = 0, hi = a.n_pieces;  // the piece holding chunk c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.first_chunk[mid] <= c) lo = mid; else hi = mid;
  }
  const plato_agg_chunk p = a.pieces[lo];
  const uint64_t begin = uint64_t(p.begin) + uint64_t(c - a.first_chunk[lo]) * kNpBuf;
  const uint64_t end = begin + kNpBuf < uint64_t(p.end) ? begin + kNpBuf : uint64_t(p.end);
  const uint32_t n = uint32_t(end - begin);
  const float* x = a.x[k] + begin;
  const float* b = a.base + begin;
  for (uint32_t i0 = 0; i0 < n; i0 += 256 * 8) {  // 16 loads in flight per lane
    float xv[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = i0 + u * 256 + threadIdx.x;
      xv[u] = i < n ? __builtin_nontemporal_load(x + i) : 0.f;
      bv[u] = i < n ? b[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = i0 + u * 256 + threadIdx.x;
      const float d = xv[u] - bv[u];
      if (i < n) sq[np_pad(i)] = d * d;
    }
  }
  __syncthreads();
  const auto v = [&](uint64_t e) { return sq[np_pad(e)]; };
  float* dst = a.chunk_sums + uint64_t(k) * a.n_chunks + c;
  if (n == kNpBuf) {
    if (threadIdx.x < 64) {
      float s = pw_leaf(v, uint64_t(threadIdx.x) * kPW, kPW);
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) s = s + __shfl_xor(s, m);
      if (threadIdx.x == 0) *dst = s;
    }
  } else if (threadIdx.x == 0) {
    uint32_t so[16], sn[16], stage[16];
    float sl[16];
    *dst = pw_walk([&](uint32_t o, uint32_t m) { return pw_leaf(v, o, m); }, 0, n, PwStack{so, sn, sl, stage});
  }
}

// One client per workgroup, latency-shaped: a full chunk's 64 loads per lane (32 of x, 32 of b) go
// out before the first square is staged (one memory round trip per workgroup instead of four), and
// the leaves are summed by 8 lanes each — lane (leaf, j) runs numpy's accumulator r[j] over its 16
// steps, the 8 partials of a leaf combine by xor 1, 2, 4 shuffles (((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
// a + b == b + a), then the 64 leaves by the same butterfly as before; a leaf pitch of 136 floats
// keeps the 64 lanes' reads in 64 banks.  Partial chunks walk as before.
constexpr int kLeafPitch = kPW + 8;
__device__ __forceinline__ uint32_t np_pad8(uint64_t e) { return uint32_t(e + (e / kPW) * 8); }


// Task t of the chunk-major numbering: client t mod K of chunk t / K (the K clients of a chunk are
// consecutive: each XCD's L2 serves the chunk's baseline to its share of them).  Client-major order
// (the K passes over the baseline a whole model apart) measured 1.61 ms against 1.26, all K
// clients of a chunk on one XCD 1.24.
struct NpTask {
  uint32_t k, c, n;
  uint64_t begin;
};
__device__ __forceinline__ NpTask np_task_lane(const SumsqArgs& a, uint64_t t) {  // any t per lane
  NpTask r;
  r.k = uint32_t(t % uint64_t(a.K));
  r.c = uint32_t(t / uint64_t(a.K));
  uint32_t lo = 0, hi = a.n_pieces;  // the piece holding chunk c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.first_chunk[mid] <= r.c) lo = mid; else hi = mid;
  }
  const plato_agg_chunk p = a.pieces[lo];
  r.begin = uint64_t(p.begin) + uint64_t(r.c - a.first_chunk[lo]) * kNpBuf;
  const uint64_t end = r.begin + kNpBuf < uint64_t(p.end) ? r.begin + kNpBuf : uint64_t(p.end);
  r.n = uint32_t(end - r.begin);
  return r;
}
__device__ __forceinline__ NpTask np_task(const SumsqArgs& a, uint64_t t) {  // t workgroup-uniform
  NpTask r = np_task_lane(a, t);
  // workgroup-uniform: keep the task in SGPRs (scalar bases for the loads)
  r.k = __builtin_amdgcn_readfirstlane(r.k);
  r.c = __builtin_amdgcn_readfirstlane(r.c);
  r.n = __builtin_amdgcn_readfirstlane(r.n);
  r.begin = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(r.begin >> 32))) << 32) |
            __builtin_amdgcn_readfirstlane(uint32_t(r.begin));
  return r;
}

// kT threads per workgroup, kNpBuf / kT elements per lane: element q * kT + tid.
// kB = false: delta arenas (a null baseline; the rows already hold x - b, so b = 0: x - 0 is x bit for bit)
template <int kT, bool kB = true>
__device__ __forceinline__ void np_load(const SumsqArgs& a, const NpTask& t, float (&xv)[kNpBuf / kT],
                                        float (&bv)[kNpBuf / kT]) {
  const float* x = a.x[t.k] + t.begin;
  const float* b = kB ? a.base + t.begin : nullptr;
#pragma unroll
  for (int q = 0; q < int(kNpBuf / kT); ++q) {
    const uint32_t i = uint32_t(q * kT) + threadIdx.x;
    xv[q] = i < t.n ? __builtin_nontemporal_load(x + i) : 0.f;
    bv[q] = (kB && i < t.n) ? b[i] : 0.f;
  }
}

// A partial chunk (an entry's last), walked by one lane over the staged squares.
__device__ __forceinline__ float np_partial(const float* sq, uint32_t n) {
  const auto v = [&](uint64_t e) { return sq[np_pad8(e)]; };
  uint32_t so[16], sn[16], stage[16];
  float sl[16];
  return pw_walk([&](uint32_t o, uint32_t m) { return pw_leaf(v, o, m); }, 0, n, PwStack{so, sn, sl, stage});
}

// The same sum with the leaves in parallel (every thread of the workgroup calls it): lane 0 lists the
// recursion's leaves left to right (offsets and lengths only), the threads sum one leaf each (pw_leaf,
// as np_partial), and lane 0 walks the recursion again adding the leaf values in post-order — the same
// additions in the same order as np_partial, which ran every leaf's ~128 dependent adds on one lane
// (an entry's partial last chunk: up to 8,191 of them; 0.33 of the 1.15 ms Polaris launch,
// profiles/r05zz_kernel_stats.csv).  Leaves hold more than 56 elements unless the chunk is shorter, so a
// chunk below 8,192 has fewer than 150.  Returns the sum on lane 0.
constexpr int kNpMaxLeaves = 256;
__device__ float np_partial_par(const float* sq, uint32_t n) {
  __shared__ uint32_t leaf_off[kNpMaxLeaves], leaf_n[kNpMaxLeaves];
  __shared__ float leaf_val[kNpMaxLeaves];
  __shared__ int n_leaves;
  const int tid = int(threadIdx.x);
  if (tid == 0) {
    int cnt = 0;
    uint32_t so[16], sn[16], stage[16];
    float sl[16];
    pw_walk([&](uint32_t o, uint32_t m) {
      leaf_off[cnt] = o;
      leaf_n[cnt] = m;
      ++cnt;
      return 0.f;
    }, 0, n, PwStack{so, sn, sl, stage});
    n_leaves = cnt;
  }
  __syncthreads();
  const int nl = n_leaves;
  const auto v = [&](uint64_t e) { return sq[np_pad8(e)]; };
  for (int i = tid; i < nl; i += int(blockDim.x)) leaf_val[i] = pw_leaf(v, leaf_off[i], leaf_n[i]);
  __syncthreads();
  float r = 0.f;
  if (tid == 0) {
    int idx = 0;
    uint32_t so[16], sn[16], stage[16];
    float sl[16];
    r = pw_walk([&](uint32_t, uint32_t) { return leaf_val[idx++]; }, 0, n, PwStack{so, sn, sl, stage});
  }
  return r;
}

// The chunk's numpy sum of squares from this lane's values: squares staged in LDS, 64 leaves x 8
// accumulators (numpy's r[0..7] over 16 steps), the 8 partials of a leaf by xor 1, 2, 4 shuffles,
// the 64 leaves by a 6-level butterfly; a partial chunk walked by lane 0.  Ends with a barrier
// (the next chunk may restage sq).
template <int kT, bool kParLeaves = false>
__device__ __forceinline__ void np_chunk(const SumsqArgs& a, const NpTask& t, const float (&xv)[kNpBuf / kT],
                                         const float (&bv)[kNpBuf / kT], float* sq, float* leaf_sum) {
  const int tid = int(threadIdx.x);
#pragma unroll
  for (int q = 0; q < int(kNpBuf / kT); ++q) {
    const uint32_t i = uint32_t(q * kT + tid);
    const float d = xv[q] - bv[q];
    if (i < t.n) sq[np_pad8(i)] = d * d;
  }
  __syncthreads();
  float* dst = a.chunk_sums + uint64_t(t.k) * a.n_chunks + t.c;
  if (t.n == kNpBuf) {
    // 64 leaves x 8 accumulators = 512 lanes: 512 / kT passes (kT = 1,024: waves 8-15 idle)
#pragma unroll
    for (int pass = 0; pass < (512 + kT - 1) / kT; ++pass) {
      const int slot = pass * kT + tid, leaf = slot >> 3, j = slot & 7;
      if (kT > 512 && slot >= 512) break;  // wave-uniform
      const float* l = sq + leaf * kLeafPitch + j;
      float r = l[0];
#pragma unroll
      for (int i = 8; i < kPW; i += 8) r += l[i];
      r = r + __shfl_xor(r, 1);
      r = r + __shfl_xor(r, 2);
      r = r + __shfl_xor(r, 4);
      if (j == 0) leaf_sum[leaf] = r;
    }
    __syncthreads();
    if (tid < 64) {
      float s = leaf_sum[tid];
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) s = s + __shfl_xor(s, m);
      if (tid == 0) *dst = s;
    }
  } else {  // workgroup-uniform
    const float r = kParLeaves ? np_partial_par(sq, t.n) : (tid == 0 ? np_partial(sq, t.n) : 0.f);
    if (tid == 0) *dst = r;
  }
  __syncthreads();
}

// One workgroup per task, a full chunk's loads (2 x 8,192 / kT per lane) out before the first square
// is staged.
// kProbe (timing probes, wrong results by design, never a default): 1 no baseline loads (b = 0),
// 2 no LDS staging or leaf sums (a lane's own squares summed in registers).
template <int kT, int kProbe = 0>
__global__ __launch_bounds__(kT) void np_sumsq_chunks_v2_kernel(SumsqArgs a) {
  __shared__ float sq[kNpBuf / kPW * kLeafPitch];
  __shared__ float leaf_sum[kNpBuf / kPW];
  const NpTask t = np_task(a, blockIdx.x);
  constexpr int kQ = int(kNpBuf / kT);
  float xv[kQ], bv[kQ];
  if (kProbe == 1) {
    const float* x = a.x[t.k] + t.begin;
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const uint32_t i = uint32_t(q * kT) + threadIdx.x;
      xv[q] = i < t.n ? __builtin_nontemporal_load(x + i) : 0.f;
      bv[q] = 0.f;
    }
  } else {
    np_load<kT>(a, t, xv, bv);
  }
  if (kProbe == 2) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kQ; ++q) r += (xv[q] - bv[q]) * (xv[q] - bv[q]);
    if (r == 12345.f) a.chunk_sums[blockIdx.x] = r;  // keeps the loads; practically never stores
    return;
  }
  np_chunk<kT>(a, t, xv, bv, sq, leaf_sum);
}

// Full chunks staged in two halves (round 4): 32 leaves' squares at a time, so the LDS per workgroup
// halves (17.4 KB) and more workgroups share a CU; same leaves, same order.  Partial chunks (an entry's
// last) take np_sumsq_tail_kernel.
__global__ __launch_bounds__(256) void np_sumsq_half_kernel(SumsqArgs a) {
  __shared__ float sq[kNpBuf / kPW / 2 * kLeafPitch];
  __shared__ float leaf_sum[kNpBuf / kPW];
  const NpTask t = np_task(a, blockIdx.x);
  if (t.n != kNpBuf) return;  // workgroup-uniform
  constexpr int kQ = int(kNpBuf / 256), kHalfQ = kQ / 2;
  float xv[kQ], bv[kQ];
  np_load<256>(a, t, xv, bv);
  const int tid = int(threadIdx.x), leaf = tid >> 3, j = tid & 7;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();  // the first half's leaf reads are done
#pragma unroll
    for (int q = 0; q < kHalfQ; ++q) {
      const uint32_t i = uint32_t(q * 256 + tid);  // element h * 4096 + i
      const float d = xv[h * kHalfQ + q] - bv[h * kHalfQ + q];
      sq[np_pad8(i)] = d * d;
    }
    __syncthreads();
    // 32 leaves x 8 accumulators = the 256 threads
    const float* l = sq + leaf * kLeafPitch + j;
    float r = l[0];
#pragma unroll
    for (int i = 8; i < kPW; i += 8) r += l[i];
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (j == 0) leaf_sum[h * 32 + leaf] = r;
  }
  __syncthreads();
  if (tid < 64) {
    float s = leaf_sum[tid];
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) s = s + __shfl_xor(s, m);
    if (tid == 0) a.chunk_sums[uint64_t(t.k) * a.n_chunks + t.c] = s;
  }
}

// np_sumsq_half_kernel with 16-byte loads and stores: lane tid holds elements q * 1,024 + 4 tid .. + 3
// (q < 8) of the chunk, x read non-temporally, and stages its 4 squares with one ds_write_b128 (4
// consecutive elements never cross a 128-element leaf, and the padded layout keeps them 16-byte
// aligned).  A quarter of the load and LDS-write instructions of the dword form; the same leaves, the
// same accumulators, the same order.
typedef __attribute__((address_space(1))) const f4 gcf4;
template <bool kB = true>
__global__ __launch_bounds__(256) void np_sumsq_half4_kernel(SumsqArgs a) {
  __shared__ __attribute__((aligned(16))) float sq[kNpBuf / kPW / 2 * kLeafPitch];
  __shared__ float leaf_sum[kNpBuf / kPW];
  const NpTask t = np_task(a, blockIdx.x);
  if (t.n != kNpBuf) return;  // workgroup-uniform
  constexpr int kQ = int(kNpBuf / 1024), kHalfQ = kQ / 2;
  const int tid = int(threadIdx.x);
  f4 xv[kQ], bv[kQ];
  const gcf4* x = (const gcf4*)(a.x[t.k] + t.begin) + tid;
  const gcf4* b = kB ? (const gcf4*)(a.base + t.begin) + tid : nullptr;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    xv[q] = __builtin_nontemporal_load(x + q * 256);
    bv[q] = kB ? b[q * 256] : f4{0.f, 0.f, 0.f, 0.f};
  }
  const int leaf = tid >> 3, j = tid & 7;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();  // the first half's leaf reads are done
#pragma unroll
    for (int q = 0; q < kHalfQ; ++q) {
      const uint32_t i = uint32_t(q * 1024 + 4 * tid);  // element h * 4096 + i
      const f4 d = xv[h * kHalfQ + q] - bv[h * kHalfQ + q];
      *reinterpret_cast<f4*>(sq + np_pad8(i)) = d * d;
    }
    __syncthreads();
    // 32 leaves x 8 accumulators = the 256 threads
    const float* l = sq + leaf * kLeafPitch + j;
    float r = l[0];
#pragma unroll
    for (int i = 8; i < kPW; i += 8) r += l[i];
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (j == 0) leaf_sum[h * 32 + leaf] = r;
  }
  __syncthreads();
  if (tid < 64) {
    float s = leaf_sum[tid];
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) s = s + __shfl_xor(s, m);
    if (tid == 0) a.chunk_sums[uint64_t(t.k) * a.n_chunks + t.c] = s;
  }
}

// np_sumsq_half4_kernel for C clients of one chunk: the baseline's 16-byte loads are issued once for
// all of them (the L2-served b re-reads take as many of a CU's in-flight read slots as the client
// bytes), the clients' squares staged and summed one after the other through the same
// half-chunk buffer.  A ragged last group (K mod C) loads and stores only its own clients.
template <int C, bool kFirstThenRest = false, bool kB = true>
__global__ __launch_bounds__(256) void np_sumsq_half4xc_kernel(SumsqArgs a) {
  __shared__ __attribute__((aligned(16))) float sq[kNpBuf / kPW / 2 * kLeafPitch];
  __shared__ float leaf_sum[C][kNpBuf / kPW];
  const uint32_t groups = (uint32_t(a.K) + C - 1) / C;
  const NpTask t = np_task(a, uint64_t(blockIdx.x / groups) * uint64_t(a.K) + (blockIdx.x % groups) * C);
  if (t.n != kNpBuf) return;  // workgroup-uniform
  const int nc = a.K - int(t.k) < C ? a.K - int(t.k) : C;  // clients in this group
  constexpr int kQ = int(kNpBuf / 1024), kHalfQ = kQ / 2;
  const int tid = int(threadIdx.x);
  f4 xv[C][kQ], bv[kQ];
  const gcf4* b = kB ? (const gcf4*)(a.base + t.begin) + tid : nullptr;
  if constexpr (kFirstThenRest) {  // the first client and b, then the others: client 0's squares can be
                                   // staged while the later clients' loads are still in flight
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      xv[0][q] = __builtin_nontemporal_load((const gcf4*)(a.x[t.k] + t.begin) + tid + q * 256);
      bv[q] = kB ? b[q * 256] : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 1; c < C; ++c) {
      const gcf4* x = (const gcf4*)(a.x[c < nc ? t.k + c : t.k] + t.begin) + tid;
#pragma unroll
      for (int q = 0; q < kQ; ++q)
        xv[c][q] = c < nc ? __builtin_nontemporal_load(x + q * 256) : f4{0.f, 0.f, 0.f, 0.f};  // nc is uniform
    }
  } else {
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const gcf4* x = (const gcf4*)(a.x[c < nc ? t.k + c : t.k] + t.begin) + tid;
        xv[c][q] = c < nc ? __builtin_nontemporal_load(x + q * 256) : f4{0.f, 0.f, 0.f, 0.f};  // nc is uniform
      }
      bv[q] = kB ? b[q * 256] : f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const int leaf = tid >> 3, j = tid & 7;
#pragma unroll
  for (int s = 0; s < 2 * C; ++s) {  // (client, half) in order
    const int c = s >> 1, h = s & 1;
    if (s) __syncthreads();  // the previous pass's leaf reads are done
#pragma unroll
    for (int q = 0; q < kHalfQ; ++q) {
      const uint32_t i = uint32_t(q * 1024 + 4 * tid);  // element h * 4096 + i
      const f4 d = xv[c][h * kHalfQ + q] - bv[h * kHalfQ + q];
      *reinterpret_cast<f4*>(sq + np_pad8(i)) = d * d;
    }
    __syncthreads();
    // 32 leaves x 8 accumulators = the 256 threads
    const float* l = sq + leaf * kLeafPitch + j;
    float r = l[0];
#pragma unroll
    for (int i = 8; i < kPW; i += 8) r += l[i];
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (j == 0) leaf_sum[c][h * 32 + leaf] = r;
  }
  __syncthreads();
  // wave w: client w's 64 leaves (clients 4 .. C - 1 on a second pass)
#pragma unroll
  for (int c0 = 0; c0 < C; c0 += 4) {
    const int c = c0 + (tid >> 6);
    if (c < C) {
      float s = leaf_sum[c][tid & 63];
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) s = s + __shfl_xor(s, m);
      if ((tid & 63) == 0 && c < nc) a.chunk_sums[uint64_t(t.k + c) * a.n_chunks + t.c] = s;
    }
  }
}

// The partial last chunk of every (piece, client), through the full-staging path (kPar: its leaves
// summed in parallel, np_partial_par).
template <bool kPar = true, bool kB = true>
__global__ __launch_bounds__(256) void np_sumsq_tail_kernel(SumsqArgs a) {
  __shared__ float sq[kNpBuf / kPW * kLeafPitch];
  __shared__ float leaf_sum[kNpBuf / kPW];
  const uint32_t k = blockIdx.x % uint32_t(a.K), pc = blockIdx.x / uint32_t(a.K);
  const uint32_t c_end = pc + 1 < a.n_pieces ? a.first_chunk[pc + 1] : a.n_chunks;
  if (c_end == a.first_chunk[pc]) return;
  const NpTask t = np_task(a, uint64_t(c_end - 1) * uint64_t(a.K) + k);
  if (t.n == kNpBuf) return;  // workgroup-uniform: a whole last chunk went through the half kernel
  float xv[kNpBuf / 256], bv[kNpBuf / 256];
  np_load<256, kB>(a, t, xv, bv);
  np_chunk<256, kPar>(a, t, xv, bv, sq, leaf_sum);
}

// One wave per (client, piece): numpy's outer loop adds the inner loops' pairwise sums one after the
// other (out = ((0 + s_0) + s_1) + ...), a serial chain of dependent adds.  The wave loads 64 chunk sums at
// a time (one per lane, independent loads) and folds them in order from lane 0 up (readlane: the chain
// runs on wave-uniform values), instead of one thread walking the chunks with a dependent load per
// add (up to 288 L2 round trips for ResNet-18's longest entries: ~30 us, round 5).
__global__ __launch_bounds__(256) void np_sumsq_pieces_kernel(SumsqArgs a) {
  // wave-uniform task index (the launch checks n_pieces * K < 2^32)
  const uint32_t t = blockIdx.x * 4u + uint32_t(__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)));
  if (t >= a.n_pieces * uint32_t(a.K)) return;
  const int lane = int(threadIdx.x & 63);
  const uint32_t k = t / a.n_pieces, pc = t % a.n_pieces;
  const uint32_t c0 = a.first_chunk[pc];
  const uint32_t c1 = pc + 1 < a.n_pieces ? a.first_chunk[pc + 1] : a.n_chunks;
  const float* sums = a.chunk_sums + uint64_t(k) * a.n_chunks;
  float out = 0.f;  // the reduction's identity, then out += pairwise(chunk) per inner loop
  for (uint32_t b = c0; b < c1; b += 64) {
    // lanes past the piece's last chunk hold +0: every sum here is >= +0 (sums of squares, from +0), so
    // adding +0 leaves its bits as they are, and the fold runs unrolled with constant lane indices
    const float v = b + uint32_t(lane) < c1 ? sums[b + uint32_t(lane)] : 0.f;
#pragma unroll
    for (int j = 0; j < 64; ++j) out = out + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
  }
  if (lane == 0) a.out[uint64_t(k) * a.n_pieces + pc] = out;
}

// variant 0 (the default): four clients of a chunk per workgroup sharing the baseline loads
// (np_sumsq_half4xc_kernel<4>; two when K = 2-3, one when K = 1) plus the partial last chunks with their
// leaves summed in parallel (np_sumsq_tail_kernel<true>) on a side stream beside the full chunks
// (run_np_sumsq): 0.979-0.985 ms against 1.004-1.032 for two clients (variant 14, the form before) in two
// interleaved runs (profiles/r05zzc, r05zzd_polaris_variants.log), bitwise equal.  With the partial chunks
// serialised after the full ones, four clients had lost to two (1.169 / 1.153): the shapes trade against
// the partial chunks' overlap.  14: two clients, the first client's and the baseline's loads issued first
// (np_sumsq_half4xc_kernel<2, true>); 11: variant 14 with both launches on one stream, 1.060-1.086;
// 10: variant 14 with the partial chunks walked by one lane, 1.033-1.048 (on one stream: 1.148, against
// 1.053 leaf-parallel, profiles/r05zza_polaris_variants.log); 9: two clients, loads interleaved; 7, 8:
// three / four clients, loads interleaved; 12, 13: three / four clients, the first client's loads first;
// 6: the one-client form (np_sumsq_half4_kernel, full chunks staged in two halves with 16-byte loads and
// LDS writes, 17.4 KB of LDS; the first round-5 default, 1.5-1.8 % under variant 5,
// profiles/r05b_polaris_variants.log, r05e-h);
// 1: the round-2 form (np_sumsq_chunks_lds_kernel, client-major, four memory round trips per
// workgroup); 2, 3: timing probes of variant 4 (wrong results by design: no baseline loads / no LDS
// phase); 4: the round-3 default (np_sumsq_chunks_v2_kernel, every chunk staged whole); 5: the round-4
// default (np_sumsq_half_kernel, dword loads and LDS writes).  A persistent loader / summer form (four
// loader waves keeping the next chunk's loads in flight, one summer wave per chunk, lane = leaf)
// measured 1.51 ms against 1.25 and was removed.
// Round 3's G clients per workgroup (4.1-5.9 ms: baseline staged through LDS, one load at a time) were
// dropped; a persistent software-pipelined form (2.9 ms: its two register sets left one workgroup per
// CU), 512 / 1,024 threads per chunk (1.70 / 2.79 ms against 1.38) and an LDS-free form loading each
// accumulator's stride-8 elements directly (2.20 ms) in round 4.
void launch_sumsq(int variant, const SumsqArgs& a, hipStream_t st, hipStream_t tail_st) {
  const uint64_t tasks = uint64_t(a.n_chunks) * uint64_t(a.K);
  const dim3 grid{uint32_t(tasks)}, tail_grid{uint32_t(uint64_t(a.n_pieces) * uint64_t(a.K))};
  if ((variant == 0 || variant == 11 || variant == 14) && a.K == 1) variant = 6;  // one client: nothing to share
  if (variant == 0 && a.K < 4) variant = 14;  // two or three clients: two per workgroup
  if (variant >= 1 && variant <= 4) {  // whole-chunk forms: no separate partial-chunk launch
    if (variant == 1) hipLaunchKernelGGL(np_sumsq_chunks_lds_kernel, grid, dim3(256), 0, st, a);
    else if (variant == 2) hipLaunchKernelGGL((np_sumsq_chunks_v2_kernel<256, 1>), grid, dim3(256), 0, st, a);
    else if (variant == 3) hipLaunchKernelGGL((np_sumsq_chunks_v2_kernel<256, 2>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((np_sumsq_chunks_v2_kernel<256>), grid, dim3(256), 0, st, a);
    return;
  }
  // the partial last chunks first (on tail_st: beside the full chunks), then the full chunks
  if (!a.base) {  // delta arenas (the default family only, run_np_sumsq): no baseline loads
    hipLaunchKernelGGL((np_sumsq_tail_kernel<true, false>), tail_grid, dim3(256), 0, tail_st, a);
    const int cd = variant == 6 ? 1 : variant == 14 ? 2 : 4;
    const dim3 gd{uint32_t(uint64_t(a.n_chunks) * uint64_t((a.K + cd - 1) / cd))};
    if (cd == 1) hipLaunchKernelGGL(np_sumsq_half4_kernel<false>, grid, dim3(256), 0, st, a);
    else if (cd == 2) hipLaunchKernelGGL((np_sumsq_half4xc_kernel<2, true, false>), gd, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((np_sumsq_half4xc_kernel<4, false, false>), gd, dim3(256), 0, st, a);
    return;
  }
  if (variant == 10) hipLaunchKernelGGL(np_sumsq_tail_kernel<false>, tail_grid, dim3(256), 0, tail_st, a);
  else hipLaunchKernelGGL(np_sumsq_tail_kernel<true>, tail_grid, dim3(256), 0, tail_st, a);
  const int c = (variant == 7 || variant == 12) ? 3 : (variant == 0 || variant == 8 || variant == 13) ? 4 : 2;
  const dim3 gc{uint32_t(uint64_t(a.n_chunks) * uint64_t((a.K + c - 1) / c))};
  if (variant == 5) hipLaunchKernelGGL(np_sumsq_half_kernel, grid, dim3(256), 0, st, a);
  else if (variant == 6) hipLaunchKernelGGL(np_sumsq_half4_kernel<>, grid, dim3(256), 0, st, a);
  else if (variant == 7) hipLaunchKernelGGL(np_sumsq_half4xc_kernel<3>, gc, dim3(256), 0, st, a);
  else if (variant == 8 || variant == 0) hipLaunchKernelGGL(np_sumsq_half4xc_kernel<4>, gc, dim3(256), 0, st, a);
  else if (variant == 9) hipLaunchKernelGGL(np_sumsq_half4xc_kernel<2>, gc, dim3(256), 0, st, a);
  else if (variant == 12) hipLaunchKernelGGL((np_sumsq_half4xc_kernel<3, true>), gc, dim3(256), 0, st, a);
  else if (variant == 13) hipLaunchKernelGGL((np_sumsq_half4xc_kernel<4, true>), gc, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((np_sumsq_half4xc_kernel<2, true>), gc, dim3(256), 0, st, a);  // 10, 11, 14
}
[[maybe_unused]] constexpr int kNumSumsqVariants = 15;
constexpr int kSumsqDefault = 0;  // four clients per workgroup + side-stream parallel-leaf tail: 0.98 ms (128 ResNet-18)
int run_np_sumsq(int variant, const float* const* d_x, int K, const float* d_base, const plato_agg_chunk* d_pieces,
                 const uint32_t* d_first_chunk, uint32_t n_pieces, uint32_t n_chunks, void* d_workspace,
                 float* d_out, hipStream_t stream);

}  // namespace

extern "C" {

size_t plato_agg_np_sumsq_workspace(int K, uint32_t n_chunks) {
  return size_t(K > 0 ? K : 0) * size_t(n_chunks) * sizeof(float);
}

int plato_agg_np_sumsq(const float* const* d_x, int K, const float* d_base, const plato_agg_chunk* d_pieces,
                       const uint32_t* d_first_chunk, uint32_t n_pieces, uint32_t n_chunks, void* d_workspace,
                       float* d_out, hipStream_t stream) {
  return run_np_sumsq(kSumsqDefault, d_x, K, d_base, d_pieces, d_first_chunk, n_pieces, n_chunks, d_workspace, d_out,
                      stream);
}

#ifdef PLATO_AGG_TUNE
int plato_agg_tune_num_np_sumsq_variants(void) { return kNumSumsqVariants; }

int plato_agg_tune_np_sumsq(int variant, const float* const* d_x, int K, const float* d_base,
                            const plato_agg_chunk* d_pieces, const uint32_t* d_first_chunk, uint32_t n_pieces,
                            uint32_t n_chunks, void* d_workspace, float* d_out, hipStream_t stream) {
  if (variant < 0 || variant >= kNumSumsqVariants) return set_error(PLATO_AGG_EINVAL, "bad np_sumsq variant");
  return run_np_sumsq(variant, d_x, K, d_base, d_pieces, d_first_chunk, n_pieces, n_chunks, d_workspace, d_out,
                      stream);
}
#endif

}  // extern "C"

namespace {
int run_np_sumsq(int variant, const float* const* d_x, int K, const float* d_base, const plato_agg_chunk* d_pieces,
                 const uint32_t* d_first_chunk, uint32_t n_pieces, uint32_t n_chunks, void* d_workspace,
                 float* d_out, hipStream_t stream) {
  if (K <= 0) return set_error(PLATO_AGG_EINVAL, "K must be >= 1");
  if (!n_pieces) return clear_error();
  if (!d_x || !d_pieces || !d_first_chunk || !d_workspace || !d_out)
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  // a null baseline: the client rows hold deltas (delta arenas) — the default's kernels (variants 0, 6, 14)
  if (!d_base && variant != 0 && variant != 6 && variant != 14)
    return set_error(PLATO_AGG_EINVAL, "a null baseline (delta arenas) needs variant 0, 6 or 14");
  SumsqArgs a{};
  a.x = d_x;
  a.base = d_base;
  a.pieces = d_pieces;
  a.first_chunk = d_first_chunk;
  a.n_pieces = n_pieces;
  a.n_chunks = n_chunks;
  a.K = K;
  a.chunk_sums = static_cast<float*>(d_workspace);
  a.out = d_out;
  const uint64_t t1 = uint64_t(n_chunks) * uint64_t(K), t2 = uint64_t(n_pieces) * uint64_t(K);
  if (t1) {
    if (t1 > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "too many chunks");
    // the partial-chunk kernel (variants 0, 5-10) runs on a side stream beside the full-chunk kernel
    // (0.23 ms of the launch when serialised after it, profiles/r05zzb kernel trace)
    const bool tail = !(variant >= 1 && variant <= 4) && variant != 11;  // 11: the default, one stream
    hipDevice_t dev = 0;
    int cur = 0;
    SideStream* ss = nullptr;
    if (tail && hipStreamGetDevice(stream, &dev) == hipSuccess && hipGetDevice(&cur) == hipSuccess) {
      if (cur != dev) (void)hipSetDevice(dev);
      ss = side_stream(dev);
    }
    if (ss) {
      std::lock_guard<std::mutex> lk(ss->mu);
      (void)hipEventRecord(ss->fork, stream);
      (void)hipStreamWaitEvent(ss->s, ss->fork, 0);
      launch_sumsq(variant, a, stream, ss->s);
      (void)hipEventRecord(ss->join, ss->s);
      (void)hipStreamWaitEvent(stream, ss->join, 0);
    } else {
      launch_sumsq(variant, a, stream, stream);
    }
    if (tail && cur != int(dev)) (void)hipSetDevice(cur);
    if (int rc = check_launch("np_sumsq chunks launch")) return rc;
  }
  if (t2 > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "too many pieces");
  hipLaunchKernelGGL(np_sumsq_pieces_kernel, dim3(uint32_t((t2 + 3) / 4)), dim3(256), 0, stream, a);
  return check_launch("np_sumsq pieces launch");
}
}  // namespace

namespace {
int run_cosine(bool scaled, const float* d_a, const float* const* d_b, int K, size_t n, const float* d_norm_a,
               const float* d_norm_b, float eps, int threads, void* d_workspace, float* d_out, hipStream_t stream,
               int variant = 0) {
  if (K <= 0 || K > 65535) return set_error(PLATO_AGG_EINVAL, "K must be in [1, 65535]");
  if (threads < 1 || threads > 1024) return set_error(PLATO_AGG_EINVAL, "threads must be in [1, 1024]");
  if (!d_a || !d_b || (!scaled && !d_norm_a) || !d_norm_b || !d_workspace || !d_out)
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (n == 0) return set_error(PLATO_AGG_EINVAL, "empty vectors");
  CosArgs a{};
  a.av = d_a;
  a.bv = d_b;
  a.norm_a = d_norm_a;
  a.norm_b = d_norm_b;
  a.eps = eps;
  a.n = n;
  a.T = threads;
  a.partial = static_cast<float*>(d_workspace);
  a.out = d_out;
  // TensorIterator's parallel_reduce: one pass below the grain or on one
  // thread, else two passes over min(T, ceil(n / 32768)) OpenMP chunks
  const uint64_t grain = 32768;
  a.single = (n < grain || threads == 1) ? 1 : 0;
  if (a.single) {
    a.nt = 1;
    a.chunk = n;
  } else {
    uint64_t nt = uint64_t(threads);
    const uint64_t by_grain = (n + grain - 1) / grain;
    if (by_grain < nt) nt = by_grain;
    a.chunk = (n + nt - 1) / nt;
    a.nt = int((n + a.chunk - 1) / a.chunk);
  }
  // the level-0 sums of one level-1 group are staged in LDS: L = 2^lp <= 64 rows
  {
    const uint64_t size_ilp = (a.chunk / 8) / 4;
    int r = 0;
    while ((uint64_t(1) << r) < size_ilp) ++r;
    if (r / 4 > 6) return set_error(PLATO_AGG_EINVAL, "thread chunk too long (> 2^33 elements)");
  }
  // variant (tuning only): 1 = one LDS buffer, two barriers per level-1 group (round 3).  Held to 64
  // VGPRs (eight waves per SIMD, the 2,048-workgroup grid in one round) the default spilled (2.23 ms)
  // and, loading one level-0 group at a time, ran 1.070 against 1.044 (profiles/r04zh_cosine.log).  Two
  // clients of a chunk per workgroup sharing the loads of a in registers (118 VGPRs, lanes 32c.. of wave 0
  // running client c's higher levels) ran 1.117 against 1.083, bitwise equal (profiles/r05z_cosine_variants.log);
  // removed.  Shared through LDS instead (cosine_chunks2_kernel), two clients win: the default below
  const dim3 grid{uint32_t(K), uint32_t(a.nt)};
  // variant 0 (the default): two clients of a chunk per 512-thread workgroup, a shared through LDS
  // (cosine_chunks2_kernel<2>), when every chunk has L = 16 (at most 2^24 elements) and K >= 2: 1.041 /
  // 1.042 ms against 1.109 / 1.111 for the one-client kernel (variant 2, the round-4/5 default) in two
  // interleaved runs, 1.056 / 1.074 against 1.093 / 1.101 on another lease (profiles/r05zzzb_cosine_shared_a.log,
  // r05zzza_…), bitwise equal; four clients per workgroup (variant 3) 1.23-1.27.  Else the one-client kernel.
  const bool two = a.chunk <= (uint64_t(1) << 24) && K >= 2;
  if (variant == 1) {
    if (scaled) hipLaunchKernelGGL((cosine_chunks_kernel<true, false>), grid, dim3(kSumThreads), 0, stream, a);
    else hipLaunchKernelGGL((cosine_chunks_kernel<false, false>), grid, dim3(kSumThreads), 0, stream, a);
  } else if (variant == 0 && two) {
    const dim3 g2{uint32_t((K + 1) / 2), uint32_t(a.nt)};
    if (scaled) hipLaunchKernelGGL((cosine_chunks2_kernel<true, 2>), g2, dim3(2 * kSumThreads), 0, stream, a, K);
    else hipLaunchKernelGGL((cosine_chunks2_kernel<false, 2>), g2, dim3(2 * kSumThreads), 0, stream, a, K);
  } else if (variant == 3 && two) {  // four clients per workgroup
    const dim3 g4{uint32_t((K + 3) / 4), uint32_t(a.nt)};
    if (scaled) hipLaunchKernelGGL((cosine_chunks2_kernel<true, 4>), g4, dim3(4 * kSumThreads), 0, stream, a, K);
    else hipLaunchKernelGGL((cosine_chunks2_kernel<false, 4>), g4, dim3(4 * kSumThreads), 0, stream, a, K);
  } else {  // variant 2 and the fallback: one client per workgroup, double-buffered level-0 sums
    if (scaled) hipLaunchKernelGGL(cosine_chunks_kernel<true>, grid, dim3(kSumThreads), 0, stream, a);
    else hipLaunchKernelGGL(cosine_chunks_kernel<false>, grid, dim3(kSumThreads), 0, stream, a);
  }
  if (int rc = check_launch("cosine chunks launch")) return rc;
  hipLaunchKernelGGL(cosine_combine_kernel, dim3(uint32_t((K + 63) / 64)), dim3(64), 0, stream, a, K);
  return check_launch("cosine combine launch");
}
}  // namespace

extern "C" {


int plato_agg_flatten(int mode, const void* const* d_src_f32, const void* const* d_src_i64, int K,
                      const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
                      uint32_t n_segs, size_t n_flat, float lr, float* const* d_out, hipStream_t stream) {
  if (mode < PLATO_AGG_FLAT_DELTA || mode > PLATO_AGG_FLAT_RAW) return set_error(PLATO_AGG_EINVAL, "bad mode");
  if (K <= 0 || K > 65535) return set_error(PLATO_AGG_EINVAL, "K must be in [1, 65535]");
  if (n_flat == 0) return clear_error();
  if (!d_src_f32 || !d_src_i64 || !d_segs || !n_segs || !d_out)
    return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (mode != PLATO_AGG_FLAT_RAW && (!d_base_f32 || !d_base_i64))
    return set_error(PLATO_AGG_EINVAL, "the delta modes need the baseline");
  FlatArgs a{};
  a.src_f = d_src_f32;
  a.src_i = d_src_i64;
  a.base_f = d_base_f32;
  a.base_i = d_base_i64;
  a.segs = d_segs;
  a.n_segs = n_segs;
  a.n_flat = n_flat;
  a.lr = lr;
  a.out = d_out;
  a.mode = mode;
  a.K = K;
  const uint64_t blocks = (uint64_t(n_flat) + 256 * kFlatPer - 1) / (256 * kFlatPer);
  if (blocks > 0x7fffffffull) return set_error(PLATO_AGG_EINVAL, "vector too long");
  hipLaunchKernelGGL(flatten_kernel, dim3(uint32_t(blocks), uint32_t((K + kFlatK - 1) / kFlatK)), dim3(256), 0,
                     stream, a);
  return check_launch("flatten launch");
}

int plato_agg_sdot_pairs(const float* const* d_x, const float* const* d_y, int n_pairs, size_t n, float* d_out_xy,
                         float* d_out_yy, hipStream_t stream) {
  if (n_pairs <= 0) return set_error(PLATO_AGG_EINVAL, "no pairs");
  if (!d_x || !d_y || !d_out_xy) return set_error(PLATO_AGG_EINVAL, "null pointer");
  SdotArgs a{d_x, d_y, uint64_t(n), d_out_xy, d_out_yy};
  hipLaunchKernelGGL(sdot_skx_kernel, dim3(uint32_t(n_pairs)), dim3(kSdotThreads), 0, stream, a);
  return check_launch("sdot launch");
}

size_t plato_agg_sdot_shared_workspace(int n_pairs, int with_xx) {
  return size_t(n_pairs > 0 ? n_pairs : 0) * 128 * sizeof(float) + (with_xx ? 128 * sizeof(float) : 0);
}

int plato_agg_sdot_shared(const float* d_x, const float* const* d_y, int n_pairs, size_t n, int with_xx,
                          float* d_workspace, float* d_out_xy, float* d_out_yy, hipStream_t stream) {
  return run_sdot_shared(-1, d_x, d_y, n_pairs, n, with_xx, d_workspace, d_out_xy, d_out_yy, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_sdot_shared_variants(void) { return kNumSdotSVariants; }

int plato_agg_tune_sdot_shared(int variant, const float* d_x, const float* const* d_y, int n_pairs, size_t n,
                               int with_xx, float* d_workspace, float* d_out_xy, float* d_out_yy,
                               hipStream_t stream) {
  if (variant < 0) return set_error(PLATO_AGG_EINVAL, "bad sdot_shared variant");
  return run_sdot_shared(variant, d_x, d_y, n_pairs, n, with_xx, d_workspace, d_out_xy, d_out_yy, stream);
}
#endif  // PLATO_AGG_TUNE

size_t plato_agg_torch_cosine_workspace(int K, int threads) {
  return size_t(K > 0 ? K : 0) * size_t(threads > 0 ? threads : 1) * sizeof(float);
}

int plato_agg_torch_cosine_sum(const float* d_a, const float* const* d_b, int K, size_t n, const float* d_norm_a,
                               const float* d_norm_b, float eps, int threads, void* d_workspace, float* d_out,
                               hipStream_t stream) {
  return run_cosine(false, d_a, d_b, K, n, d_norm_a, d_norm_b, eps, threads, d_workspace, d_out, stream);
}

int plato_agg_torch_cosine_sum_scaled(const float* d_a_scaled, const float* const* d_b, int K, size_t n,
                                      const float* d_norm_b, float eps, int threads, void* d_workspace, float* d_out,
                                      hipStream_t stream) {
  return run_cosine(true, d_a_scaled, d_b, K, n, nullptr, d_norm_b, eps, threads, d_workspace, d_out, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_cosine_variants(void) { return 4; }

int plato_agg_tune_torch_cosine_sum_scaled(int variant, const float* d_a_scaled, const float* const* d_b, int K,
                                           size_t n, const float* d_norm_b, float eps, int threads,
                                           void* d_workspace, float* d_out, hipStream_t stream) {
  if (variant < 0 || variant > 3) return set_error(PLATO_AGG_EINVAL, "bad cosine variant");
  return run_cosine(true, d_a_scaled, d_b, K, n, nullptr, d_norm_b, eps, threads, d_workspace, d_out, stream,
                    variant);
}
#endif  // PLATO_AGG_TUNE

int plato_agg_scale_by_norm(const float* d_a, size_t n, const float* d_norm, float eps, float* d_out,
                            hipStream_t stream) {
  if (!d_a || !d_norm || !d_out) return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (n == 0) return clear_error();
  const uint64_t blocks = (uint64_t(n) + 255) / 256;
  hipLaunchKernelGGL(scale_by_norm_kernel, dim3(uint32_t(blocks < 8192 ? blocks : 8192)), dim3(256), 0, stream, d_a,
                     uint64_t(n), d_norm, eps, d_out);
  return check_launch("scale_by_norm launch");
}

}  // extern "C"

namespace plato_agg_internal {

SideStream* side_stream(int dev) {
  static std::mutex mu;
  static std::map<int, SideStream*> all;
  std::lock_guard<std::mutex> lk(mu);
  auto it = all.find(dev);
  if (it != all.end()) return it->second;
  auto* ss = new SideStream();  // process lifetime
  if (hipStreamCreateWithFlags(&ss->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ss->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ss->join, hipEventDisableTiming) != hipSuccess) {
    delete ss;
    return nullptr;
  }
  all[dev] = ss;
  return ss;
}

}  // namespace plato_agg_internal
