// port.hip — Port's vector norms straight from the staged arenas, for gfx950.
// C ABI: include/plato_agg.h (plato_agg_port_norms).  CPU restatement: oracle/reductions.c (torch norm).
//
// The reference (examples/async/port/port_server.py:38-50) flattens the current model minus the
// previous one and every client delta with torch.cat in state_dict order (int64 entries cast to
// float32 on the way) and takes F.cosine_similarity, whose vector norms are ATen's
// linalg_vector_norm of a contiguous float32 vector: on x86-64, 8 fma chains (chain j sums the
// squares of positions = j mod 8, serially), the 8 lanes added in order, then ATen's scalar tail.
//
// The round-2 path flattened the vectors (plato_agg_flatten: 5.7 GB read and written for 128
// ResNet-18 clients, 2.4 ms) before plato_agg_entry_norms_f32 read them again.  Here the
// flattening is folded into the norm kernel: producer waves gather four positions per lane from
// the arenas through the state_dict-order segment map (the int64 counters interleaved where
// state_dict puts them), form the delta in registers and write it transposed into an LDS tile —
// chain j's steps contiguous in row j; the chain wave walks the 8 chains out of LDS with
// ds_read_b128.  The producers also store the flattened vector (d_flat_out) for the cosine sums,
// which need the norms first: the store rides in the shadow of the serial chain.
//
// Shape: one workgroup per vector (V = K + 1: vector 0 = current - previous, vectors 1..K the
// client deltas), 1 chain wave + kWp producer waves, kT-position tiles (kT / 8 steps per chain),
// a two-slot tile ring and one s_barrier per tile; each producer keeps kD tiles of loads in flight.
// The launch is bound by the serial chain (n / 8 dependent fmas), not by HBM; DESIGN.md §13.
// Compiled with -ffp-contract=off; the chain fma is an explicit fma (torch's vfmadd231ps).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "common.h"
#include "plato_agg.h"

using plato_agg_internal::clear_error;
using plato_agg_internal::set_error;

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ T sld(const T* p, int i) {
  return ((__attribute__((address_space(4))) const T*)p)[i];
}

constexpr int kLanes = 8;                 // torch's 8-lane vectorised accumulation
// Tile of kT positions (2,048 the default; 4,096 halves the chain wave's per-tile barrier and first
// read): kSteps steps per chain, row pitch kR (conflict-free writes, see pn_write, and reads), kIts
// gather iterations of 256 positions (4 per lane).
template <int kT>
struct PnTile {
  static constexpr int kSteps = kT / kLanes;
  static constexpr int kR = kSteps + 4;
  static constexpr int kSlot = kLanes * kR;
  static constexpr int kIts = kT / 256;
};
constexpr int kMaxSegs = 2048;
constexpr uint32_t kSegI64 = 1u;

struct PnSeg {
  uint32_t flat, end, src, info;  // positions [flat, end) read element src + (p - flat) of the region
};

struct PnArgs {
  const float* const* xf;    // [V] fp32 arenas: the minuends
  const int64_t* const* xi;  // [V] int64 arenas
  const float* const* bf;    // [V] fp32 arenas subtracted
  const int64_t* const* bi;  // [V] int64 arenas subtracted
  const plato_agg_segment* segs;
  uint32_t n_segs;
  uint32_t n;                // flat length
  uint32_t m;                // n - n % 8: the vectorised part
  uint64_t n_f32;
  int cast_first;            // vector 0 subtracts its int64 entries as torch.cat(...) - torch.cat(...)
  float* out;                // [V]
  float* const* flat;        // [V] rows for the flattened vectors (16-byte aligned), or null
  const uint32_t* lengths;   // [V] per-vector lengths (<= n), or null: every vector n long
};

// ATen's scalar tail of the last-dim 2-norm as x86-64 PyTorch 2.10 compiled it (entrywise.hip,
// torch_norm_tail_step): 4 or more remaining -> separately rounded product and add, else fused.
__device__ __forceinline__ float pn_tail_step(float s, float v, uint32_t e, uint32_t m, uint32_t n) {
  if (n - m >= 4 && e < m + 4) return s + v * v;
  return __builtin_fmaf(v, v, s);
}

// The flattened delta at position p (the slow path: entry boundaries, int64 entries, the tail).
// fp32: x - b.  int64: torch.cat casts each int64 entry to float32 — vector 0 (current - previous)
// subtracts the casts, the deltas (compute_weight_deltas, algorithms/fedavg.py:23) are int64
// differences (wrapping) cast once.
__device__ __forceinline__ float pn_value(const PnArgs& a, const PnSeg* S, int& idx, uint32_t p, int v) {
  while (idx + 1 < int(a.n_segs) && S[idx + 1].flat <= p) ++idx;
  const PnSeg sg = S[idx];
  const uint32_t e = p - sg.flat + sg.src;
  const float* bf = a.bf[v];  // null: vector v's arena already holds x - b (delta arenas)
  if (!(sg.info & kSegI64)) return a.xf[v][e] - (bf ? bf[e] : 0.f);
  const int64_t* bi = a.bi[v];
  const int64_t x = a.xi[v][e], b = bi ? bi[e] : int64_t(0);
  if (v == 0 && a.cast_first) return float(x) - float(b);
  return float(int64_t(uint64_t(x) - uint64_t(b)));
}

struct PnCursor {  // a producer wave's current entry, wave-uniform (positions only move forward)
  int idx;
  uint32_t flat, end, src, info;
};

__device__ __forceinline__ void pn_cursor_load(const PnSeg* S, int idx, PnCursor& c) {
  c.idx = idx;
  c.flat = __builtin_amdgcn_readfirstlane(S[idx].flat);
  c.end = __builtin_amdgcn_readfirstlane(S[idx].end);
  c.src = __builtin_amdgcn_readfirstlane(S[idx].src);
  c.info = __builtin_amdgcn_readfirstlane(S[idx].info);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pn_rsrc(const void* base, uint64_t bytes) {
  const uint64_t n = bytes < 0xffffffffull ? bytes : 0xffffffffull;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)uint32_t(n), 0x00020000);
}

__device__ __forceinline__ f4 pn_load4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  // dword-aligned 16-byte loads (an entry's arena offset is 4-byte aligned only)
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

template <int kIt>
struct PnRegs {
  f4 x[kIt], b[kIt];
  int seg[kIt];   // the wave's entry at the iteration's first position (where a slow iteration's walk starts)
  uint32_t fast;  // bit i: iteration i lies inside one fp32 entry and below m (wave-uniform)
};

template <int kT, int kWp, int kIt>
__device__ __forceinline__ void pn_issue(const PnArgs& a, const PnSeg* S, PnCursor& cur, __amdgpu_buffer_rsrc_t rx,
                                         __amdgpu_buffer_rsrc_t rb, uint32_t t, int w, int lane, PnRegs<kIt>& r) {
  r.fast = 0;
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    const uint32_t pf = t * kT + uint32_t(i * kWp + w) * 256;  // the iteration's first position
    const uint32_t pl = pf + 255;
    while (pf >= cur.end && cur.idx + 1 < int(a.n_segs)) pn_cursor_load(S, cur.idx + 1, cur);  // rare
    uint32_t e = 0;  // slow iterations still issue their loads (same count on every path)
    r.seg[i] = cur.idx;
    if (!(cur.info & kSegI64) && pl < cur.end && pl < a.m) {
      r.fast |= 1u << i;
      e = pf + uint32_t(4 * lane) - cur.flat + cur.src;
    }
    r.x[i] = pn_load4(rx, e * 4u);
    r.b[i] = pn_load4(rb, e * 4u);
  }
}

// Lane L holds positions p .. p + 3 (p = pf + 4L): chains 4 (L & 1) .. + 3, step (p - tile) / 8.
// Row pitch kR = 260: ds_write_b32 banks (a/4) mod 32 per 32-lane half, and rows 0 and 4 are
// 4 kR = 16 mod 32 apart, so each write's half-wave covers 32 banks (pitch 264 put lanes L and L ^ 1
// on one bank: 45 M extra LDS cycles per 129-vector launch, profiles/r03x_pmc_paths.txt); the chain
// wave's ds_read_b128 of rows 0..7 (banks mod 64) sit on 8 different 16-byte slots.
template <int kT, int kWp, int kIt, bool kNT>
__device__ __forceinline__ void pn_write(const PnArgs& a, const PnSeg* S, float* slot, float* flat, uint32_t t, int w,
                                         int lane, int v, const PnRegs<kIt>& r) {
#pragma unroll
  for (int i = 0; i < kIt; ++i) {
    constexpr int kR = PnTile<kT>::kR;
    const int q = i * kWp + w;
    float* dst = slot + (4 * (lane & 1)) * kR + q * 32 + (lane >> 1);
    const uint32_t p = t * kT + uint32_t(q) * 256 + uint32_t(4 * lane);
    if (r.fast & (1u << i)) {
      const f4 d = r.x[i] - r.b[i];
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[c * kR] = d[c];
      if (flat) {  // the flattened vector for the cosine sums, as a by-product
        if (kNT) __builtin_nontemporal_store(d, reinterpret_cast<f4*>(flat + p));
        else *reinterpret_cast<f4*>(flat + p) = d;
      }
    } else {  // an entry boundary, an int64 entry or the end of the vectorised part inside the iteration
      int idx = r.seg[i];
      for (int c = 0; c < 4; ++c) {
        const float d = p + c < a.m ? pn_value(a, S, idx, p + c, v) : 0.f;
        dst[c * kR] = d;
        if (flat && p + c < a.m) flat[p + c] = d;  // positions m .. n - 1: the tail loop
      }
    }
  }
}

// s_waitcnt lgkmcnt(N) alone (gfx9 encoding; vmcnt and expcnt at their maxima)
template <int N>
__device__ __forceinline__ void pn_wait_lgkm() {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (N << 8) | (3 << 14));
}

// kOW: the chain's LDS reads per wait.  0: the compiler's waits, one s_waitcnt per ds_read_b128 of
// a 16-step block; 1: one s_waitcnt per 16-step block (4 reads), 2: per 32-step block (8 reads).
// scripts/micro/chain_b128.hip: each ds_read_b128 costs the chain wave ~5 issue cycles and each
// s_waitcnt ~3.7 on top of the 4 of a dependent v_fmac_f32 (profiles/r04_micro_chain_b128.log).
template <int kWp, int kD, bool kNT = false, int kT = 2048, int kOW = 0>
__global__ __launch_bounds__(64 * (1 + kWp)) void port_norms_kernel(PnArgs a_in) {
  using Tl = PnTile<kT>;
  constexpr int kIts = Tl::kIts, kSlot = Tl::kSlot, kR = Tl::kR, kSteps = Tl::kSteps;
  constexpr int kIt = kIts / kWp;
  PnArgs a = a_in;
  if (a.lengths) {  // this vector's own length (FedAtt: one entry of one client)
    a.n = a.lengths[blockIdx.x];
    a.m = a.n - a.n % kLanes;
  }
  static_assert(kIts % kWp == 0, "whole gather iterations per producer");
  __shared__ __attribute__((aligned(16))) float ring[2 * kSlot];
  __shared__ PnSeg S[kMaxSegs];
  const int v = int(blockIdx.x);
  for (int j = int(threadIdx.x); j < int(a.n_segs); j += int(blockDim.x)) {
    const plato_agg_segment sg = a.segs[j];
    S[j] = PnSeg{uint32_t(sg.flat_offset), uint32_t(sg.flat_offset + sg.numel), uint32_t(sg.src_offset),
                 sg.region ? kSegI64 : 0u};
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = int(threadIdx.x & 63);
  const uint32_t ntiles = (a.m + kT - 1) / kT;
  const uint32_t nbar = (ntiles + kD - 1) / kD * kD;  // barriers: whole trips of kD tiles
  if (wave > 0) {  // producer
    const int w = wave - 1;
    // a null subtrahend (delta arenas: the arena holds x - b): a zero-length buffer, whose loads return 0
    // without a memory request, so x - 0 = x bit for bit
    const float* bfv = sld(a.bf, v);
    const __amdgpu_buffer_rsrc_t rx = pn_rsrc(sld(a.xf, v), a.n_f32 * 4), rb = pn_rsrc(bfv, bfv ? a.n_f32 * 4 : 0);
    PnCursor cur;
    pn_cursor_load(S, 0, cur);
    float* flat = a.flat ? sld(a.flat, v) : nullptr;
    PnRegs<kIt> regs[kD];
#pragma unroll
    for (int j = 0; j < kD; ++j) pn_issue<kT, kWp, kIt>(a, S, cur, rx, rb, uint32_t(j), w, lane, regs[j]);
    for (uint32_t t = 0; t < nbar; t += kD) {
#pragma unroll
      for (int j = 0; j < kD; ++j) {
        pn_write<kT, kWp, kIt, kNT>(a, S, ring + ((t + j) & 1) * kSlot, flat, t + j, w, lane, v, regs[j]);
        // past the last tile every load reads the arena's first elements: valid, never consumed
        const uint32_t nxt = t + j + kD;
        pn_issue<kT, kWp, kIt>(a, S, cur, rx, rb, nxt < ntiles ? nxt : ntiles, w, lane, regs[j]);
        __builtin_amdgcn_s_barrier();  // tile t + j published in slot (t + j) & 1
      }
    }
    return;
  }
  // chain wave: lane & 7 walks chain j over row j (lanes 8..63 repeat rows 0..7)
  __builtin_amdgcn_s_setprio(3);
  const int j = lane & 7;
  float acc = 0.f;
  for (uint32_t t = 0; t < nbar; ++t) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (t >= ntiles) continue;
    const f4* row = reinterpret_cast<const f4*>(ring + (t & 1) * kSlot + j * kR);
    if constexpr (kOW > 0) {
      // kQ reads (4 kQ steps) per block, the next block's reads in flight, one wait per block
      constexpr int kQ = 4 * kOW, kNB = kSteps / (4 * kQ);
      f4 buf[2][kQ];
#pragma unroll
      for (int q = 0; q < kQ; ++q) buf[0][q] = row[q];
#pragma unroll
      for (int blk = 0; blk < kNB; ++blk) {
        const int cb = blk & 1;
        if (blk + 1 < kNB) {
#pragma unroll
          for (int q = 0; q < kQ; ++q) buf[cb ^ 1][q] = row[kQ * (blk + 1) + q];
          pn_wait_lgkm<kQ>();  // this block's reads have landed; the next block's stay in flight
        } else {
          pn_wait_lgkm<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
          acc = __builtin_fmaf(buf[cb][q].x, buf[cb][q].x, acc);
          acc = __builtin_fmaf(buf[cb][q].y, buf[cb][q].y, acc);
          acc = __builtin_fmaf(buf[cb][q].z, buf[cb][q].z, acc);
          acc = __builtin_fmaf(buf[cb][q].w, buf[cb][q].w, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      continue;
    }
    // 16 steps per block as 4 ds_read_b128, the next block's reads in flight (positions past m are +0:
    // fma(0, 0, acc) leaves the non-negative sum unchanged)
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
  // the 8 lanes added in order (ATen's buffer[0] + buffer[1] + ...), then the scalar tail
  float s = __shfl(acc, 0, 64);
  for (int l = 1; l < kLanes; ++l) s = s + __shfl(acc, l, 64);
  if (lane != 0) return;
  int idx = 0;
  float* flat = a.flat ? sld(a.flat, v) : nullptr;
  for (uint32_t e = a.m; e < a.n; ++e) {
    const float d = pn_value(a, S, idx, e, v);
    if (flat) flat[e] = d;
    s = pn_tail_step(s, d, e, a.m, a.n);
  }
  a.out[v] = sqrtf(s);
}

using PnFn = void (*)(const PnArgs&, hipStream_t, int);
template <int kWp, int kD, bool kNT = false, int kT = 2048, int kOW = 0>
void launch_pn(const PnArgs& a, hipStream_t st, int V) {
  hipLaunchKernelGGL((port_norms_kernel<kWp, kD, kNT, kT, kOW>), dim3(uint32_t(V)), dim3(64 * (1 + kWp)), 0, st, a);
}
// producer waves x tiles of loads in flight (x non-temporal flat stores, x tile positions)
// 8,192-position tiles: 4.098 against 4.156 ms for 4,096 interleaved (profiles/r04zz_port.log; 4.12 against
// 4.17 in round 4's first sweep); one s_waitcnt per 32-step block: 3.536 against 4.099 ms
// (6.07 cycles per chain step; profiles/r04zz_port_onewait.log); with it, 4 producer waves (3.83 ms) and 3
// tiles of loads in flight (3.56) lose to the default's 3.51 (profiles/r04zz_port_producers.log)
constexpr PnFn kPnDefault = &launch_pn<8, 2, true, 8192, 2>;
#ifdef PLATO_AGG_TUNE
// The round-3 sweep (1-8 producer waves x 2-4 tiles in flight, plain or non-temporal flat stores;
// profiles/r03l_port.log) and round 4's tile sizes (profiles/r04n_port_variants.log) are in DESIGN.md
// §13-14; kept: the default, the round-3 default and the runners-up.
const PnFn kPnVariants[] = {
    &launch_pn<8, 2, true, 8192, 2>,  // 0: the default, 3.54 ms storing the flat vectors (8,192-position
                                      //    tiles, one s_waitcnt per 32 chain steps)
    &launch_pn<8, 3, true>,        // 1: the round-3 default (2,048), 4.70 ms
    &launch_pn<4, 2>,              // 2: 4.25 ms without the stores
    &launch_pn<8, 3, true, 4096>,  // 3: 4.17 ms
    &launch_pn<8, 2, true, 4096>,  // 4: the first round-4 default (4,096-position tiles), 4.16 ms
    &launch_pn<8, 1, true, 4096>,  // 5
    &launch_pn<8, 2, true, 8192, 1>,  // 6: one s_waitcnt per 16-step block, 3.67 ms
    &launch_pn<8, 2, true, 8192>,     // 7: the compiler's waits (one per ds_read_b128), 4.10 ms
};
constexpr int kNumPnVariants = sizeof(kPnVariants) / sizeof(kPnVariants[0]);
#endif

int run_port_norms(PnFn fn, const void* const* d_x_f32, const void* const* d_x_i64, const void* const* d_b_f32,
                   const void* const* d_b_i64, int n_vectors, const uint32_t* d_lengths, const plato_agg_segment* d_segs,
                   uint32_t n_segs, size_t n_flat, size_t n_f32, int flags, float* d_out, float* const* d_flat_out,
                   hipStream_t stream) {
  if (n_vectors <= 0) return set_error(PLATO_AGG_EINVAL, "n_vectors must be >= 1");
  if (!d_x_f32 || !d_x_i64 || !d_b_f32 || !d_b_i64 || !d_segs || !d_out) return set_error(PLATO_AGG_EINVAL, "null pointer");
  if (n_segs == 0 || n_segs > uint32_t(kMaxSegs)) return set_error(PLATO_AGG_EINVAL, "segment count must be in [1, 2048]");
  if (n_flat == 0 || n_flat >= (size_t(1) << 31)) return set_error(PLATO_AGG_EINVAL, "flat length must be in [1, 2^31)");
  if (n_f32 >= (size_t(1) << 30)) return set_error(PLATO_AGG_EINVAL, "fp32 arena must be < 2^30 elements");
  if (flags & ~PLATO_AGG_PORT_CAST_FIRST) return set_error(PLATO_AGG_EINVAL, "unknown flags");
  PnArgs a{};
  a.xf = reinterpret_cast<const float* const*>(d_x_f32);
  a.xi = reinterpret_cast<const int64_t* const*>(d_x_i64);
  a.bf = reinterpret_cast<const float* const*>(d_b_f32);
  a.bi = reinterpret_cast<const int64_t* const*>(d_b_i64);
  a.segs = d_segs;
  a.n_segs = n_segs;
  a.n = uint32_t(n_flat);
  a.m = uint32_t(n_flat - n_flat % kLanes);
  a.n_f32 = n_f32;
  a.cast_first = (flags & PLATO_AGG_PORT_CAST_FIRST) ? 1 : 0;
  a.out = d_out;
  a.flat = d_flat_out;
  a.lengths = d_lengths;
  fn(a, stream, n_vectors);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(PLATO_AGG_EHIP, std::string("port_norms launch: ") + hipGetErrorString(err));
  return clear_error();
}

}  // namespace

extern "C" {

int plato_agg_port_norms(const void* const* d_x_f32, const void* const* d_x_i64, const void* const* d_b_f32,
                         const void* const* d_b_i64, int n_vectors, const uint32_t* d_lengths,
                         const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat, size_t n_f32, int flags,
                         float* d_out, float* const* d_flat_out, hipStream_t stream) {
  return run_port_norms(kPnDefault, d_x_f32, d_x_i64, d_b_f32, d_b_i64, n_vectors, d_lengths, d_segs, n_segs, n_flat,
                        n_f32, flags, d_out, d_flat_out, stream);
}

#ifdef PLATO_AGG_TUNE  // include/plato_agg_tune.h
int plato_agg_tune_num_port_norms_variants(void) { return kNumPnVariants; }

int plato_agg_tune_port_norms(int variant, const void* const* d_x_f32, const void* const* d_x_i64,
                              const void* const* d_b_f32, const void* const* d_b_i64, int n_vectors,
                              const uint32_t* d_lengths, const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat,
                              size_t n_f32, int flags, float* d_out, float* const* d_flat_out, hipStream_t stream) {
  if (variant < 0 || variant >= kNumPnVariants) return set_error(PLATO_AGG_EINVAL, "bad port_norms variant");
  return run_port_norms(kPnVariants[variant], d_x_f32, d_x_i64, d_b_f32, d_b_i64, n_vectors, d_lengths, d_segs, n_segs,
                        n_flat, n_f32, flags, d_out, d_flat_out, stream);
}
#endif  // PLATO_AGG_TUNE

}  // extern "C"
