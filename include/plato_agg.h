/*
 * plato_agg.h — C ABI of the MI355X (gfx950) FedAvg aggregation engine.
 *
 * This is the drop-in boundary for Plato's server-side aggregation hot path.
 * Every entry point takes plain device pointers, element counts and a HIP
 * stream; nothing here allocates device memory, keeps a pointer after it
 * returns, or synchronises the stream (so the calls can be captured in a
 * hipGraph).  Host code (plato_amd/, ctypes) owns all buffers.
 *
 * Arithmetic contract (bit-exact with the reference CPU path):
 *   for every element e, clients i = 0..K-1 in the order of `d_x`:
 *     d   = x_i[e] - b[e]                  (fp32, RNE)       algorithms/fedavg.py:23
 *     t   = d * w_i                        (fp32, RNE)       servers/fedavg.py:154
 *     t   = t * s_i      (only if d_s)     (fp32, RNE)       pisces_server.py:94
 *     acc = acc + t                        (fp32, RNE, acc starts at +0)
 *   new[e] = b[e] + acc                    (fp32, RNE)       algorithms/fedavg.py:35
 * No FMA contraction, no reordering of the K-sum.  int64 entries (BatchNorm
 * num_batches_tracked) follow torch's promotion: d = x - b exactly in int64,
 * converted to fp32 (RNE) before the multiply, new = fp32(b) + acc as fp32;
 * load_state_dict's fp32 -> int64 truncation is plato_agg_cast_f32_i64.
 *
 * Errors: every call returns 0 on success or a negative PLATO_AGG_E* code;
 * plato_agg_last_error() gives a thread-local message for the last failure.
 * (The reference raises Python exceptions; plato_amd/_lib.py maps a non-zero
 * return to RuntimeError/ValueError.)
 *
 * Reference interfaces replaced (TL-System/plato @ 2025-10-03):
 *   plato_agg_fedavg_weights   <- Server._process_reports' deltas -> aggregate
 *                                 -> update chain, i.e. what an
 *                                 `aggregate_weights` hook must return
 *                                 (plato/servers/fedavg.py:171-196,
 *                                  plato/algorithms/fedavg.py:13-37)
 *   plato_agg_fedavg_deltas    <- Server.aggregate_deltas
 *                                 (plato/servers/fedavg.py:137-159)
 *   plato_agg_compute_deltas   <- Algorithm.compute_weight_deltas
 *                                 (plato/algorithms/fedavg.py:13-27)
 *   plato_agg_update_weights   <- Algorithm.update_weights
 *                                 (plato/algorithms/fedavg.py:29-37)
 *   plato_agg_cast_f32_i64     <- Algorithm.load_weights' load_state_dict
 *                                 fp32 -> int64 copy (plato/algorithms/fedavg.py:46-48)
 *   plato_agg_fedavg_weights_bf16 <- the model_dequantize inbound processor
 *                                 (plato/processors/model_dequantize.py:15-18)
 *                                 followed by the same chain, on bf16 payloads
 *   plato_agg_mix_weights      <- FedAsync Algorithm.aggregate_weights
 *                                 (examples/async/fedasync/fedasync_algorithm.py:9-20)
 *   plato_agg_client_dots      <- the model-wide reductions of Port's
 *                                 cosine_similarity (examples/async/port/
 *                                 port_server.py:24-52, F.cosine_similarity over
 *                                 the flattened models)
 *   plato_agg_entry_stats      <- the per-tensor reductions of the norm- and
 *                                 angle-based variants: FedAtt's per-layer
 *                                 torch.linalg.norm (examples/server_aggregation/
 *                                 fedatt/fedatt_algorithm.py:34-39), FedAdp's
 *                                 np.inner / np.linalg.norm of flattened deltas
 *                                 (examples/server_aggregation/fedadp/
 *                                 fedadp_server.py:95-99), Polaris' per-client
 *                                 conv-layer squared deltas (examples/
 *                                 client_selection/polaris/polaris_server.py:76-89)
 *   plato_agg_fedavg_qsgd      <- the model_dequantize_qsgd inbound processor
 *                                 (plato/processors/model_dequantize_qsgd.py:34-60)
 *                                 followed by the FedAvg chain, on QSGD payloads
 *   plato_agg_fedavg_entrywise <- weighted sums whose weight depends on the
 *                                 tensor as well as the client: FedAtt's
 *                                 attentive aggregation (fedatt_algorithm.py:44-69)
 *                                 and FedAdp's global-gradient pass
 *                                 (fedadp_server.py:43-50)
 */
#ifndef PLATO_AGG_H
#define PLATO_AGG_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLATO_AGG_ABI_VERSION 4

#define PLATO_AGG_OK 0
#define PLATO_AGG_EINVAL (-1)   /* bad argument (null, misaligned, K <= 0) */
#define PLATO_AGG_EHIP (-2)     /* HIP runtime error (launch / copy)      */
#define PLATO_AGG_ERCCL (-3)    /* RCCL unavailable or a collective failed */

/* ABI version of the loaded library (== PLATO_AGG_ABI_VERSION). */
int plato_agg_abi_version(void);

/* Thread-local description of the last failure on this thread ("" if none). */
const char* plato_agg_last_error(void);

/*
 * Fused FedAvg over K client weight arenas (a3 -> a4 -> a6 in one pass).
 *   d_x_f32  device array of K pointers, each to n_f32 fp32 client weights
 *            (16-byte aligned); summation order = array order.
 *   d_x_i64  device array of K pointers to n_i64 int64 client entries, or
 *            NULL when n_i64 == 0.
 *   d_w      device array of K fp32 weights (fp32(n_i / N) for FedAvg).
 *   d_s      device array of K fp32 second scalars, or NULL.
 *   d_base_* the global model (baseline) entries.
 *   d_out_f32   n_f32 fp32 new weights (may alias d_base_f32).
 *   d_out_i64f  n_i64 fp32 new values of the int64 entries (the reference's
 *               update_weights yields fp32 for them; cast with
 *               plato_agg_cast_f32_i64 to get what load_state_dict stores).
 */
int plato_agg_fedavg_weights(const float* const* d_x_f32,
                             const int64_t* const* d_x_i64,
                             const float* d_w, const float* d_s, int K,
                             const float* d_base_f32, const int64_t* d_base_i64,
                             float* d_out_f32, float* d_out_i64f,
                             size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * Weighted sum of K client delta arenas (Server.aggregate_deltas):
 *   avg[e] = sum_i fp32(d_i[e]) * w_i  (sequential, fp32), avg is fp32 for
 * every entry, including the int64 ones (trainers/basic.py:59-63).
 */
int plato_agg_fedavg_deltas(const float* const* d_d_f32,
                            const int64_t* const* d_d_i64,
                            const float* d_w, const float* d_s, int K,
                            float* d_avg_f32, float* d_avg_i64f,
                            size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * Fused FedAvg over K bf16-quantized client payloads (Plato's model_quantize
 * codec: every entry .to(bfloat16), plato/processors/model_quantize.py:15),
 * equal to dequantizing them on the server (model_dequantize.py:15-18,
 * .to(float32), exact) and running plato_agg_fedavg_weights: the payload
 * stays bf16 through PCIe and HBM and is widened in registers.  The int64
 * entries' payload values are bf16 as well; as in the reference, they are
 * subtracted from the int64 baseline in fp32: d = fp32(x) - fp32(b).
 *   d_x_bf16      K pointers to n_f32 bf16 values (16-byte aligned)
 *   d_x_i64_bf16  K pointers to n_i64 bf16 values (or NULL if n_i64 == 0)
 * Other arguments as plato_agg_fedavg_weights.
 */
int plato_agg_fedavg_weights_bf16(const uint16_t* const* d_x_bf16,
                                  const uint16_t* const* d_x_i64_bf16,
                                  const float* d_w, const float* d_s, int K,
                                  const float* d_base_f32, const int64_t* d_base_i64,
                                  float* d_out_f32, float* d_out_i64f,
                                  size_t n_f32, size_t n_i64, hipStream_t stream);

/* One client's deltas: out = x - base (fp32), and exact int64 x - base. */
int plato_agg_compute_deltas(const float* d_x_f32, const int64_t* d_x_i64,
                             const float* d_base_f32, const int64_t* d_base_i64,
                             float* d_out_f32, int64_t* d_out_i64,
                             size_t n_f32, size_t n_i64, hipStream_t stream);

/* update_weights: out = base + avg (fp32; int64 base converted to fp32). */
int plato_agg_update_weights(const float* d_base_f32, const int64_t* d_base_i64,
                             const float* d_avg_f32, const float* d_avg_i64f,
                             float* d_out_f32, float* d_out_i64f,
                             size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * load_state_dict's fp32 -> int64 copy: truncation toward zero; NaN and
 * values outside [-2^63, 2^63) give INT64_MIN (the x86-64 conversion result
 * the reference CPU path produces).
 */
int plato_agg_cast_f32_i64(const float* d_src, int64_t* d_dst, size_t n,
                           hipStream_t stream);

/*
 * FedAsync mixing: out = fp32(b * fp32(1 - m)) + fp32(x * fp32(m)), computed
 * as the reference does with two fp32 scalars one_minus_m and m.
 */
int plato_agg_mix_weights(const float* d_x_f32, const int64_t* d_x_i64,
                          const float* d_base_f32, const int64_t* d_base_i64,
                          float one_minus_m, float m,
                          float* d_out_f32, float* d_out_i64f,
                          size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * Per-client model-wide reductions (Port cosine similarity, norms) over the
 * whole arena, int64 entries included as torch.cat promotes them (fp32):
 *   d_i = x_i - base (fp32, as compute_weight_deltas; int64: fp32(x - b)),
 *         or x_i if d_base is NULL
 *   d_out[i]     = sum_e d_i[e] * v[e]         (0 <= i < K)
 *   d_out[K + i] = sum_e d_i[e]^2
 *   d_out[2K]    = sum_e v[e]^2                (v's int64 entries as fp32)
 * accumulated in fp64 in a fixed order (bitwise reproducible run to run; it
 * matches torch's fp32 CPU reductions within tolerance, not bit for bit).
 * d_workspace must hold plato_agg_client_dots_workspace(K, n_f32) bytes.
 */
size_t plato_agg_client_dots_workspace(int K, size_t n_f32);
int plato_agg_client_dots(const float* const* d_x, const int64_t* const* d_x_i64, int K,
                          const float* d_base, const int64_t* d_base_i64,
                          const float* d_v, const int64_t* d_v_i64,
                          size_t n_f32, size_t n_i64, double* d_workspace,
                          double* d_out, hipStream_t stream);

/*
 * Per-entry work: a state_dict entry ("tensor") is a contiguous element range
 * of the fp32 or the int64 arena.  Kernels that need the entry of an element
 * read a chunk table: each chunk is a piece of ONE entry, [begin, end) in
 * elements of its region, numbered with the entry's index `entry` in the
 * layout (0 <= entry < n_entries, across both regions).  Chunks of the same
 * entry are contiguous and the tables are sorted by entry (host-built once
 * per layout: plato_amd/arena.py ArenaLayout.chunk_tables).  Chunk length
 * sets the work per workgroup; any length is correct.
 */
typedef struct plato_agg_chunk {
  uint32_t entry;
  uint32_t begin;
  uint32_t end;
  uint32_t reserved;
} plato_agg_chunk;

/*
 * Per (client, entry) reductions, accumulated in fp64 in a fixed order:
 *   d_i = x_i - base (fp32; int64 entries: fp32(int64 x - b)), or x_i if d_base is NULL
 *   d_out[i * E + e]           = sum_{elements of e} d_i * v     (0 <= i < K; 0 if d_v is NULL)
 *   d_out[(K + i) * E + e]     = sum d_i^2
 *   d_out[2K * E + e]          = sum v^2                         (0 if d_v is NULL)
 * v is an fp32 arena (its int64 entries given as fp32 in d_v_i64f).
 * d_workspace must hold plato_agg_entry_stats_workspace(K, n_chunks_f32 + n_chunks_i64) bytes.
 */
size_t plato_agg_entry_stats_workspace(int K, uint32_t n_chunks);
int plato_agg_entry_stats(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                          const float* d_base_f32, const int64_t* d_base_i64,
                          const float* d_v_f32, const float* d_v_i64f,
                          const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                          const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                          int n_entries, size_t n_f32, size_t n_i64,
                          double* d_workspace, double* d_out, hipStream_t stream);

/*
 * Weighted sum with a weight per (entry, client), bit-exact with torch's fp32
 * CPU ops:
 *   d_i = x_i - b (as above), or x_i if d_base is NULL
 *   acc = +0; for i in order: acc = acc + fp32(d_i * W[e * K + i])
 *   u   = fp32(acc * scale); if d_noise: u = fp32(u + fp32(noise * noise_scale))
 *   out = (flags & PLATO_AGG_ADD_BASE) ? fp32(b + u) : u      (int64 b: fp32(b) + u)
 * FedAtt: W = -softmax(norms), scale = -epsilon, noise = torch.randn draws,
 * noise_scale = magnitude, ADD_BASE (update_weights).  d_base is required
 * with ADD_BASE.  Alignment: base/out/noise fp32 arrays 16-byte aligned.
 */
#define PLATO_AGG_ADD_BASE 1
int plato_agg_fedavg_entrywise(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                               const float* d_w, int n_entries,
                               const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                               const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                               const float* d_base_f32, const int64_t* d_base_i64,
                               const float* d_noise_f32, const float* d_noise_i64f,
                               float scale, float noise_scale, int flags,
                               float* d_out_f32, float* d_out_i64f,
                               size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * torch.linalg.norm of every (client, entry) delta, in x86-64 PyTorch's CPU
 * order (ATen's vectorised 2-norm: 8 fp32 lanes of fma(v, v, acc) over the
 * first n - n%8 elements, lanes added in order, tail fma'd, fp32 sqrt), so
 * the fp32 result equals the reference's bit for bit:
 *   d_out[i * n_entries + entry] = norm(d_i restricted to entry)
 * d_entries_* hold ONE piece per entry (ArenaLayout.chunk_tables(2**32)), in
 * any order: the table order is the dispatch order, and since each norm is one
 * serial chain, passing the longest entries first shortens the launch (the
 * engine does, FedAvgEngine._norm_tables).
 * FedAtt: examples/server_aggregation/fedatt/fedatt_algorithm.py:34-39.
 */
int plato_agg_entry_norms_f32(const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                              const float* d_base_f32, const int64_t* d_base_i64,
                              const plato_agg_chunk* d_entries_f32, uint32_t n_entries_f32,
                              const plato_agg_chunk* d_entries_i64, uint32_t n_entries_i64,
                              int n_entries, size_t n_f32, size_t n_i64, float* d_out,
                              hipStream_t stream);

/*
 * FedAvg over QSGD-coded payloads (one byte per element: bit 7 sign, bits
 * 0-6 |zeta|; one max_v per (entry, client)), decoded exactly as
 * model_dequantize_qsgd.py:51-58 does before the FedAvg chain:
 *   x   = fp32(fp32(fp32(zeta) * max_v[entry * K + i]) / divisor)   (divisor = level - 1)
 *   d   = x - b   (int64 entries: x - fp32(b)),  t = fp32(d * w_i) [* s_i],  acc += t
 *   out = fp32(b + acc)     (int64 entries: fp32(b) + acc)
 * d_codes_* are K device pointers to byte arenas laid out like the fp32 /
 * int64 regions (element e <-> byte e), 16-byte aligned.  Chunk tables as
 * for plato_agg_fedavg_entrywise (pieces of <= 4096 elements run one pass).
 */
int plato_agg_fedavg_qsgd(const uint8_t* const* d_codes_f32, const uint8_t* const* d_codes_i64, int K,
                          const float* d_max_v, int n_entries, float divisor,
                          const float* d_w, const float* d_s,
                          const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                          const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                          const float* d_base_f32, const int64_t* d_base_i64,
                          float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64,
                          hipStream_t stream);

/*
 * Deterministic synthetic payloads for tests and benchmarks (a counter-based
 * generator restated bit for bit by oracle/synth.py):
 *   h = splitmix64(splitmix64(seed ^ (stream * 0xD1B54A32D192ED03)) + e)
 *   r = (int32)(h >> 40) - 2^23
 *   out[e] = (d_add ? d_add[e] : +0) + (float)r * 2^scale_log2   (fp32 add)
 */
int plato_agg_fill_synth_f32(float* d_out, const float* d_add, size_t n,
                             uint64_t seed, uint64_t stream_id, int scale_log2,
                             hipStream_t stream);

/*   out[e] = (d_add ? d_add[e] : 0) + (int64)(h % modulus)   (modulus >= 1) */
int plato_agg_fill_synth_i64(int64_t* d_out, const int64_t* d_add, size_t n,
                             uint64_t seed, uint64_t stream_id, uint64_t modulus,
                             hipStream_t stream);

/*
 * The same streams from element ``first`` on: out[e] is element first + e of
 * the stream (h = splitmix64(key + first + e)) and d_add[e] its addend.  A
 * rank of the bucket-sharded bench fills its pieces as slices of the one
 * global model and client set this way (bench.py, N > 1).
 */
int plato_agg_fill_synth_f32_at(float* d_out, const float* d_add, size_t n,
                                uint64_t seed, uint64_t stream_id, uint64_t first,
                                int scale_log2, hipStream_t stream);
int plato_agg_fill_synth_i64_at(int64_t* d_out, const int64_t* d_add, size_t n,
                                uint64_t seed, uint64_t stream_id, uint64_t first,
                                uint64_t modulus, hipStream_t stream);

/*
 * FedAvg with float64 weights on the fp32 entries (ABI 2): for every fp32
 * element, clients in order,
 *   d = x_i - b (fp32; d = x_i when d_base_* are NULL: deltas mode)
 *   acc = fp32( double(acc) + double(d) * d_w64[i] )      (one double rounding
 *         for the product, one for the sum, then the cast: torch's in-place add
 *         of a float64 tensor into an fp32 one)
 *   new = fp32(b + acc)            (deltas mode: acc)
 * and for the int64 entries the fp32 chain with d_w_i64[i] (fp32):
 *   acc = acc + fp32(fp32(x_i - b) * w_i64),  new = fp32(b) + acc.
 * Replaces the RL server's smart weighting (plato/utils/reinforcement_learning/
 * rl_server.py:66-71: `delta * smart_weighting[i]` with a float64 [K, 1]
 * action for the fp32 entries, `delta * smart_weighting[i][0]` for the int64
 * ones).  Arena < 4 GiB per call.
 */
int plato_agg_fedavg_w64(const float* const* d_x_f32, const int64_t* const* d_x_i64, const double* d_w64,
                         const float* d_w_i64, int K, const float* d_base_f32, const int64_t* d_base_i64,
                         float* d_out_f32, float* d_out_i64f, size_t n_f32, size_t n_i64, hipStream_t stream);

/*
 * float64 weighted sum of K float64 vectors (16-byte aligned):
 *   out[e] = (((0 + x_0[e]*w_0) + x_1[e]*w_1) + ...)   float64, separately rounded.
 * The plaintext half of HE hybrid FedAvg (plato/servers/fedavg_he.py:88-98):
 * the unencrypted weights are float64 numpy vectors (homo_enc.py:50-63), so
 * `unencrypted_avg_update += unenc_w * (n_i / N)` runs in numpy float64 and
 * turns the fp32 zeros into a float64 accumulator.
 */
int plato_agg_weighted_sum_f64(const double* const* d_x, const double* d_w, int K, double* d_out, size_t n,
                               hipStream_t stream);

/*
 * Flattened-model reductions of the variant servers, in the reference's own
 * float32 order (bit-exact; CPU restatements in oracle/reductions.c).
 *
 * plato_agg_flatten writes K flat fp32 vectors: position p of vector k lies in
 * segment s (the last with flat_offset <= p), element e = src_offset +
 * (p - flat_offset) of its region, and is
 *   PLATO_AGG_FLAT_DELTA      fp32: x_k[e] - b[e];   int64: fp32(x_k[e] - b[e])
 *   PLATO_AGG_FLAT_CAST_DIFF  fp32: x_k[e] - b[e];   int64: fp32(x_k[e]) - fp32(b[e])
 *   PLATO_AGG_FLAT_RAW        fp32: x_k[e];          int64 region given as fp32 values
 * and, with PLATO_AGG_SEG_NEG_DIV, (-v) / lr instead (int64 deltas: the int64
 * negation, then the cast and the division).  Port concatenates the entries in
 * state_dict order (examples/async/port/port_server.py:36-48, CAST_DIFF for
 * current - previous, DELTA for the update); FedAdp sorts them by name.lower()
 * and divides all but the first by -lr (examples/server_aggregation/fedadp/
 * fedadp_server.py:122-133, RAW for the global gradient, DELTA for a client).
 * d_src_*: K device pointers; d_out: K device pointers to n_flat floats.
 */
typedef struct plato_agg_segment {
  uint64_t flat_offset;
  uint64_t src_offset;
  uint64_t numel;
  uint32_t region;  /* 0: fp32 region, 1: int64 region */
  uint32_t flags;   /* PLATO_AGG_SEG_NEG_DIV */
} plato_agg_segment;
#define PLATO_AGG_FLAT_DELTA 0
#define PLATO_AGG_FLAT_CAST_DIFF 1
#define PLATO_AGG_FLAT_RAW 2
#define PLATO_AGG_SEG_NEG_DIV 1u
int plato_agg_flatten(int mode, const void* const* d_src_f32, const void* const* d_src_i64, int K,
                      const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
                      uint32_t n_segs, size_t n_flat, float lr, float* const* d_out, hipStream_t stream);

/*
 * numpy's float32 np.inner(x_j, y_j) (and y_j . y_j if d_out_yy) for n_pairs
 * pairs of flat vectors, in the order of numpy's bundled OpenBLAS 0.3.29
 * sdot_k_SKYLAKEX (the x86-64 AVX-512 kernel; cblas_sdot calls it unthreaded):
 * FedAdp's inner products and norms (fedadp_server.py:95-99; np.linalg.norm
 * is sqrt of the float32 self dot).  Vectors 16-byte aligned.
 */
int plato_agg_sdot_pairs(const float* const* d_x, const float* const* d_y, int n_pairs, size_t n,
                         float* d_out_xy, float* d_out_yy, hipStream_t stream);

/*
 * The same sdot_k_SKYLAKEX results (bitwise equal to plato_agg_sdot_pairs) for
 * pairs that share x: FedAdp's np.inner(g, loc_k) and loc_k . loc_k for every
 * client (fedadp_server.py:91-99); with with_xx = 1 also g . g, written to
 * d_out_xy[n_pairs] and d_out_yy[n_pairs].  The 64 chains are split over
 * workgroups and each workgroup reads x once for its pairs; d_workspace holds
 * plato_agg_sdot_shared_workspace(n_pairs, with_xx) bytes of chain partials.
 * x 16-byte aligned; y rows any float alignment.
 */
size_t plato_agg_sdot_shared_workspace(int n_pairs, int with_xx);
int plato_agg_sdot_shared(const float* d_x, const float* const* d_y, int n_pairs, size_t n, int with_xx,
                          float* d_workspace, float* d_out_xy, float* d_out_yy, hipStream_t stream);

/*
 * FedAdp's dots straight from the staged arenas, bit-equal to plato_agg_flatten
 * (PLATO_AGG_FLAT_DELTA with the segment map) followed by plato_agg_sdot_shared,
 * without the flattened copies: process_grad(update) positions are gathered
 * through d_segs (flat order: entries sorted by name.lower(), NEG_DIV on all but
 * the first) from client k's arenas d_src_f32[k] / d_src_i64[k] and the baseline
 * (loc = x - b, or -(x - b) / lr), and d_out_xy[k] = np.inner(x, loc_k),
 * d_out_yy[k] = loc_k . loc_k in numpy's OpenBLAS sdot_k_SKYLAKEX order
 * (examples/server_aggregation/fedadp/fedadp_server.py:91-99, 122-133).  d_x is
 * the flattened global gradient (plato_agg_flatten RAW, 16-byte aligned, at
 * least n_flat rounded up to 64 floats); with_xx = 1 also writes x . x to
 * d_out_xy[n_pairs] and d_out_yy[n_pairs].  Segments: 1 .. 2^22 - 1 (ABI 3: no
 * longer capped at 2048 entries), n_flat < 2^30, n_pairs <= 65535; n_f32 / n_i64 =
 * lengths of the arenas' fp32 (< 2^30) and int64 regions.  d_workspace (256-byte
 * aligned): plato_agg_fedadp_dots_workspace(n_pairs, with_xx, n_i64, n_flat,
 * n_segs) bytes — chain sums, per-group descriptors, the finished values of
 * the groups that cross an entry boundary and the chain-group-major copy of x
 * and the flattened baseline the kernel streams.
 * Delta arenas: d_base_f32 = d_base_i64 = NULL means the client arenas already
 * hold x - b (fp32 differences, int64 wrapping differences: compute_weight_deltas,
 * plato/algorithms/fedavg.py:13-27, formed when each payload was staged); the
 * values and their order are the same, and the kernel streams no baseline.
 */
size_t plato_agg_fedadp_dots_workspace(int n_pairs, int with_xx, size_t n_i64, size_t n_flat, uint32_t n_segs);
int plato_agg_fedadp_dots(const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64, int n_pairs,
                          const float* d_base_f32, const int64_t* d_base_i64, const plato_agg_segment* d_segs,
                          uint32_t n_segs, size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace,
                          float* d_out_xy, float* d_out_yy, hipStream_t stream);

/*
 * plato_agg_fedadp_dots with flags (ABI 4).  PLATO_AGG_FEDADP_TABLES_READY: d_workspace
 * already holds the layout-only tables (per-group descriptors, boundary rows and their
 * source positions) of an earlier call with the same d_segs contents, n_segs, n_flat,
 * n_i64, n_pairs and with_xx, completed on or ordered before `stream`; they depend on
 * the segment map only, so a server whose layout is unchanged between rounds builds
 * them once (replaces nothing in the reference: the same dots as plato_agg_fedadp_dots,
 * examples/server_aggregation/fedadp/fedadp_server.py:91-99).  flags = 0 is
 * plato_agg_fedadp_dots.
 */
#define PLATO_AGG_FEDADP_TABLES_READY 1
int plato_agg_fedadp_dots_ex(const float* d_x, const void* const* d_src_f32, const void* const* d_src_i64,
                             int n_pairs, const float* d_base_f32, const int64_t* d_base_i64,
                             const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat, size_t n_f32,
                             size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy, float* d_out_yy,
                             hipStream_t stream, int flags);

/*
 * Port's vector norms gathered from the arenas (replaces the flatten + norm of
 * examples/async/port/port_server.py:38-50: torch.cat in state_dict order, then
 * the norms inside F.cosine_similarity).  Vector v is x_v - b_v flattened by
 * the segment map (state_dict order; int64 entries cast to float32 as
 * torch.cat does: the wrapped int64 difference cast once, or with
 * PLATO_AGG_PORT_CAST_FIRST for vector 0, current - previous, the difference
 * of the two casts); d_out[v] = torch.linalg.vector_norm of it in x86-64
 * ATen's order (8 fma chains over n - n % 8 positions, the lanes added in
 * order, the scalar tail).  d_x_f32 / d_x_i64 / d_b_f32 / d_b_i64: n_vectors
 * device pointers each (arenas of n_f32 fp32 elements / the int64 counters).
 * d_flat_out: null, or n_vectors 16-byte aligned rows of >= n_flat floats that
 * receive the flattened vectors (what plato_agg_torch_cosine_sum then reads).
 * d_lengths: null, or n_vectors lengths <= n_flat, vector v taking only its
 * first d_lengths[v] positions (FedAtt's per-(entry, client) norms,
 * fedatt_algorithm.py:34-39: one fp32 entry of one client per vector, the
 * pointers offset to the entry and one segment covering it).  A null
 * d_b_f32[v] (and d_b_i64[v]) means vector v's arenas already hold the
 * difference (delta arenas): nothing is subtracted, the same values result.
 */
#define PLATO_AGG_PORT_CAST_FIRST 1
int plato_agg_port_norms(const void* const* d_x_f32, const void* const* d_x_i64, const void* const* d_b_f32,
                         const void* const* d_b_i64, int n_vectors, const uint32_t* d_lengths,
                         const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat, size_t n_f32, int flags,
                         float* d_out, float* const* d_flat_out, hipStream_t stream);

/*
 * The sum in Port's F.cosine_similarity(a, b_k, dim=0) (port_server.py:50),
 * as x86-64 PyTorch 2.10 forms it on `threads` CPU threads:
 *   q = (a / max(|a|, eps)) * (b_k / max(|b_k|, eps)),  out[k] = sum(q)
 * in TensorIterator's two-pass order (min(threads, ceil(n/32768)) chunks;
 * one pass below 32768 elements or on one thread), each chunk by ATen's
 * cascade sum.  |a|, |b_k|: device floats, e.g. plato_agg_entry_norms_f32 of
 * the flat vectors with no baseline (torch.linalg.vector_norm's order).
 * d_workspace: plato_agg_torch_cosine_workspace(K, threads) bytes.
 */
size_t plato_agg_torch_cosine_workspace(int K, int threads);
int plato_agg_torch_cosine_sum(const float* d_a, const float* const* d_b, int K, size_t n, const float* d_norm_a,
                               const float* d_norm_b, float eps, int threads, void* d_workspace, float* d_out,
                               hipStream_t stream);

/*
 * plato_agg_torch_cosine_sum with a already divided by its clamped norm
 * (F.cosine_similarity's x1 / x1_norm, the same fp32 quotients: one division
 * per element and client instead of two).  plato_agg_scale_by_norm forms it:
 * d_out[i] = d_a[i] / max(*d_norm, eps) (NaN norms stay NaN).
 */
int plato_agg_torch_cosine_sum_scaled(const float* d_a_scaled, const float* const* d_b, int K, size_t n,
                                      const float* d_norm_b, float eps, int threads, void* d_workspace, float* d_out,
                                      hipStream_t stream);
int plato_agg_scale_by_norm(const float* d_a, size_t n, const float* d_norm, float eps, float* d_out,
                            hipStream_t stream);

/*
 * numpy's float32 np.sum(np.square(x_k - b)) of each fp32 piece (one per
 * entry, d_pieces rows (entry, begin, end)): the ufunc reduction's 8192-element
 * inner loops, out += pairwise_sum(chunk) from 0, pairwise_sum as numpy's
 * (8 partial sums up to 128 elements, halved at multiples of 8 above).
 * Polaris' per-layer squared deltas (examples/client_selection/polaris/
 * polaris_server.py:78-81).  d_first_chunk[p] = sum over earlier pieces of
 * ceil(len / 8192); n_chunks the total.  d_out: [K][n_pieces] floats.
 * d_workspace: plato_agg_np_sumsq_workspace(K, n_chunks) bytes (the per-chunk sums).
 */
size_t plato_agg_np_sumsq_workspace(int K, uint32_t n_chunks);
int plato_agg_np_sumsq(const float* const* d_x, int K, const float* d_base, const plato_agg_chunk* d_pieces,
                       const uint32_t* d_first_chunk, uint32_t n_pieces, uint32_t n_chunks, void* d_workspace,
                       float* d_out, hipStream_t stream);

/*
 * Coded client payloads (or the baseline) as fp32 rows of the "promoted"
 * layout, for the variant servers' per-entry reductions: what the reference's
 * inbound dequantizers hand the server (plato/processors/model_dequantize.py:
 * 15-18, model_dequantize_qsgd.py:34-60), every entry float32 — the int64
 * counters included, so a counter's delta is float32(x) - float32(b).
 *   PLATO_AGG_DECODE_NATIVE  fp32 copied, int64 cast to fp32 (RNE)
 *   PLATO_AGG_DECODE_BF16    bf16 widened (exact), both regions
 *   PLATO_AGG_DECODE_QSGD    fp32(fp32(fp32(zeta) * max_v[entry][k]) / divisor)
 * Element e of the fp32 region lands at d_dst[k][e], element e of the int64
 * region at d_dst[k][i64_dst_offset + e]; pieces from d_chunks_* (entry, begin,
 * end); d_max_v: [n_entries][K] (QSGD only).
 */
#define PLATO_AGG_DECODE_NATIVE 0
#define PLATO_AGG_DECODE_BF16 1
#define PLATO_AGG_DECODE_QSGD 2
int plato_agg_decode_rows(int codec, const void* const* d_src_f32, const void* const* d_src_i64, int K,
                          const float* d_max_v, float divisor, const plato_agg_chunk* d_chunks_f32,
                          uint32_t n_chunks_f32, const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64,
                          size_t i64_dst_offset, float* const* d_dst, hipStream_t stream);

/*
 * Single-process RCCL communicator over the GPUs one Plato server drives.
 * The reference has no collectives (aggregation runs on one CPU
 * process); these serve the multi-GPU engine behind the same
 * aggregate_weights hook (plato/servers/fedavg.py:171-182), which bucket-
 * shards the arena over the node's GPUs.  Rank g is
 * devices[g]; every collective is issued for all ranks inside one
 * ncclGroupStart/End, each on its own stream (streams[g] on devices[g]).
 * RCCL is bound at run time (dlopen "librccl.so.1"): PLATO_AGG_ERCCL if absent.
 */
typedef struct plato_agg_comm plato_agg_comm;

/* ncclCommInitAll over `ndev` distinct device ordinals. */
int plato_agg_comm_create(int ndev, const int* devices, plato_agg_comm** out);
int plato_agg_comm_destroy(plato_agg_comm* comm);
int plato_agg_comm_size(const plato_agg_comm* comm);

/* d_recv[g][r*count .. (r+1)*count) = d_send[r][0 .. count) for every rank r:
 * assembles the bucket-sharded new model on every GPU. */
int plato_agg_comm_allgather_f32(plato_agg_comm* comm, const float* const* d_send, float* const* d_recv,
                                 size_t count, const hipStream_t* streams);

/* d_recv[g][0 .. count) = sum over ranks r of d_send[r][g*count .. (g+1)*count)
 * (client-sharded tolerance mode: per-GPU partial weighted sums -> bucket g). */
int plato_agg_comm_reduce_scatter_f32(plato_agg_comm* comm, const float* const* d_send, float* const* d_recv,
                                      size_t count, const hipStream_t* streams);

#ifdef __cplusplus
}
#endif

#endif /* PLATO_AGG_H */
