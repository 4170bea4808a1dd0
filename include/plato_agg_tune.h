/*
 * plato_agg_tune.h — benchmarking / tuning entry points of libplato_agg_tune.so.
 *
 * libplato_agg_tune.so is built from the same sources as libplato_agg.so with
 * -DPLATO_AGG_TUNE: it carries every kernel variant and these exports besides
 * the plato_agg.h entry points.  The product library carries only the default
 * variants and does not export these.
 *
 * Not part of the drop-in boundary (no reference interface behind them):
 * bench.py and the tuning sweep use them to time the kernel variants
 * (V float4 per lane, U clients unrolled, non-temporal loads) that the
 * public entry points choose between.  Same argument conventions and
 * arithmetic contract as plato_agg_fedavg_weights / _deltas in plato_agg.h.
 */
#ifndef PLATO_AGG_TUNE_H
#define PLATO_AGG_TUNE_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#include "plato_agg.h"

#ifdef __cplusplus
extern "C" {
#endif

int plato_agg_tune_num_variants(void);

// Largest fp32 range (in groups of 4 elements) one FedAvg launch covers;
// 0 restores the default (the 4 GiB reach of 32-bit lane offsets).  Arenas
// above it run as consecutive launches.  Tests lower it to exercise the split
// on small arenas; process-wide, not thread-safe against concurrent launches.
void plato_agg_tune_set_launch_groups(uint64_t groups);

/* Writes the variant's workgroup size, V (float4 per lane), U (clients per
 * batch) and flags: bit 0 non-temporal loads, bit 1 non-temporal stores,
 * bit 2 software-pipelined batches, bit 3 buffer loads, bits 4..11 persistent
 * workgroups per CU (0 = one workgroup per chunk), bit 12 XCD-contiguous chunk
 * order (each of the 8 XCDs streams one contiguous eighth of the arena), bit 13
 * balanced grid (occupancy x CUs workgroups, one equal contiguous share each). */
int plato_agg_tune_describe(int variant, int* block, int* v, int* u, int* flags);

/* has_base != 0: plato_agg_fedavg_weights; == 0: plato_agg_fedavg_deltas. */
int plato_agg_tune_fedavg(int variant, int has_base,
                          const float* const* d_x_f32,
                          const int64_t* const* d_x_i64,
                          const float* d_w, const float* d_s, int K,
                          const float* d_base_f32, const int64_t* d_base_i64,
                          float* d_out_f32, float* d_out_i64f,
                          size_t n_f32, size_t n_i64, hipStream_t stream);

/* Threads per plato_agg_fedavg_entrywise workgroup: 64, 128 or 256 (0 restores the default, 64; any
 * other value too).  Process-wide, for A/B timings of the tuning library's entry point. */
void plato_agg_tune_set_entrywise_block(int threads);

/* bf16-payload kernel variants (plato_agg_fedavg_weights_bf16 uses 0). */
int plato_agg_tune_num_bf16_variants(void);
int plato_agg_tune_fedavg_bf16(int variant, const uint16_t* const* d_x_bf16,
                               const uint16_t* const* d_x_i64_bf16,
                               const float* d_w, const float* d_s, int K,
                               const float* d_base_f32, const int64_t* d_base_i64,
                               float* d_out_f32, float* d_out_i64f,
                               size_t n_f32, size_t n_i64, hipStream_t stream);

/* Ceiling probes: mode 0 = non-temporal copy src -> dst, mode 1 = non-temporal
 * read of src only; n fp32 elements (n % 4 == 0), `blocks` workgroups of 256
 * grid-striding (<= 0: 2048).  bench.py --sweep reports them as the measured
 * streaming ceilings of the device next to the FedAvg kernel variants. */
int plato_agg_tune_stream(int mode, const float* d_src, float* d_dst, size_t n,
                          int blocks, hipStream_t stream);

/* plato_agg_entry_norms_f32 kernel variants (bitwise identical results; csrc/entrywise.hip), one
 * workgroup per (entry, client):
 *   0 = register-staged producer / consumer (the default): 2 producer waves hold 2 tiles of x and b
 *       (2,048 elements) in VGPRs and write the delta tiles transposed into a two-slot LDS ring, the
 *       chain wave walks the 8 chains (the long entries' chains at s_setprio 3)
 *   1 = variant 0 with one producer wave; 2 = with 3 tiles in flight and the long entries' producers
 *       at s_setprio 2
 *   3, 4 = the round-3 defaults: one producer wave streams x and b into an LDS-DMA ring
 *       (1,024-element tiles x 5 stages / 2,048 x 3)
 *   5 = one wavefront per (entry, client), one-tile register prefetch (the first version) */
int plato_agg_tune_num_entry_norms_variants(void);
int plato_agg_tune_entry_norms(int variant, const float* const* d_x_f32, const int64_t* const* d_x_i64, int K,
                               const float* d_base_f32, const int64_t* d_base_i64,
                               const plato_agg_chunk* d_entries_f32, uint32_t n_entries_f32,
                               const plato_agg_chunk* d_entries_i64, uint32_t n_entries_i64, int n_entries,
                               size_t n_f32, size_t n_i64, float* d_out, hipStream_t stream);

/* plato_agg_sdot_shared kernel variants (pairs per workgroup x chains per workgroup x 64-element
 * blocks per stage x ring stages x producer waves): 0 = 4x16x64x6x4, 1 = 2x16x64x6x4,
 * 2 = 1x16x64x4x2, each with a pair group's chain groups on one XCD (one L2); 3 = variant 0
 * without the XCD grouping.  plato_agg_sdot_shared runs 1 (with_xx, <= 128 pairs), 2 (with_xx,
 * <= 64 pairs) or 0.  Bitwise identical results. */
int plato_agg_tune_num_sdot_shared_variants(void);
int plato_agg_tune_sdot_shared(int variant, const float* d_x, const float* const* d_y, int n_pairs, size_t n,
                               int with_xx, float* d_workspace, float* d_out_xy, float* d_out_yy,
                               hipStream_t stream);

/* plato_agg_fedavg_qsgd kernel variants, workgroup size x clients per decode-table batch x
 * elements per lane: 0 = 512x8x8 plain form (two barriers per table batch, max_v by scalar loads,
 * the batch's codes issued before its table build; plato_agg_fedavg_qsgd), 1 = 512x4x8 pipelined
 * (double-buffered tables, the next batch's codes loaded before the current batch is summed; the
 * rounds 2-3 default), 2-4 = timing probes of variant 1 (NOT the FedAvg: no code loads / no table
 * lookups / neither), 5 = 1024x8x8 plain form of round 1, 6 = variant 0 at 256 threads.
 * plato_agg_tune_qsgd_chunk gives the chunk capacity (elements per workgroup pass) the variant is
 * built for. */
int plato_agg_tune_num_qsgd_variants(void);
int plato_agg_tune_qsgd_chunk(int variant);
int plato_agg_tune_fedavg_qsgd(int variant, const uint8_t* const* d_codes_f32, const uint8_t* const* d_codes_i64,
                               int K, const float* d_max_v, int n_entries, float divisor, const float* d_w,
                               const float* d_s, const plato_agg_chunk* d_chunks_f32, uint32_t n_chunks_f32,
                               const plato_agg_chunk* d_chunks_i64, uint32_t n_chunks_i64, const float* d_base_f32,
                               const int64_t* d_base_i64, float* d_out_f32, float* d_out_i64f, size_t n_f32,
                               size_t n_i64, hipStream_t stream);

/* plato_agg_fedadp_dots with an explicit tile shape (0 = the default; see csrc/fedadp.hip). */
int plato_agg_tune_num_fedadp_variants(void);
/* 1 if that variant is a timing probe (results wrong by design), else 0. */
int plato_agg_tune_fedadp_is_probe(int variant);
/* 1 if the variant runs on delta arenas (pass a null baseline), else 0 */
int plato_agg_tune_fedadp_is_delta(int variant);
int plato_agg_tune_fedadp_dots(int variant, const float* d_x, const void* const* d_src_f32,
                               const void* const* d_src_i64, int n_pairs, const float* d_base_f32,
                               const int64_t* d_base_i64, const plato_agg_segment* d_segs, uint32_t n_segs,
                               size_t n_flat, size_t n_f32, size_t n_i64, float lr, int with_xx, void* d_workspace, float* d_out_xy,
                               float* d_out_yy, hipStream_t stream);

/* plato_agg_np_sumsq with an explicit kernel (csrc/flat.hip): 0 = full chunks staged in two halves
 * with 16-byte loads plus a tail kernel for the partial last chunks (the default); 1 = the round-2
 * client-major kernel; 2, 3 = timing probes of variant 4 (wrong results by design: no baseline loads /
 * no LDS phase); 4 = the round-3 default (chunk-major, every chunk staged whole); 5 = the round-4
 * default (variant 0 with dword loads). */
int plato_agg_tune_num_np_sumsq_variants(void);
int plato_agg_tune_np_sumsq(int variant, const float* const* d_x, int K, const float* d_base,
                            const plato_agg_chunk* d_pieces, const uint32_t* d_first_chunk, uint32_t n_pieces,
                            uint32_t n_chunks, void* d_workspace, float* d_out, hipStream_t stream);

/* plato_agg_torch_cosine_sum_scaled with an explicit cascade form: 0 = two alternating LDS
 * buffers, one barrier per level-1 group (the default), 1 = one buffer, two barriers (round 3)
 * (csrc/flat.hip chunk_cascade).  Bitwise identical results. */
int plato_agg_tune_num_cosine_variants(void);
int plato_agg_tune_torch_cosine_sum_scaled(int variant, const float* d_a_scaled, const float* const* d_b, int K,
                                           size_t n, const float* d_norm_b, float eps, int threads,
                                           void* d_workspace, float* d_out, hipStream_t stream);

/* plato_agg_port_norms with an explicit shape (see csrc/port.hip). */
int plato_agg_tune_num_port_norms_variants(void);
int plato_agg_tune_port_norms(int variant, const void* const* d_x_f32, const void* const* d_x_i64,
                              const void* const* d_b_f32, const void* const* d_b_i64, int n_vectors,
                              const uint32_t* d_lengths, const plato_agg_segment* d_segs, uint32_t n_segs, size_t n_flat,
                              size_t n_f32, int flags, float* d_out, float* const* d_flat_out, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* PLATO_AGG_TUNE_H */
