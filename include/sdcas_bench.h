/*
 * sdcas_bench.h — benchmark / test plumbing exported by libsdcas.so next to
 * the sdcas.h boundary: device generators of the synthetic corpora
 * (include/sdcas_synth.h). Not part of the reference interface.
 */
#ifndef SDCAS_BENCH_H
#define SDCAS_BENCH_H
#include <stddef.h>
#include <stdint.h>

#include "sdcas.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cas_id messages of synthetic files (content key, size) written at device
 * offsets d_offs (16-byte aligned) of d_blob. */
int sdcas_dev_synth_cas_messages(sdcas_ctx *ctx, const uint64_t *d_keys, const uint64_t *d_sizes,
                                 const uint64_t *d_offs, size_t n, uint8_t *d_blob, void *stream);
/* raw content ranges [d_starts[i], +d_lens[i]) of content streams d_keys[i]. */
int sdcas_dev_synth_content(sdcas_ctx *ctx, const uint64_t *d_keys, const uint64_t *d_starts,
                            const uint64_t *d_lens, const uint64_t *d_offs, size_t n, uint8_t *d_blob,
                            void *stream);
/* device-resident dedup of a whole job in file order, no existing Objects
 * (keys etc. are device pointers; d_counts: 2 x u64, overwritten): the
 * single-rank path of sdcas_dev_dedup_local with ids 0..n-1. */
int sdcas_dev_dedup(sdcas_ctx *ctx, const uint64_t *d_keys, const uint8_t *d_has_key,
                    const int32_t *d_status, size_t n, size_t chunk_size, int64_t *d_out_link,
                    uint64_t *d_counts, void *stream);
/* With profiling enabled (sdcas_dev_profile(ctx, 1), which also clears the
 * record), every batch launch records HIP events on its own stream around the
 * leaf/tree kernel and around the whole launch sequence;
 * sdcas_dev_last_kernel_ms returns the MEAN milliseconds of each over all
 * launches recorded since (it synchronises on the events). */
int sdcas_dev_profile(sdcas_ctx *ctx, int enable);
int sdcas_dev_last_kernel_ms(sdcas_ctx *ctx, float *leaf_ms, float *total_ms);

/* Tuning: select the leaf/tree kernel variant (-1 = default). Returns
 * SDCAS_OK, or SDCAS_E_INVALID (selection unchanged) for a variant this
 * build does not hold: libsdcas.so holds only the bit-exact product kernels;
 * the ablation build (libsdcas_ablate.so, tools only) holds all of them. */
int sdcas_dev_set_leaf_variant(sdcas_ctx *ctx, int variant);
/* Tuning: select the 1 MiB-piece kernel variant of the checksum path (-1 =
 * default); same return convention. */
int sdcas_dev_set_piece_variant(sdcas_ctx *ctx, int variant);
/* Tuning: hash messages in length-sorted slot order (1, default) or in caller
 * order (0). Results are identical either way. */
int sdcas_dev_set_sort(sdcas_ctx *ctx, int enable);

#ifdef __cplusplus
}
#endif
#endif
