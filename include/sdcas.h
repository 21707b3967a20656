/*
 * sdcas.h — C ABI of the MI355X content-identification engine (libsdcas.so).
 *
 * Drop-in boundary for sd-core's content identification. The
 * Rust host keeps its signatures and binds these entry points (cgo-style
 * `extern "C"`, plain pointers and sizes, no ownership transfer; binding shown
 * in INTEGRATION.md):
 *
 *   sdcas_cas_ids        replaces per-file generate_cas_id(path, size)
 *                        core/src/object/cas.rs:23-62, called from
 *                        core/src/object/file_identifier/mod.rs:78-82 (the
 *                        join_all of FileMetadata::new at mod.rs:105-147
 *                        becomes one call per chunk), non_indexed.rs:181,
 *                        location/manager/watcher/utils.rs:236-240
 *   sdcas_checksums      replaces file_checksum(path)
 *                        core/src/object/validation/hash.rs:11-25, called from
 *                        validation/validator_job.rs:154 and watcher/utils.rs:496
 *   sdcas_dedup          replaces the cas_id -> Object group-by/link of
 *                        file_identifier/mod.rs:149-254 (HashSet at :149-154,
 *                        existing-object lookup :181-188, linear find :214-224,
 *                        new Objects :246-254)
 *   sdcas_*_from_messages / sdcas_hash_messages / sdcas_dev_*
 *                        the same engine on pre-assembled messages (host or
 *                        device memory) for tests and benchmarks
 *
 * Conventions
 *   - Return value: SDCAS_OK (0) or a negative SDCAS_E_* library failure (no
 *     device, invalid arguments, out of memory, HIP error). On failure the
 *     caller falls back to its CPU path for the whole batch.
 *   - Per-item status (out_status): 0, a positive errno from the file I/O, or
 *     SDCAS_STATUS_UNEXPECTED_EOF when read_exact() ran out of file
 *     (cas.rs:36,43,56). The Rust side maps errno with
 *     io::Error::from_raw_os_error, reproducing the per-file skip of
 *     file_identifier/mod.rs:125-141.
 *   - cas keys: u64 whose big-endian bytes are digest bytes 0..7, so
 *     format!("{:016x}", key) == hasher.finalize().to_hex()[..16] (cas.rs:61).
 *     Digests: 32 bytes in BLAKE3 output order; lowercase hex of them is
 *     hash.rs:22-24's to_hex().
 *   - Ownership: the caller owns every input and output array; the library
 *     owns device memory, pinned staging and streams inside the context and
 *     retains no caller pointer after a call returns.
 *   - Threading: calls on one context serialise internally (a mutex on the
 *     host; on the device, a call's stream waits for the previous call's work
 *     whatever stream either names, because they share the context's device
 *     scratch). Use one context per concurrent job for parallelism; the path
 *     calls block, so wrap them in spawn_blocking.
 *   - Progress and cancellation (job/worker.rs:35-36,458-480 kill a job that
 *     reports no progress for 10 minutes; job/mod.rs:862-960 pause/cancel):
 *     the path calls (sdcas_cas_ids, sdcas_checksums, sdcas_hash_messages,
 *     sdcas_cas_ids_from_messages) call the context's progress function after
 *     every staging slot / 1 MiB-piece window completes, with bytes of input
 *     whose results are final, and stop at the next such point once the
 *     cancel flag reads nonzero, returning SDCAS_E_CANCELLED. sdcas_cas_ids
 *     and sdcas_checksums report per item: items already complete keep their
 *     results and status, every other item gets SDCAS_STATUS_CANCELLED. The
 *     two message calls have no per-item status: after SDCAS_E_CANCELLED
 *     their outputs are undefined. The progress function runs on the calling
 *     thread with the context's lock held: it must not call into the same
 *     context.
 *   - Limits: a batch holds at most SDCAS_MAX_BATCH (2^31 - 1) items.
 */
#ifndef SDCAS_H
#define SDCAS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDCAS_OK 0
#define SDCAS_E_NO_DEVICE (-1)
#define SDCAS_E_INVALID (-2)
#define SDCAS_E_OOM (-3)
#define SDCAS_E_HIP (-4)
#define SDCAS_E_CAPACITY (-5)
#define SDCAS_E_CANCELLED (-6)

#define SDCAS_STATUS_UNEXPECTED_EOF 100001
/* per-item status of an item the call did not complete because it was
 * cancelled (ECANCELED) */
#define SDCAS_STATUS_CANCELLED 125

#define SDCAS_MAX_BATCH 0x7FFFFFFF

/* constants of core/src/object/cas.rs:10-15 and validation/hash.rs:9 */
#define SDCAS_SAMPLE_COUNT 4
#define SDCAS_SAMPLE_SIZE 10240
#define SDCAS_HEADER_OR_FOOTER_SIZE 8192
#define SDCAS_MINIMUM_FILE_SIZE 102400
#define SDCAS_SAMPLED_MESSAGE_LEN 57352
#define SDCAS_CHECKSUM_BLOCK_LEN 1048576
/* file_identifier/mod.rs:34 */
#define SDCAS_IDENTIFIER_CHUNK_SIZE 100

typedef struct sdcas_ctx sdcas_ctx;

/* Progress report: `done` of `total` bytes of input have final results. Called
 * on the thread that made the path call. */
typedef void (*sdcas_progress_fn)(void *user, uint64_t done, uint64_t total);

/* sdcas_options.flags */
#define SDCAS_OPT_DIRECT_IO 1u /* the path calls (sdcas_cas_ids, sdcas_checksums) read files with
                                   O_DIRECT (cold storage: no page-cache copy; small and unaligned
                                   reads go through an aligned per-thread buffer); a file whose
                                   filesystem refuses O_DIRECT is read through the page cache.
                                   Same bytes, same statuses. */

typedef struct sdcas_options {
  uint32_t struct_size;    /* sizeof(sdcas_options) as the caller compiled it (SDCAS_OPTIONS_INIT sets it):
                              sdcas_init refuses any other size with SDCAS_E_INVALID, so a caller built
                              against another revision of this struct fails loudly instead of passing
                              garbage for the fields it lacks */
  int32_t device;          /* HIP device ordinal (-1: current device) */
  uint32_t io_threads;     /* reader threads of the path calls (0: 16, or the CPU count if lower; at most 256), started by the first one */
  uint32_t flags;          /* SDCAS_OPT_* */
  uint64_t staging_bytes;  /* pinned host staging per batch (0: 256 MiB) */
  sdcas_progress_fn progress;      /* may be NULL; runs on the calling thread and must not call back into
                                      the same context (its lock is held) */
  void *progress_user;             /* passed to progress */
  const volatile int32_t *cancel;  /* may be NULL; caller-owned, read atomically: nonzero cancels */
} sdcas_options;
#define SDCAS_OPTIONS_INIT {(uint32_t)sizeof(sdcas_options), -1, 0, 0, 0, NULL, NULL, NULL}

/* "sdcas-mi355x <major>.<minor>.<patch> (gfx950)"; the C ABI of this header is
 * SDCAS_ABI_VERSION (changes: 2 added sdcas_options.progress/cancel; 3 the
 * struct_size field, sdcas_dedup_window and the dedup step plan; 4
 * sdcas_dev_bind_stream; 5 the combine's output contract: one record per
 * distinct key, any order within an owner's range — same signatures, but a
 * caller that relied on ABI 4's documented key order must change; 6
 * sdcas_file_metadata, and resolve_buckets may overwrite the received
 * records' value words) */
#define SDCAS_ABI_VERSION 6
int sdcas_abi_version(void);
const char *sdcas_version(void);

/* Create / destroy a context bound to one GPU. opts may be NULL. */
int sdcas_init(const sdcas_options *opts, sdcas_ctx **out_ctx);
void sdcas_destroy(sdcas_ctx *ctx);
/* Text of the last library failure on this context ("" if none). */
const char *sdcas_last_error(const sdcas_ctx *ctx);
/* Re-bind the progress function and cancel flag (e.g. to the job now using
 * the context); any of them may be NULL. */
int sdcas_set_progress(sdcas_ctx *ctx, sdcas_progress_fn progress, void *user, const volatile int32_t *cancel);

/* ---- the reference functions, batched --------------------------------- */

/* cas_id of n files: generate_cas_id(paths[i], sizes[i]) (cas.rs:23-62).
 * sizes[i] is fs::metadata().len() as the identifier passes it (mod.rs:78-79);
 * it feeds the size prefix and the sample spacing, while file bytes come from
 * the file as it is now. out_keys[i] is valid iff out_status[i] == 0.
 * A small file (size <= 100 KiB) that has grown past its staging room when
 * read is read again with room for its new length, up to 4 times; one that
 * keeps growing through all of them gets out_status EAGAIN (the reference's
 * fs::read would hash whatever it read at that moment — a race with the
 * writer either way; the caller may retry the file later). */
int sdcas_cas_ids(sdcas_ctx *ctx, const char *const *paths, const uint64_t *sizes, size_t n,
                  uint64_t *out_keys, int32_t *out_status);

/* FileMetadata::new (file_identifier/mod.rs:48-96) of n files: fs::metadata,
 * then generate_cas_id(path, len) when the file is not empty (mod.rs:78-86) —
 * the metadata being fstat of the descriptor the cas_id reads use (one path
 * lookup per file; the same statuses). size_hints (may be NULL: one stat
 * pass first) only plan the staging — the indexer's sizes (file_path
 * size_in_bytes); a file of another size now is read again with room for
 * it. Per file: out_sizes[i] the metadata's len, out_flags[i]
 * SDCAS_META_HAS_CAS_ID when out_keys[i] holds the cas key (a non-empty
 * file read without error), SDCAS_META_DIR for a directory (the reference
 * refuses those, mod.rs:67-70; no cas_id), out_status[i] 0 or the errno of
 * the metadata or of the reads (SDCAS_STATUS_UNEXPECTED_EOF as
 * sdcas_cas_ids). ABI 6. */
#define SDCAS_META_HAS_CAS_ID 1u
#define SDCAS_META_DIR 2u
int sdcas_file_metadata(sdcas_ctx *ctx, const char *const *paths, const uint64_t *size_hints, size_t n,
                        uint64_t *out_sizes, uint64_t *out_keys, int32_t *out_status, uint8_t *out_flags);

/* file_checksum of n files (hash.rs:11-25): BLAKE3 of the whole content.
 * out32 receives 32*n bytes. The content hashed is the file's first L bytes,
 * L = its length when the call stats it (hash.rs reads to its first short
 * read, which on a regular local file is EOF): a file that grows while it is
 * read is hashed over L bytes, and one that shrinks below L before its bytes
 * are read gets SDCAS_STATUS_UNEXPECTED_EOF (the reference would hash the
 * shorter content). Neither happens to a file nobody writes meanwhile. */
int sdcas_checksums(sdcas_ctx *ctx, const char *const *paths, size_t n, uint8_t *out32,
                    int32_t *out_status);

/* ---- pre-assembled messages in host memory -----------------------------
 *
 * The bytes go through the context's pinned staging slots (a host copy by the
 * I/O threads, overlapped with the GPU). When `blob` is itself page-locked
 * (hipHostMalloc / hipHostRegister) and the messages lie in ascending,
 * non-overlapping ranges at 16-byte aligned offsets, each slot's byte range
 * is DMA'd straight from the caller's buffer instead (no host copy). */

/* BLAKE3 of n messages blob[offsets[i] .. offsets[i]+lens[i]) -> out32 (32*n B). */
int sdcas_hash_messages(sdcas_ctx *ctx, const uint8_t *blob, const uint64_t *offsets,
                        const uint64_t *lens, size_t n, uint8_t *out32);
/* the same, keeping only the cas key of each message */
int sdcas_cas_ids_from_messages(sdcas_ctx *ctx, const uint8_t *blob, const uint64_t *offsets,
                                const uint64_t *lens, size_t n, uint64_t *out_keys);

/* ---- device-resident batches (inputs already in HBM) ------------------- */

/* Size the device workspace for batches of up to max_msgs messages and
 * max_chunks total 1 KiB chunks (sum of max(1, ceil(len/1024))). Allocates;
 * call outside timed regions. */
int sdcas_dev_reserve(sdcas_ctx *ctx, size_t max_msgs, uint64_t max_chunks);
/* Enqueue the hash of n device-resident messages on `stream` (a hipStream_t,
 * NULL = the context's stream). Requirements: every offset 16-byte aligned,
 * and the blob readable for at least 64 bytes past the end of every message.
 * Either output may be NULL. Asynchronous; sdcas_dev_sync() reports a
 * capacity overflow detected on the device. */
int sdcas_dev_hash_messages(sdcas_ctx *ctx, const uint8_t *d_blob, const uint64_t *d_offsets,
                            const uint64_t *d_lens, size_t n, uint8_t *d_out32, uint64_t *d_out_keys,
                            void *stream);
int sdcas_dev_sync(sdcas_ctx *ctx, void *stream);
/* Name a stream's identity. The device calls of a context share its scratch
 * workspace, so each call makes its stream wait for the previous call's use
 * of it (an event wait: a barrier that idles the GPU ~15 us) unless both ran
 * on the same stream, whose order covers it. A handle alone cannot tell
 * "the same stream" (a destroyed stream's handle can come back for a new
 * one); a token can: consecutive calls on a stream bound with one nonzero
 * token skip the wait. The caller never hands the same token to another
 * stream while the context lives, and binds again (a new token, or 0 to
 * unbind) before destroying a bound stream or reusing its handle for a new
 * one. The end-of-call event a bound stream owes is recorded only when
 * another stream or a host wait needs it (a recorded event idles the GPU
 * ~6-8 us between calls). At most 64 streams per context are bound at once
 * (SDCAS_E_CAPACITY beyond). */
int sdcas_dev_bind_stream(sdcas_ctx *ctx, void *stream, uint64_t token);

/* ---- device-resident big messages, streamed in pieces ------------------
 *
 * file_checksum (hash.rs:11-25) of messages too large to be resident at once
 * (config C4: 1-4 GiB files, 256 GB): the caller delivers each message's
 * bytes in any order as segments already in HBM; every full 1 MiB piece
 * reduces to its level-10 BLAKE3 subtree node on the device, and finish
 * merges each message's nodes into its root.
 *   begin:  nfiles message lengths (host array), each > 1 MiB (smaller
 *           messages go through sdcas_dev_hash_messages).
 *   update: nseg segments (host arrays): bytes [h_msg_off[k], +h_len[k]) of
 *           message h_file[k], resident at device address h_dev_addr[k]
 *           (16-byte aligned, readable 64 B past the end). h_msg_off is a
 *           multiple of 1 MiB; h_len is too unless the segment ends the
 *           message. Every byte of every message exactly once over the
 *           session. Enqueued on `stream`; the segments must stay resident
 *           until the stream has passed this call. Use one stream per session.
 *   finish: 32-byte digests to d_out32 (device, 32*nfiles), on `stream`. */
int sdcas_dev_stream_begin(sdcas_ctx *ctx, const uint64_t *lens, size_t nfiles);
int sdcas_dev_stream_update(sdcas_ctx *ctx, size_t nseg, const uint64_t *h_file, const uint64_t *h_msg_off,
                            const uint64_t *h_len, const uint64_t *h_dev_addr, void *stream);
int sdcas_dev_stream_finish(sdcas_ctx *ctx, uint8_t *d_out32, void *stream);
/* One message's pieces split over several GPUs (a file larger
 * than one GPU's share): every rank opens the same session (same lens),
 * updates with its own disjoint segments, exports its node list (32 B per
 * node: one per full 1 MiB piece, then the tail piece's nodes; entries it did
 * not hash are zero), the ranks sum the lists (an all-reduce over int64 words:
 * each entry is nonzero on one rank only), import the sum, and finish. Bytes
 * must equal sdcas_dev_stream_node_bytes(); device pointers; on `stream`. */
size_t sdcas_dev_stream_node_bytes(sdcas_ctx *ctx);
int sdcas_dev_stream_export(sdcas_ctx *ctx, uint8_t *d_dst, size_t bytes, void *stream);
int sdcas_dev_stream_import(sdcas_ctx *ctx, const uint8_t *d_src, size_t bytes, void *stream);

/* ---- dedup / link (file_identifier/mod.rs:149-254) --------------------- */

/* out_link codes besides the ordinals (below) */
#define SDCAS_LINK_DROPPED INT64_MIN             /* I/O error: the file is dropped (mod.rs:125-141) */
#define SDCAS_LINK_DEFERRED (INT64_MIN + 1)      /* no step the job runs reaches the file: it stays an
                                                    orphan for the next batch / job */

/* The file identifier job's step loop around one batch of its orphans
 * (file_identifier_job.rs:86-236). A step reads the next chunk_size orphans
 * with id >= cursor and the cursor becomes its LAST row (:296-319,
 * mod.rs:401-405), so a last row that stays an orphan — an I/O error, or a
 * cas_id of None, which gets an Object but keeps cas_id NULL — is read again
 * by the next step, and the job runs a fixed task_count = ceil(orphans /
 * chunk_size) steps (:146). */
typedef struct sdcas_job_window {
  uint64_t max_steps; /* in: steps the job may still run; 0 = ceil(n / chunk_size), the task_count of a
                         job whose orphans are exactly these n rows */
  uint32_t more;      /* in: nonzero when more orphans follow row n-1: a step that would reach past it is
                         not run (its rows are DEFERRED) */
  uint32_t reserved;
  uint64_t steps;     /* out: steps run over the batch */
  uint64_t rows;      /* out: 1 + the last row the steps read (0: none); the job's next cursor is the id
                         of row rows-1, which the next batch reads again if it is still an orphan */
  uint64_t rereads;   /* out: rows read by two consecutive steps */
} sdcas_job_window;

/* Canonical group-by of the identifier steps over n orphan file_paths in id
 * order, chunk_size rows per step (0 -> 100). has_key[i] == 0 marks a cas_id
 * of None (empty file, mod.rs:78-86); status[i] != 0 drops the file (may be
 * NULL). existing_keys are the cas keys of Objects already in the library,
 * in DB order (may be NULL when n_existing == 0).
 * out_link[i] = i        file i creates a new Object (its last, if two steps read it)
 *             = j < i    file i links to the Object created by file j
 *             = -(e+1)   file i links to existing Object e
 *             = SDCAS_LINK_DROPPED / SDCAS_LINK_DEFERRED
 * *out_created / *out_linked receive the counts identifier_job_step returns
 * (mod.rs:349), summed over the steps. window may be NULL: the whole job over
 * these n rows. */
int sdcas_dedup_window(sdcas_ctx *ctx, const uint64_t *keys, const uint8_t *has_key, const int32_t *status,
                       size_t n, size_t chunk_size, const uint64_t *existing_keys, size_t n_existing,
                       sdcas_job_window *window, int64_t *out_link, int64_t *out_created, int64_t *out_linked);
/* The same steps' bookkeeping on the host, no device: window->steps / rows /
 * rereads for these rows, out_step[i] = the step that first reads row i
 * (UINT64_MAX if none does) and out_reads[i] = how many steps read it (each
 * read of a row without cas_id creates an Object); both may be NULL. The job
 * calls it before writing the cas_ids of the rows its steps read
 * (mod.rs:157-178 precede the existing Object lookup of :181-188);
 * sdcas_dedup_window returns the same window. */
int sdcas_job_plan(const uint8_t *has_key, const int32_t *status, size_t n, size_t chunk_size,
                   sdcas_job_window *window, uint64_t *out_step, uint32_t *out_reads);
/* sdcas_dedup_window with window = NULL */
int sdcas_dedup(sdcas_ctx *ctx, const uint64_t *keys, const uint8_t *has_key, const int32_t *status,
                size_t n, size_t chunk_size, const uint64_t *existing_keys, size_t n_existing,
                int64_t *out_link, int64_t *out_created, int64_t *out_linked);

/* ---- multi-GPU dedup stages (one process per GPU) -------
 *
 * sdcas_dedup's group-by split at its one exchange step, for a node whose
 * orphan file_paths (and existing Objects) are sharded over ranks. The host
 * runs, on every rank, with its own communicator (RCCL all-to-all over xGMI;
 * spacedrive_amd/dist_dedup.py is the reference driver):
 *   0. stays(files)      -> this rank's stays ordinals; all-gather them and
 *      plan                 build the job's step plan (the same on every rank)
 *   1. combine(files)    -> records grouped by owner rank + per-file slot
 *      combine(existing) -> records grouped by owner rank (ids = DB order)
 *   2. all-to-all both record sets (counts from out_starts)
 *   3. resolve on the received records -> one int64 answer per file record
 *   4. all-to-all the answers back (the reverse of step 2's file exchange)
 *   5. apply -> out_link / counts with sdcas_dedup's encoding, except that
 *      every file index is the GLOBAL orphan ordinal d_ids[i].
 * All pointers except out_starts are device pointers; calls are enqueued on
 * `stream` (NULL = the context's); combine synchronises once to return
 * out_starts. The owner of a key is its top 12 bits (the 3-hex thumbnail
 * shard prefix) split into `world` equal ranges.
 *
 * stays: the ordinals of this rank's files that stay orphans after their
 *   step (d_status != 0 or d_has_key == 0; both may be NULL) -> d_stays[cap],
 *   ascending, padded with UINT64_MAX; *d_count (device int64) = all of them,
 *   also when more than cap (then gather them again with a larger cap).
 * plan: d_stays = every rank's stays lists (n_stays entries in any order,
 *   UINT64_MAX entries ignored); the job's orphans are ordinals [0, n_total);
 *   max_steps / more as in sdcas_job_window -> d_plan (device u64,
 *   SDCAS_PLAN_WORDS(n_stays)): word 2 the steps run, 3 rows and 8 rereads
 *   (as in sdcas_job_window); the rest is the plan's own (dist_dedup.h).
 *   Word 9 stamps the building context's coarse index of the plan's re-read
 *   list (64 or more re-reads; 0: none): an apply on that context uses it
 *   until the context builds another plan, any other apply searches the
 *   whole list — the links are the same either way.
 * combine: d_ids[n] ascending; d_has_key / d_status may be NULL (all
 *   present / all ok). Writes exactly one record d_rec[2*u], d_rec[2*u+1] =
 *   (cas key, min id over the files carrying it) per distinct key (capacity
 *   2*n u64), grouped by owner: owner r's records are d_rec's records
 *   [out_starts[r], out_starts[r+1]), in NO particular order inside that
 *   range (ABI 5; ABI 4 and earlier documented ascending top-32-bit order and
 *   possibly several records per key — do not binary-search or merge the
 *   ranges); d_slot[i] = record of file i (0xFFFFFFFF no cas_id, 0xFFFFFFFE
 *   dropped; may be NULL), and out_starts[0..world] (host) = first record of
 *   each owner; out_starts[world] is the record count.
 * resolve: d_result[p] for received file record p = -(db+1) if existing
 *   Object db carries the key (the first in DB order), else the lowest orphan
 *   ordinal carrying it on any rank.
 * apply: d_result indexed by this rank's records (in send order); d_plan from
 *   plan (NULL: no file of the job stays an orphan and its steps read every
 *   row); d_counts (2 x u64, zeroed by the caller) += (created, linked). */
#define SDCAS_PLAN_HEADER_WORDS 12
#define SDCAS_PLAN_WORDS(n_stays) (SDCAS_PLAN_HEADER_WORDS + (n_stays))
int sdcas_dev_dedup_stays(sdcas_ctx *ctx, const uint8_t *d_has_key, const int32_t *d_status, const uint64_t *d_ids,
                          size_t n, size_t cap, uint64_t *d_stays, int64_t *d_count, void *stream);
int sdcas_dev_dedup_plan(sdcas_ctx *ctx, const uint64_t *d_stays, size_t n_stays, uint64_t n_total,
                         size_t chunk_size, uint64_t max_steps, uint32_t more, uint64_t *d_plan, void *stream);
int sdcas_dev_dedup_combine(sdcas_ctx *ctx, const uint64_t *d_keys, const uint8_t *d_has_key,
                            const int32_t *d_status, const uint64_t *d_ids, size_t n, uint32_t world,
                            uint64_t *d_rec, uint32_t *d_slot, uint64_t *out_starts, void *stream);
/* combine without the host synchronisation: the owner ranges go to
 * d_starts[0..world] (device u32) instead of out_starts, so that a caller
 * driving several GPUs enqueues every GPU's combine before it reads any
 * (sdcas_node_dedup_window) */
int sdcas_dev_dedup_combine_async(sdcas_ctx *ctx, const uint64_t *d_keys, const uint8_t *d_has_key,
                                  const int32_t *d_status, const uint64_t *d_ids, size_t n, uint32_t world,
                                  uint64_t *d_rec, uint32_t *d_slot, uint32_t *d_starts, void *stream);
int sdcas_dev_dedup_resolve(sdcas_ctx *ctx, const uint64_t *d_frec, size_t nf, const uint64_t *d_erec,
                            size_t ne, int64_t *d_result, void *stream);
int sdcas_dev_dedup_apply(sdcas_ctx *ctx, const uint64_t *d_ids, const uint32_t *d_slot, size_t n,
                          const int64_t *d_result, size_t chunk_size, const uint64_t *d_plan, int64_t *d_link,
                          uint64_t *d_counts, void *stream);
/* The same two stages without any host synchronisation, for RCCL's
 * all-to-all with equal splits (spacedrive_amd/dist_dedup.py): the combine
 * writes owner r's records to bucket r of d_send (world x cap records of 16 B,
 * record p of bucket r at d_send[2 * (r * cap + p)]), d_counts[r] (device
 * int64) = its valid records, d_slot[i] = the bucket position r * cap + p of
 * file i, and sets *d_overflow (device u32) to 1 when some owner has
 * more than cap records (the buckets are then unusable: rerun the exact
 * stages). The bucket combine may send several records of one key (one per
 * key per 2048-file tile of the rank, each with the tile's lowest ordinal);
 * the owner's minimum covers them. resolve_buckets answers the received
 * buckets (world x fcap file records, world x ecap existing records, the
 * first d_fcounts[r] / d_ecounts[r] of bucket r valid) into
 * d_result[world * fcap], bucket layout, and uses the received buckets as
 * scratch: the value word of valid records may be overwritten (each key's
 * claiming record takes the key's minimum). apply then reads the answers
 * returned in the same layout. */
int sdcas_dev_dedup_combine_buckets(sdcas_ctx *ctx, const uint64_t *d_keys, const uint8_t *d_has_key,
                                    const int32_t *d_status, const uint64_t *d_ids, size_t n, uint32_t world,
                                    size_t cap, uint64_t *d_send, uint32_t *d_slot, int64_t *d_counts,
                                    uint32_t *d_overflow, void *stream);
int sdcas_dev_dedup_resolve_buckets(sdcas_ctx *ctx, const uint64_t *d_frec, size_t fcap, const int64_t *d_fcounts,
                                    const uint64_t *d_erec, size_t ecap, const int64_t *d_ecounts, uint32_t world,
                                    int64_t *d_result, void *stream);
/* A world of one: the stages without the combine (nothing is exchanged, so
 * files and existing Objects go straight into resolve's table, and the plan
 * comes from this call's own stays rows): the same d_link / d_counts as
 * stays -> plan -> combine -> resolve -> apply. d_ekeys/d_eids [ne]: existing
 * Objects' cas keys and DB indices (may be NULL when ne == 0). d_ids lie in
 * [0, n_total) (n_total 0: n); max_steps / more as in sdcas_job_window.
 * d_plan_header (may be NULL) receives the plan's SDCAS_PLAN_HEADER_WORDS. */
int sdcas_dev_dedup_local(sdcas_ctx *ctx, const uint64_t *d_keys, const uint8_t *d_has_key,
                          const int32_t *d_status, const uint64_t *d_ids, size_t n, const uint64_t *d_ekeys,
                          const uint64_t *d_eids, size_t ne, size_t chunk_size, uint64_t n_total,
                          uint64_t max_steps, uint32_t more, int64_t *d_link, uint64_t *d_counts,
                          uint64_t *d_plan_header, void *stream);

/* ---- one process, several GPUs (a node) ----------------------------------
 *
 * sd-core is one process (Node::new, apps/server/src/main.rs:40; jobs run
 * in-process, job/manager.rs:32). A node is one context per entry of
 * `devices` (a device may repeat: two contexts on one GPU), with the batch
 * calls sharded over them and the dedup's exchange run in this process as
 * device-to-device copies (hipMemcpyPeerAsync; over xGMI between distinct
 * GPUs), or over RCCL (ncclCommInitAll, grouped ncclSend / ncclRecv) when every
 * device is distinct and the environment sets SDCAS_NODE_EXCHANGE=rccl (opt-in
 * until measured on a multi-GPU box). Results are those of the single-context
 * calls. opts (may be NULL) applies to every context; its progress function
 * receives the node's sums and may run on any of the node's threads (one at a
 * time). Calls on one node serialise. */
typedef struct sdcas_node sdcas_node;
int sdcas_node_init(const int32_t *devices, size_t n_devices, const sdcas_options *opts, sdcas_node **out_node);
void sdcas_node_destroy(sdcas_node *node);
const char *sdcas_node_last_error(const sdcas_node *node);
size_t sdcas_node_size(const sdcas_node *node);
/* 1 when the dedup exchange runs over RCCL, 0 over device copies */
int sdcas_node_uses_rccl(const sdcas_node *node);
int sdcas_node_set_progress(sdcas_node *node, sdcas_progress_fn progress, void *user, const volatile int32_t *cancel);
/* sdcas_cas_ids with the files cut into contiguous ranges of about equal
 * cas-message bytes, one per context */
int sdcas_node_cas_ids(sdcas_node *node, const char *const *paths, const uint64_t *sizes, size_t n,
                       uint64_t *out_keys, int32_t *out_status);
/* sdcas_checksums with the files assigned largest first to the least loaded context */
int sdcas_node_checksums(sdcas_node *node, const char *const *paths, size_t n, uint8_t *out32, int32_t *out_status);
/* sdcas_dedup_window over the node: contiguous ordinal ranges per context,
 * stays all-gathered and planned on every context, records exchanged to the
 * key's owner context (top 12 key bits), resolved there, answers returned */
int sdcas_node_dedup_window(sdcas_node *node, const uint64_t *keys, const uint8_t *has_key, const int32_t *status,
                            size_t n, size_t chunk_size, const uint64_t *existing_keys, size_t n_existing,
                            sdcas_job_window *window, int64_t *out_link, int64_t *out_created, int64_t *out_linked);

/* ---- helpers ------------------------------------------------------------ */

void sdcas_key_to_hex(uint64_t key, char out[17]);
void sdcas_digest_to_hex(const uint8_t digest[32], char out[65]);
uint64_t sdcas_cas_message_len(uint64_t size);

#ifdef __cplusplus
}
#endif
#endif /* SDCAS_H */
