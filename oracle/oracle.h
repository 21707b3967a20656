/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see blake3_ref.c header). CPU restatement
 * of the reference's content-identification path:
 *   generate_cas_id   core/src/object/cas.rs:23-62
 *   file_checksum     core/src/object/validation/hash.rs:11-25
 *   dedup/link        core/src/object/file_identifier/mod.rs:98-350
 */
#ifndef SDCAS_ORACLE_H
#define SDCAS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B3REF_BLOCK_LEN 64
#define B3REF_CHUNK_LEN 1024
#define B3REF_CHUNK_START 1
#define B3REF_CHUNK_END 2
#define B3REF_PARENT 4
#define B3REF_ROOT 8

typedef struct {
  uint32_t cv[8];
  uint64_t counter;
  uint8_t buf[64];
  uint8_t buf_len;
  uint8_t blocks_done;
} b3ref_chunk;

typedef struct {
  b3ref_chunk chunk;
  uint32_t stack[54][8];
  unsigned stack_len;
} b3ref_hasher;

void b3ref_hasher_init(b3ref_hasher *h);
void b3ref_hasher_update(b3ref_hasher *h, const void *data, size_t n);
void b3ref_hasher_finalize(const b3ref_hasher *h, uint8_t out[32]);
void b3ref_hash(const void *data, size_t n, uint8_t out[32]);
void b3ref_compress_cv(const uint32_t cv[8], const uint8_t block[64], uint8_t block_len,
                       uint64_t counter, uint8_t flags, uint32_t out_cv[8]);
void b3ref_parent_cv(const uint32_t left[8], const uint32_t right[8], int root, uint32_t out[8]);

/* status for read_exact() hitting EOF (Rust io::ErrorKind::UnexpectedEof has no errno) */
#define ORACLE_STATUS_UNEXPECTED_EOF 100001

/* cas.rs:23-62 over a real file; returns 0 or a positive status, writes 16 hex + NUL */
int oracle_generate_cas_id(const char *path, uint64_t size, char out_hex[17]);
/* hash.rs:11-25 over a real file; returns 0 or a positive status, writes 64 hex + NUL */
int oracle_file_checksum(const char *path, char out_hex[65]);

/* u64 cas key = digest bytes 0..7 big-endian, so "%016llx" == to_hex()[..16] */
uint64_t oracle_digest_key(const uint8_t digest[32]);
uint64_t oracle_cas_key_of_message(const uint8_t *msg, size_t n);

/* synthetic corpora (include/sdcas_synth.h): cas key of file (key, size) and
 * full-content checksum of a synthetic file */
uint64_t oracle_synth_cas_key(uint64_t content_key, uint64_t size);
void oracle_synth_checksum(uint64_t content_key, uint64_t size, uint8_t out[32]);
/* build the cas message of a synthetic file into out (capacity >= msg len) */
size_t oracle_synth_cas_message(uint64_t content_key, uint64_t size, uint8_t *out);

/* Dedup/link restatement of file_identifier/mod.rs:98-350 inside the file
 * identifier job's step loop (file_identifier_job.rs:86-236,296-319,
 * mod.rs:380-407), in its canonical, deterministic form (SURVEY.md §8a rows
 * a6/a7). Files are the job's orphan file_paths in id order; each step reads
 * the next `chunk_size` orphans (CHUNK_SIZE=100, mod.rs:34) with id >= the
 * cursor, which is the previous step's LAST row — so a last row that stays an
 * orphan (status != 0, or no cas_id) is read again by the next step.
 * status[i] != 0 drops the file (mod.rs:125-141); has_key[i] == 0 is a cas_id
 * of None (mod.rs:78-86). existing_keys[e] are the cas keys of Objects
 * already in the library, in DB order.
 * out_link[i]: i            -> file i creates a new Object (the last one, if
 *                              it was read twice)
 *              j (<i)       -> file i links to the Object created by file j
 *              -(e+1)       -> file i links to existing Object e
 *              INT64_MIN    -> dropped (status != 0)
 *              INT64_MIN+1  -> not reached by the steps (ORACLE_LINK_DEFERRED)
 * Returns the created count; *linked receives the linked count (mod.rs:349
 * summed over the steps). */
#define ORACLE_LINK_DEFERRED (INT64_MIN + 1)
typedef struct oracle_job_window {
  uint64_t max_steps; /* in: steps the job may still run (0: ceil(n / chunk_size)) */
  int32_t more;       /* in: nonzero when more orphans follow row n-1 */
  int32_t reserved;
  uint64_t steps;     /* out: steps run */
  uint64_t rows;      /* out: last row of the last step + 1 (0: none) */
  uint64_t rereads;   /* out: steps that began with the previous step's last row */
} oracle_job_window;
int64_t oracle_identifier_job(size_t n, const uint64_t *keys, const uint8_t *has_key, const int32_t *status,
                              size_t chunk_size, size_t n_existing, const uint64_t *existing_keys,
                              oracle_job_window *win, int64_t *out_link, int64_t *linked);
/* the whole job over the n rows (win = NULL) */
int64_t oracle_identifier_dedup(size_t n, const uint64_t *keys, const uint8_t *has_key,
                                const int32_t *status, size_t chunk_size, size_t n_existing,
                                const uint64_t *existing_keys, int64_t *out_link, int64_t *linked);

/* bench.py cpu_baseline leg (cpu_bench.c): hash the cas messages of C2 files
 * [0, count) already in memory; secs[0] one thread, secs[1] `threads` threads */
int oracle_cpu_bench_c2(uint64_t seed, size_t count, int threads, int prefer_upstream, uint64_t *keys,
                        uint64_t *bytes, double *secs, int *kind, char *version_out);
/* the same for any synthetic files (keys, sizes): mode 0 cas_id messages
 * (C3, C5), mode 1 whole-content checksums (C4) */
int oracle_cpu_bench_files(const uint64_t *keys, const uint64_t *sizes, size_t n, int mode, int threads,
                           int prefer_upstream, uint64_t *out_keys, uint64_t *bytes, double *secs, int *kind,
                           char *version_out);

/* every cas key of n synthetic files (the -m gpu corpus tests' checker), on
 * `threads` threads; returns 1 if upstream SIMD BLAKE3 hashed, 0 scalar */
int oracle_synth_cas_keys_mt(const uint64_t *keys, const uint64_t *sizes, size_t n, int threads, int prefer_upstream,
                             uint64_t *out_keys);
/* bench.py's reference-faithful CPU baseline: the identifier job's CPU shape
 * over real files (steps of `chunk` files in series; per step an I/O pool of
 * io_threads does metadata + cas.rs reads, one thread hashes in file order).
 * secs[0] = wall time; out_status[i] = errno / UnexpectedEof or 0. */
int oracle_cpu_faithful(const char *const *paths, const uint64_t *sizes, size_t n, size_t chunk, int io_threads,
                        int prefer_upstream, uint64_t *out_keys, int32_t *out_status, double *secs, int *kind,
                        char *version_out);

/* periodic.c: BLAKE3 of messages whose content repeats with a period of 2^k
 * chunks (the >= 4 TiB checksum fixture); upstream = hash each period with
 * llvm_blake3_compress_subtree_wide (1.8.2) instead of the scalar oracle */
int oracle_periodic_upstream_available(void);
int oracle_subtree_cv(const uint8_t *p, size_t len, uint64_t counter, int upstream, uint32_t out[8]);
int oracle_periodic_checksum(const uint8_t *period, size_t plen, uint64_t total, int threads, int upstream,
                             uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif
