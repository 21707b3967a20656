/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see blake3_ref.c header).
 *
 * CPU restatement of sd-core's content identification:
 *   oracle_generate_cas_id   <- core/src/object/cas.rs:23-62
 *   oracle_file_checksum     <- core/src/object/validation/hash.rs:9-25
 *   oracle_identifier_job    <- core/src/object/file_identifier/mod.rs:98-350 inside the
 *                               job's step loop (file_identifier_job.rs:86-236,296-319,
 *                               mod.rs:380-407)
 * The I/O pattern is kept (one whole read, or header / 4 samples / footer with
 * seeks; 1 MiB reads for the checksum) so this file also serves as the
 * reference-faithful CPU baseline.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "oracle.h"
#include "../include/sdcas_synth.h"

/* cas.rs:10-15 */
#define SAMPLE_COUNT 4ull
#define SAMPLE_SIZE (1024ull * 10)
#define HEADER_OR_FOOTER_SIZE (1024ull * 8)
#define MINIMUM_FILE_SIZE (1024ull * 100)
/* hash.rs:9 */
#define CHECKSUM_BLOCK_LEN 1048576ull

static const char HEXD[] = "0123456789abcdef";

static void to_hex(const uint8_t *d, size_t n, char *out) {
  for (size_t i = 0; i < n; i++) {
    out[2 * i] = HEXD[d[i] >> 4];
    out[2 * i + 1] = HEXD[d[i] & 15];
  }
  out[2 * n] = 0;
}

uint64_t oracle_digest_key(const uint8_t digest[32]) {
  uint64_t k = 0;
  for (int i = 0; i < 8; i++) k = (k << 8) | digest[i];
  return k;
}

uint64_t oracle_cas_key_of_message(const uint8_t *msg, size_t n) {
  uint8_t d[32];
  b3ref_hash(msg, n, d);
  return oracle_digest_key(d);
}

/* tokio read_exact: fill the whole buffer or fail with UnexpectedEof */
static int read_exact(int fd, uint8_t *buf, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = read(fd, buf + got, n - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) return ORACLE_STATUS_UNEXPECTED_EOF;
    got += (size_t)r;
  }
  return 0;
}

int oracle_generate_cas_id(const char *path, uint64_t size, char out_hex[17]) {
  b3ref_hasher h;
  b3ref_hasher_init(&h);
  uint8_t le[8];
  for (int i = 0; i < 8; i++) le[i] = (uint8_t)(size >> (8 * i));
  b3ref_hasher_update(&h, le, 8); /* cas.rs:25 */

  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno;
  int st = 0;
  if (size <= MINIMUM_FILE_SIZE) {
    /* cas.rs:27-29: fs::read reads the file as it is now, whatever `size` said */
    uint8_t buf[65536];
    for (;;) {
      ssize_t r = read(fd, buf, sizeof buf);
      if (r < 0) {
        if (errno == EINTR) continue;
        st = errno;
        break;
      }
      if (r == 0) break;
      b3ref_hasher_update(&h, buf, (size_t)r);
    }
  } else {
    uint8_t buf[SAMPLE_SIZE];
    /* header, cas.rs:35-38 */
    st = read_exact(fd, buf, HEADER_OR_FOOTER_SIZE);
    uint64_t current_pos = HEADER_OR_FOOTER_SIZE;
    if (!st) b3ref_hasher_update(&h, buf, HEADER_OR_FOOTER_SIZE);
    /* samples, cas.rs:41-51 */
    uint64_t seek_jump = (size - HEADER_OR_FOOTER_SIZE * 2) / SAMPLE_COUNT;
    while (!st) {
      st = read_exact(fd, buf, SAMPLE_SIZE);
      if (st) break;
      b3ref_hasher_update(&h, buf, SAMPLE_SIZE);
      if (current_pos >= HEADER_OR_FOOTER_SIZE + seek_jump * (SAMPLE_COUNT - 1)) break;
      off_t p = lseek(fd, (off_t)(current_pos + seek_jump), SEEK_SET);
      if (p < 0) {
        st = errno;
        break;
      }
      current_pos = (uint64_t)p;
    }
    /* footer, cas.rs:54-58 */
    if (!st) {
      if (lseek(fd, -(off_t)HEADER_OR_FOOTER_SIZE, SEEK_END) < 0) st = errno;
    }
    if (!st) st = read_exact(fd, buf, HEADER_OR_FOOTER_SIZE);
    if (!st) b3ref_hasher_update(&h, buf, HEADER_OR_FOOTER_SIZE);
  }
  close(fd);
  if (st) return st;
  uint8_t d[32];
  b3ref_hasher_finalize(&h, d);
  to_hex(d, 8, out_hex); /* cas.rs:61: to_hex()[..16] */
  return 0;
}

int oracle_file_checksum(const char *path, char out_hex[65]) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno;
  b3ref_hasher h;
  b3ref_hasher_init(&h);
  uint8_t *buf = (uint8_t *)malloc(CHECKSUM_BLOCK_LEN);
  int st = 0;
  /* hash.rs:15-21: one read() per iteration, stop at the first short read */
  for (;;) {
    ssize_t r;
    do {
      r = read(fd, buf, CHECKSUM_BLOCK_LEN);
    } while (r < 0 && errno == EINTR);
    if (r < 0) {
      st = errno;
      break;
    }
    b3ref_hasher_update(&h, buf, (size_t)r);
    if ((uint64_t)r != CHECKSUM_BLOCK_LEN) break;
  }
  free(buf);
  close(fd);
  if (st) return st;
  uint8_t d[32];
  b3ref_hasher_finalize(&h, d);
  to_hex(d, 32, out_hex);
  return 0;
}

/* ---- synthetic corpora ---------------------------------------------------- */

size_t oracle_synth_cas_message(uint64_t content_key, uint64_t size, uint8_t *out) {
  uint64_t n = sds_cas_msg_len(size);
  for (uint64_t x = 0; x < n; x++) out[x] = sds_cas_msg_byte(content_key, size, x);
  return (size_t)n;
}

uint64_t oracle_synth_cas_key(uint64_t content_key, uint64_t size) {
  uint64_t n = sds_cas_msg_len(size);
  uint8_t *m = (uint8_t *)malloc(n ? n : 1);
  oracle_synth_cas_message(content_key, size, m);
  uint64_t k = oracle_cas_key_of_message(m, n);
  free(m);
  return k;
}

void oracle_synth_checksum(uint64_t content_key, uint64_t size, uint8_t out[32]) {
  b3ref_hasher h;
  b3ref_hasher_init(&h);
  uint8_t buf[8192];
  uint64_t off = 0;
  while (off < size) {
    size_t take = (size - off) < sizeof buf ? (size_t)(size - off) : sizeof buf;
    for (size_t i = 0; i < take; i++) buf[i] = sds_content_byte(content_key, off + i);
    b3ref_hasher_update(&h, buf, take);
    off += take;
  }
  b3ref_hasher_finalize(&h, out);
}

/* ---- dedup / link --------------------------------------------------------- */

typedef struct {
  uint64_t *keys;
  int64_t *vals;
  uint8_t *used;
  size_t mask;
} kmap;

static void kmap_init(kmap *m, size_t n) {
  size_t cap = 16;
  while (cap < 2 * n + 16) cap <<= 1;
  m->keys = (uint64_t *)calloc(cap, sizeof(uint64_t));
  m->vals = (int64_t *)calloc(cap, sizeof(int64_t));
  m->used = (uint8_t *)calloc(cap, 1);
  m->mask = cap - 1;
}

static void kmap_free(kmap *m) {
  free(m->keys);
  free(m->vals);
  free(m->used);
}

static int64_t *kmap_find(kmap *m, uint64_t k) {
  size_t i = (size_t)(sds_mix64(k) & m->mask);
  while (m->used[i]) {
    if (m->keys[i] == k) return &m->vals[i];
    i = (i + 1) & m->mask;
  }
  return NULL;
}

/* insert only if absent: the first Object in DB order wins (mod.rs:214-224) */
static void kmap_insert_first(kmap *m, uint64_t k, int64_t v) {
  size_t i = (size_t)(sds_mix64(k) & m->mask);
  while (m->used[i]) {
    if (m->keys[i] == k) return;
    i = (i + 1) & m->mask;
  }
  m->used[i] = 1;
  m->keys[i] = k;
  m->vals[i] = v;
}

/* The file identifier job's step loop around identifier_job_step, restated
 * literally over a simulated file_path table whose rows 0..n-1 (id order) are
 * the job's orphans:
 *   init        task_count = ceil(orphans / CHUNK_SIZE) (file_identifier_job.rs:126-146),
 *               cursor = the first orphan's id (:152-173)
 *   each step   get_orphan_file_paths: orphans with id >= cursor, ORDER BY id,
 *               LIMIT CHUNK_SIZE (:296-319, filter :251-278: object_id IS NULL
 *               OR cas_id IS NULL); no rows -> EarlyFinish (:203-209);
 *               identifier_job_step over them (mod.rs:98-350); cursor = the
 *               chunk's LAST row (mod.rs:401-405)
 * A row that stays an orphan after its step — an I/O error (the file is
 * dropped, mod.rs:125-141) or a cas_id of None (it gets an Object but keeps
 * cas_id NULL, mod.rs:78-86,246-254) — is read again by the next step when it
 * was its chunk's last row (id >= cursor), and every later chunk boundary
 * shifts by one.
 * win (may be NULL = {0, 0}) cuts the loop to a batch of a longer job:
 * max_steps = the steps the job may still run (0: ceil(n / chunk_size)); more
 * != 0 when further orphans follow row n-1, so a step that would reach past
 * it is left to the next batch. Out: steps run, rows = last row of the last
 * step + 1 (the next cursor is row rows-1; 0 if no step ran), rereads =
 * steps that began with the previous step's last row. */
int64_t oracle_identifier_job(size_t n, const uint64_t *keys, const uint8_t *has_key, const int32_t *status,
                              size_t chunk_size, size_t n_existing, const uint64_t *existing_keys,
                              oracle_job_window *win, int64_t *out_link, int64_t *linked) {
  kmap objects; /* cas key -> first Object carrying it (library state) */
  kmap_init(&objects, n + n_existing);
  for (size_t e = 0; e < n_existing; e++) kmap_insert_first(&objects, existing_keys[e], -(int64_t)e - 1);
  if (chunk_size == 0) chunk_size = 100;
  uint8_t *orphan = (uint8_t *)malloc(n ? n : 1);
  size_t *rows = (size_t *)malloc(sizeof(size_t) * chunk_size);
  memset(orphan, 1, n);
  for (size_t i = 0; i < n; i++) out_link[i] = ORACLE_LINK_DEFERRED;
  const uint64_t task_count = (win && win->max_steps) ? win->max_steps : (n + chunk_size - 1) / chunk_size;
  const int more = win ? win->more : 0;
  int64_t created = 0, nlinked = 0;
  uint64_t steps = 0, rereads = 0, rows_done = 0;
  size_t cursor = 0, prev_last = (size_t)-1;
  for (uint64_t step = 0; step < task_count; step++) {
    size_t m = 0;
    for (size_t id = cursor; id < n && m < chunk_size; id++)
      if (orphan[id]) rows[m++] = id;
    if (m == 0) break;                    /* EarlyFinish */
    if (more && m < chunk_size) break;    /* the step's other rows are in the next batch */
    if (rows[0] == prev_last) rereads++;
    /* mod.rs:181-238: files whose cas_id already belongs to an Object link to
     * the first such Object; the lookup sees the library as it was before
     * this step */
    for (size_t r = 0; r < m; r++) {
      const size_t i = rows[r];
      if (status && status[i] != 0) {
        out_link[i] = INT64_MIN; /* mod.rs:125-141: logged and dropped */
        continue;
      }
      int64_t *hit = has_key[i] ? kmap_find(&objects, keys[i]) : NULL;
      if (hit) {
        out_link[i] = *hit;
        nlinked++;
      } else {
        /* mod.rs:246-254: None cas_ids and unseen cas_ids each get a new
         * Object, intra-chunk duplicates included */
        out_link[i] = (int64_t)i;
        created++;
      }
    }
    /* objects created by this step become visible to later steps (mod.rs:314-342);
     * a file with a cas_id and an Object is no longer an orphan */
    for (size_t r = 0; r < m; r++) {
      const size_t i = rows[r];
      if (status && status[i] != 0) continue;
      if (!has_key[i]) continue;
      if (out_link[i] == (int64_t)i) kmap_insert_first(&objects, keys[i], (int64_t)i);
      orphan[i] = 0;
    }
    cursor = prev_last = rows[m - 1];
    rows_done = (uint64_t)cursor + 1;
    steps++;
  }
  free(rows);
  free(orphan);
  kmap_free(&objects);
  if (win) {
    win->steps = steps;
    win->rows = rows_done;
    win->rereads = rereads;
  }
  if (linked) *linked = nlinked;
  return created;
}

int64_t oracle_identifier_dedup(size_t n, const uint64_t *keys, const uint8_t *has_key,
                                const int32_t *status, size_t chunk_size, size_t n_existing,
                                const uint64_t *existing_keys, int64_t *out_link, int64_t *linked) {
  return oracle_identifier_job(n, keys, has_key, status, chunk_size, n_existing, existing_keys, NULL, out_link,
                               linked);
}
