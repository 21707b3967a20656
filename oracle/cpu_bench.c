/*
 * ORACLE — TEST INFRASTRUCTURE ONLY: the CPU baseline leg of bench.py.
 *
 * Times the reference's CPU work for the C2 workload: the
 * cas_id of synthetic files whose messages (le64(size) || content,
 * core/src/object/cas.rs:25-29) are already in memory, hashed by BLAKE3 on
 * host cores. The reference hashes every file of a 100-file step on ONE
 * runtime thread (file_identifier/mod.rs:105-147, job/mod.rs:559-673), with
 * the SIMD `blake3` 1.5.0 crate. The crate cannot be built here (no Rust), so
 * the same SIMD algorithm class is used: upstream BLAKE3 C (SSE2/SSE4.1/AVX2/
 * AVX-512 dispatch) exported as llvm_blake3_* by ROCm's libclang-cpp, loaded
 * with dlopen. If it is absent, the scalar restatement (blake3_ref.c) is
 * timed instead and *kind reports it.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"
#include "../include/sdcas_synth.h"

typedef void (*up_init_t)(void *);
typedef void (*up_update_t)(void *, const void *, size_t);
typedef void (*up_final_t)(const void *, uint8_t *, size_t);
typedef const char *(*up_version_t)(void);

static up_init_t up_init;
static up_update_t up_update;
static up_final_t up_final;
static char up_version[32];

static int load_upstream(void) {
  if (up_init) return 1;
  const char *cands[] = {"/opt/rocm/lib/llvm/lib/libclang-cpp.so", "/opt/rocm-7.2.0/lib/llvm/lib/libclang-cpp.so.22.0git",
                         "/usr/lib/x86_64-linux-gnu/libLLVM-15.so.1", NULL};
  for (int i = 0; cands[i]; i++) {
    void *h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    up_init = (up_init_t)dlsym(h, "llvm_blake3_hasher_init");
    up_update = (up_update_t)dlsym(h, "llvm_blake3_hasher_update");
    up_final = (up_final_t)dlsym(h, "llvm_blake3_hasher_finalize");
    up_version_t v = (up_version_t)dlsym(h, "llvm_blake3_version");
    if (up_init && up_update && up_final) {
      strncpy(up_version, v ? v() : "?", sizeof up_version - 1);
      return 1;
    }
    up_init = NULL;
  }
  return 0;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
  const uint8_t *blob;
  const uint64_t *offs, *lens;
  uint64_t *keys;
  size_t lo, hi;
  int upstream;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  uint8_t d[32];
  uint8_t state[4096] __attribute__((aligned(64)));
  for (size_t i = j->lo; i < j->hi; i++) {
    if (j->upstream) {
      up_init(state);
      up_update(state, j->blob + j->offs[i], j->lens[i]);
      up_final(state, d, 32);
    } else {
      b3ref_hash(j->blob + j->offs[i], j->lens[i], d);
    }
    j->keys[i] = oracle_digest_key(d);
  }
  return NULL;
}

typedef struct {
  uint64_t seed;
  const uint64_t *offs, *lens;
  uint8_t *blob;
  size_t lo, hi;
} gen_t;

static void *gen_worker(void *arg) {
  gen_t *g = (gen_t *)arg;
  for (size_t i = g->lo; i < g->hi; i++) {
    uint64_t size = g->lens[i] - 8, key = sds_content_key(g->seed, i);
    uint8_t *m = g->blob + g->offs[i];
    for (int b = 0; b < 8; b++) m[b] = (uint8_t)(size >> (8 * b));
    for (uint64_t w = 0; 8 * w < size; w++) {
      uint64_t x = sds_content_word(key, w);
      uint64_t n = size - 8 * w < 8 ? size - 8 * w : 8;
      memcpy(m + 8 + 8 * w, &x, n);
    }
  }
  return NULL;
}

static double run_hash(const uint8_t *blob, const uint64_t *offs, const uint64_t *lens, uint64_t *keys,
                       size_t count, int threads, int up) {
  if (threads < 1) threads = 1;
  job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  double t0 = now_s();
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){blob, offs, lens, keys, count * t / threads, count * (t + 1) / threads, up};
    if (threads == 1) worker(&jobs[t]);
    else pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  double dt = now_s() - t0;
  free(jobs);
  free(th);
  return dt;
}

/* ---- generic synthetic files: C3/C4/C5 ------------------------------------ */

/* content bytes [off, off + len) of stream `key` into dst */
static void gen_content(uint64_t key, uint64_t off, uint64_t len, uint8_t *dst) {
  uint64_t w = off >> 3, end = off + len, pos = off;
  while (pos < end) {
    uint64_t x = sds_content_word(key, w);
    uint64_t wlo = w << 3, from = pos - wlo, take = 8 - from;
    if (take > end - pos) take = end - pos;
    memcpy(dst + (pos - off), (const uint8_t *)&x + from, take);
    pos += take;
    w++;
  }
}

typedef struct {
  const uint64_t *keys, *sizes, *offs, *lens;
  uint8_t *blob;
  int mode;
  size_t lo, hi;
} fgen_t;

static void *fgen_worker(void *arg) {
  fgen_t *g = (fgen_t *)arg;
  for (size_t i = g->lo; i < g->hi; i++) {
    uint8_t *m = g->blob + g->offs[i];
    uint64_t size = g->sizes[i], key = g->keys[i];
    if (g->mode == 1) { /* file_checksum: the whole content (hash.rs:15-21) */
      gen_content(key, 0, size, m);
      continue;
    }
    for (int b = 0; b < 8; b++) m[b] = (uint8_t)(size >> (8 * b)); /* cas.rs:25 */
    if (size <= SDS_MINIMUM_FILE_SIZE) {
      gen_content(key, 0, size, m + 8);
    } else { /* cas.rs:35-58 */
      uint64_t jump = (size - 2 * SDS_HEADER_OR_FOOTER_SIZE) / SDS_SAMPLE_COUNT;
      uint8_t *p = m + 8;
      gen_content(key, 0, SDS_HEADER_OR_FOOTER_SIZE, p);
      p += SDS_HEADER_OR_FOOTER_SIZE;
      for (uint64_t k = 0; k < SDS_SAMPLE_COUNT; k++, p += SDS_SAMPLE_SIZE)
        gen_content(key, SDS_HEADER_OR_FOOTER_SIZE + k * jump, SDS_SAMPLE_SIZE, p);
      gen_content(key, size - SDS_HEADER_OR_FOOTER_SIZE, SDS_HEADER_OR_FOOTER_SIZE, p);
    }
  }
  return NULL;
}

/* Messages of n synthetic files (content key, size) — mode 0: cas_id
 * messages, mode 1: whole content (checksum) — built untimed in parallel,
 * then hashed and timed on one thread (secs[0]) and on `threads` threads
 * (secs[1]). out_keys[i] = cas key of message i (first 8 digest bytes). */
int oracle_cpu_bench_files(const uint64_t *keys, const uint64_t *sizes, size_t n, int mode, int threads,
                           int prefer_upstream, uint64_t *out_keys, uint64_t *bytes, double *secs, int *kind,
                           char *version_out) {
  uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t *lens = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t total = 0, hashed = 0;
  for (size_t i = 0; i < n; i++) {
    lens[i] = mode == 1 ? sizes[i] : sds_cas_msg_len(sizes[i]);
    offs[i] = total;
    total += (lens[i] + 15) & ~15ull;
    hashed += lens[i];
  }
  uint8_t *blob = (uint8_t *)malloc(total + 64);
  if (!blob) return -1;
  int gt = threads < 1 ? 1 : threads;
  fgen_t *gj = (fgen_t *)calloc((size_t)gt, sizeof(fgen_t));
  pthread_t *th = (pthread_t *)calloc((size_t)gt, sizeof(pthread_t));
  for (int t = 0; t < gt; t++) {
    gj[t] = (fgen_t){keys, sizes, offs, lens, blob, mode, n * t / gt, n * (t + 1) / gt};
    pthread_create(&th[t], NULL, fgen_worker, &gj[t]);
  }
  for (int t = 0; t < gt; t++) pthread_join(th[t], NULL);
  free(gj);
  free(th);
  int up = prefer_upstream && load_upstream();
  if (kind) *kind = up;
  if (version_out) strcpy(version_out, up ? up_version : "scalar");
  secs[0] = run_hash(blob, offs, lens, out_keys, n, 1, up);
  secs[1] = threads > 1 ? run_hash(blob, offs, lens, out_keys, n, threads, up) : secs[0];
  if (bytes) *bytes = hashed;
  free(blob);
  free(offs);
  free(lens);
  return 0;
}

/* Build the cas messages of C2 files [0, count) (untimed, in parallel), then
 * time hashing them: secs[0] with ONE thread (the reference's shape), and
 * secs[1] with `threads` threads (all host cores given to this job).
 * *bytes = message bytes hashed; keys[count] receive the cas keys (for parity
 * against the GPU). *kind: 1 = upstream SIMD BLAKE3, 0 = scalar restatement. */
int oracle_cpu_bench_c2(uint64_t seed, size_t count, int threads, int prefer_upstream, uint64_t *keys,
                        uint64_t *bytes, double *secs, int *kind, char *version_out) {
  uint64_t *offs = (uint64_t *)malloc(sizeof(uint64_t) * (count + 1));
  uint64_t *lens = (uint64_t *)malloc(sizeof(uint64_t) * (count + 1));
  uint64_t total = 0, hashed = 0;
  for (size_t i = 0; i < count; i++) {
    uint64_t size = sds_c2_size(seed, i);
    lens[i] = sds_cas_msg_len(size);
    offs[i] = total;
    total += (lens[i] + 15) & ~15ull;
    hashed += lens[i];
  }
  uint8_t *blob = (uint8_t *)malloc(total + 64);
  if (!blob) return -1;
  int gt = threads < 1 ? 1 : threads;
  gen_t *gj = (gen_t *)calloc((size_t)gt, sizeof(gen_t));
  pthread_t *th = (pthread_t *)calloc((size_t)gt, sizeof(pthread_t));
  for (int t = 0; t < gt; t++) {
    gj[t] = (gen_t){seed, offs, lens, blob, count * t / gt, count * (t + 1) / gt};
    pthread_create(&th[t], NULL, gen_worker, &gj[t]);
  }
  for (int t = 0; t < gt; t++) pthread_join(th[t], NULL);
  free(gj);
  free(th);
  int up = prefer_upstream && load_upstream();
  if (kind) *kind = up;
  if (version_out) strcpy(version_out, up ? up_version : "scalar");
  secs[0] = run_hash(blob, offs, lens, keys, count, 1, up);
  secs[1] = threads > 1 ? run_hash(blob, offs, lens, keys, count, threads, up) : secs[0];
  if (bytes) *bytes = hashed;
  free(blob);
  free(offs);
  free(lens);
  return 0;
}
