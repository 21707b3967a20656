/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see blake3_ref.c's header).
 *
 * file_checksum (core/src/object/validation/hash.rs:11-25) of files too large
 * to hash whole on a CPU inside a test: BLAKE3 of a message whose content
 * repeats with a period of P = 2^k chunks (P >= 1 KiB), e.g. a 4 TiB + 1 MiB
 * + 17 byte file, the smallest kind of file whose chunk counters need their
 * high word (chunk index >= 2^32, blake3_ref.c b3_compress_state v[13]).
 *
 * Every full period at chunk index q*P/1024 is a complete aligned subtree of
 * BLAKE3's left-balanced tree; only its chunk counters differ between
 * periods. Each one is reduced to its chaining value (the `blake3` crate's
 * compress_subtree_wide + compress_subtree_to_parent_node, restated here with
 * the period hashed either by this oracle's scalar compression or by the
 * upstream BLAKE3 C 1.8.2 exported by ROCm's libclang-cpp as
 * llvm_blake3_compress_subtree_wide, SIMD and multi-threaded, so that the 4
 * TiB fixture takes minutes here), the tail's chunks follow, and the list is
 * merged with the crate's lazy subtree-stack rule (merge while the stack is
 * longer than popcount(chunks before the next node), fold right to left, ROOT
 * last) — the same rule blake3_ref.c's hasher applies chunk by chunk.
 *
 * Pinning: tests/test_oracle.py checks oracle_periodic_checksum against whole
 * hashes of materialised periodic messages (scalar oracle and llvm_blake3
 * hasher), and the upstream subtree CV against the scalar one at chunk
 * counters around 2^32.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define CHUNK 1024u
#define FLAG_CHUNK_START 1u
#define FLAG_CHUNK_END 2u

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

/* upstream: size_t blake3_compress_subtree_wide(const uint8_t *input, size_t
 * input_len, const uint32_t key[8], uint64_t chunk_counter, uint8_t flags,
 * uint8_t *out, bool use_tbb) — returns the number of 32-byte CVs written */
typedef size_t (*up_subtree_t)(const uint8_t *, size_t, const uint32_t *, uint64_t, uint8_t, uint8_t *, _Bool);
static up_subtree_t up_subtree;

int oracle_periodic_upstream_available(void) {
  if (up_subtree) return 1;
  const char *cands[] = {"/opt/rocm/lib/llvm/lib/libclang-cpp.so", "/opt/rocm-7.2.0/lib/llvm/lib/libclang-cpp.so.22.0git",
                         NULL};
  for (int i = 0; cands[i]; i++) {
    void *h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) continue;
    up_subtree = (up_subtree_t)dlsym(h, "llvm_blake3_compress_subtree_wide");
    if (up_subtree) return 1;
  }
  return 0;
}

/* chaining value of one chunk (1..1024 bytes; 0 only for an empty message)
 * at chunk index `counter`, never ROOT */
static void chunk_cv(const uint8_t *p, size_t n, uint64_t counter, uint32_t cv[8]) {
  memcpy(cv, IV, sizeof IV);
  size_t nblocks = n ? (n + 63) / 64 : 1;
  for (size_t b = 0; b < nblocks; b++) {
    uint8_t block[64] = {0};
    size_t len = n - b * 64 < 64 ? n - b * 64 : 64;
    memcpy(block, p + b * 64, len);
    uint8_t flags = (b == 0 ? FLAG_CHUNK_START : 0) | (b == nblocks - 1 ? FLAG_CHUNK_END : 0);
    b3ref_compress_cv(cv, block, (uint8_t)len, counter, flags, cv);
  }
}

/* pairwise parent layer (compress_parents_parallel): an odd last CV passes through */
static size_t parent_layer(uint32_t (*cvs)[8], size_t n) {
  size_t m = 0;
  for (size_t i = 0; i + 1 < n; i += 2) b3ref_parent_cv(cvs[i], cvs[i + 1], 0, cvs[m++]);
  if (n & 1) memmove(cvs[m++], cvs[n - 1], 32);
  return m;
}

/* CV of the complete subtree of len = 2^k * 1024 bytes (k >= 0) whose first
 * chunk has index `counter` */
int oracle_subtree_cv(const uint8_t *p, size_t len, uint64_t counter, int upstream, uint32_t out[8]) {
  if (len < CHUNK || (len & (len - 1))) return -1;
  size_t nchunks = len / CHUNK;
  if (nchunks == 1) {
    chunk_cv(p, len, counter, out);
    return 0;
  }
  if (upstream) {
    if (!oracle_periodic_upstream_available()) return -2;
    uint32_t cvs[64][8];  /* >= MAX_SIMD_DEGREE_OR_2 CVs */
    size_t n = up_subtree(p, len, IV, counter, 0, (uint8_t *)cvs, 0);
    if (n < 2 || n > 64) return -3;
    while (n > 2) n = parent_layer(cvs, n);
    b3ref_parent_cv(cvs[0], cvs[1], 0, out);
    return 0;
  }
  uint32_t (*cvs)[8] = malloc(nchunks * 32);
  if (!cvs) return -4;
  for (size_t c = 0; c < nchunks; c++) chunk_cv(p + c * CHUNK, CHUNK, counter + c, cvs[c]);
  size_t n = nchunks;
  while (n > 1) n = parent_layer(cvs, n);
  memcpy(out, cvs[0], 32);
  free(cvs);
  return 0;
}

typedef struct {
  const uint8_t *period;
  size_t plen;
  uint64_t q0, q1;
  int upstream, rc;
  uint32_t (*cvs)[8];
} pjob_t;

static void *pworker(void *arg) {
  pjob_t *j = (pjob_t *)arg;
  const uint64_t cpp = j->plen / CHUNK;
  for (uint64_t q = j->q0; q < j->q1 && !j->rc; q++) j->rc = oracle_subtree_cv(j->period, j->plen, q * cpp, j->upstream, j->cvs[q]);
  return NULL;
}

typedef struct {
  uint32_t (*s)[8];
  uint32_t depth;
} stack_t;

static void stack_push(stack_t *st, uint64_t j, const uint32_t cv[8]) {
  while (st->depth > (uint32_t)__builtin_popcountll(j)) {
    b3ref_parent_cv(st->s[st->depth - 2], st->s[st->depth - 1], 0, st->s[st->depth - 2]);
    st->depth--;
  }
  memcpy(st->s[st->depth++], cv, 32);
}

/* BLAKE3 of `total` bytes whose byte i is period[i mod plen]; plen = 2^k
 * chunks. threads <= 0: one. Returns 0, or < 0 (bad args / no upstream). */
int oracle_periodic_checksum(const uint8_t *period, size_t plen, uint64_t total, int threads, int upstream,
                             uint8_t out[32]) {
  if (plen < CHUNK || (plen & (plen - 1))) return -1;
  if (total <= plen) {
    b3ref_hash(period, total, out);
    return 0;
  }
  const uint64_t Q = total / plen, r = total % plen, cpp = plen / CHUNK;
  uint32_t (*cvs)[8] = malloc(Q * 32);
  if (!cvs) return -4;
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > Q) threads = (int)Q;
  pthread_t tid[256];
  pjob_t jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; t++) {
    jobs[t] = (pjob_t){period, plen, Q * t / threads, Q * (t + 1) / threads, upstream, 0, cvs};
    pthread_create(&tid[t], NULL, pworker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tid[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  if (rc) {
    free(cvs);
    return rc;
  }
  uint32_t stack[72][8];
  stack_t st = {stack, 0};
  uint32_t last[8];
  const uint64_t rc_chunks = (r + CHUNK - 1) / CHUNK;
  /* nodes in order: Q period subtrees, then the tail's chunks; the last node
   * is the right operand of the final fold, pushed nodes merge lazily */
  const uint64_t nodes = Q + rc_chunks;
  for (uint64_t i = 0; i < nodes; i++) {
    uint32_t cv[8];
    uint64_t j;
    if (i < Q) {
      memcpy(cv, cvs[i], 32);
      j = i * cpp;
    } else {
      uint64_t c = i - Q;
      size_t n = r - c * CHUNK < CHUNK ? (size_t)(r - c * CHUNK) : CHUNK;
      j = Q * cpp + c;
      chunk_cv(period + c * CHUNK, n, j, cv);
    }
    if (i + 1 < nodes) {
      stack_push(&st, j, cv);
    } else {
      /* merge what [0, j) completes, then fold right to left, ROOT last */
      while (st.depth > (uint32_t)__builtin_popcountll(j)) {
        b3ref_parent_cv(st.s[st.depth - 2], st.s[st.depth - 1], 0, st.s[st.depth - 2]);
        st.depth--;
      }
      memcpy(last, cv, 32);
      for (int d = (int)st.depth - 1; d >= 0; d--) b3ref_parent_cv(st.s[d], last, d == 0, last);
    }
  }
  free(cvs);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)last[i];
    out[4 * i + 1] = (uint8_t)(last[i] >> 8);
    out[4 * i + 2] = (uint8_t)(last[i] >> 16);
    out[4 * i + 3] = (uint8_t)(last[i] >> 24);
  }
  return 0;
}
