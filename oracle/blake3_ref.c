/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from
 * the product path (spacedrive_amd/). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * Scalar BLAKE3 (hash mode, unkeyed, 32-byte output) restated from the public
 * BLAKE3 specification. The reference does not carry this code: sd-core calls
 * the third-party Rust crate `blake3` 1.5.0 (Cargo.lock:680-690, workspace pin
 * Cargo.toml:57, checksum 0231f061...), which is NOT vendored in
 * /root/reference. Call sites whose behaviour this file must reproduce:
 *   core/src/object/cas.rs:3,24,25,29,38,44,58,61  (Hasher::new/update/finalize/to_hex)
 *   core/src/object/validation/hash.rs:3,13,17,22
 *
 * The incremental hasher mirrors the crate's observable contract: any sequence
 * of update() calls hashes the concatenation of their inputs. Internally it keeps
 * one chunk state plus a stack of subtree chaining values that is merged lazily
 * (a subtree is only merged once more input proves it is not the root).
 *
 * Parity pinning: tests/test_oracle.py checks this file against the upstream
 * BLAKE3 C implementation shipped in this image (llvm_blake3_* 1.3.1 in
 * libLLVM-15 and 1.8.2 in ROCm's libclang-cpp) through the committed fixtures
 * in tests/golden/, and against the known answers of SURVEY.md Appendix B.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include "oracle.h"

static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

/* message word order used by each of the 7 rounds (round r applies the base
 * permutation r times) */
static const uint8_t B3_SCHED[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13},
};

static inline uint32_t rotr32(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

static inline uint32_t load_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline void store_le32(uint8_t *p, uint32_t x) {
  p[0] = (uint8_t)x;
  p[1] = (uint8_t)(x >> 8);
  p[2] = (uint8_t)(x >> 16);
  p[3] = (uint8_t)(x >> 24);
}

#define G(a, b, c, d, x, y)    \
  do {                         \
    v[a] = v[a] + v[b] + (x);  \
    v[d] = rotr32(v[d] ^ v[a], 16); \
    v[c] = v[c] + v[d];        \
    v[b] = rotr32(v[b] ^ v[c], 12); \
    v[a] = v[a] + v[b] + (y);  \
    v[d] = rotr32(v[d] ^ v[a], 8);  \
    v[c] = v[c] + v[d];        \
    v[b] = rotr32(v[b] ^ v[c], 7);  \
  } while (0)

/* Full compression: returns the 16-word state after 7 rounds (before the
 * feed-forward), from which both the chaining value and the root output are
 * derived. */
static void b3_compress_state(const uint32_t cv[8], const uint8_t block[64], uint8_t block_len,
                              uint64_t counter, uint8_t flags, uint32_t v[16]) {
  uint32_t m[16];
  for (int i = 0; i < 16; i++) m[i] = load_le32(block + 4 * i);
  for (int i = 0; i < 8; i++) v[i] = cv[i];
  v[8] = B3_IV[0];
  v[9] = B3_IV[1];
  v[10] = B3_IV[2];
  v[11] = B3_IV[3];
  v[12] = (uint32_t)counter;
  v[13] = (uint32_t)(counter >> 32);
  v[14] = block_len;
  v[15] = flags;
  for (int r = 0; r < 7; r++) {
    const uint8_t *s = B3_SCHED[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
}

void b3ref_compress_cv(const uint32_t cv[8], const uint8_t block[64], uint8_t block_len,
                       uint64_t counter, uint8_t flags, uint32_t out_cv[8]) {
  uint32_t v[16];
  b3_compress_state(cv, block, block_len, counter, flags, v);
  for (int i = 0; i < 8; i++) out_cv[i] = v[i] ^ v[i + 8];
}

/* ---- chunk state ---------------------------------------------------------- */

static void chunk_init(b3ref_chunk *c, uint64_t counter) {
  memcpy(c->cv, B3_IV, sizeof(B3_IV));
  c->counter = counter;
  memset(c->buf, 0, sizeof(c->buf));
  c->buf_len = 0;
  c->blocks_done = 0;
}

static size_t chunk_len(const b3ref_chunk *c) { return (size_t)B3REF_BLOCK_LEN * c->blocks_done + c->buf_len; }

static uint8_t chunk_start_flag(const b3ref_chunk *c) { return c->blocks_done == 0 ? B3REF_CHUNK_START : 0; }

static void chunk_update(b3ref_chunk *c, const uint8_t *in, size_t n) {
  while (n > 0) {
    if (c->buf_len == B3REF_BLOCK_LEN) {
      /* buffered block is full and more input follows: it is not the last block */
      b3ref_compress_cv(c->cv, c->buf, B3REF_BLOCK_LEN, c->counter, chunk_start_flag(c), c->cv);
      c->blocks_done++;
      c->buf_len = 0;
      memset(c->buf, 0, sizeof(c->buf));
    }
    size_t take = B3REF_BLOCK_LEN - c->buf_len;
    if (take > n) take = n;
    memcpy(c->buf + c->buf_len, in, take);
    c->buf_len += (uint8_t)take;
    in += take;
    n -= take;
  }
}

/* "output" of a chunk or parent: the inputs of its final compression */
typedef struct {
  uint32_t cv[8];
  uint8_t block[64];
  uint8_t block_len;
  uint64_t counter;
  uint8_t flags;
} b3_output;

static b3_output chunk_output(const b3ref_chunk *c) {
  b3_output o;
  memcpy(o.cv, c->cv, 32);
  memcpy(o.block, c->buf, 64);
  o.block_len = c->buf_len;
  o.counter = c->counter;
  o.flags = (uint8_t)(chunk_start_flag(c) | B3REF_CHUNK_END);
  return o;
}

static b3_output parent_output(const uint32_t left[8], const uint32_t right[8]) {
  b3_output o;
  memcpy(o.cv, B3_IV, 32);
  for (int i = 0; i < 8; i++) {
    store_le32(o.block + 4 * i, left[i]);
    store_le32(o.block + 32 + 4 * i, right[i]);
  }
  o.block_len = B3REF_BLOCK_LEN;
  o.counter = 0;
  o.flags = B3REF_PARENT;
  return o;
}

static void output_cv(const b3_output *o, uint32_t out[8]) {
  b3ref_compress_cv(o->cv, o->block, o->block_len, o->counter, o->flags, out);
}

static void output_root_bytes(const b3_output *o, uint8_t out[32]) {
  uint32_t v[16];
  b3_compress_state(o->cv, o->block, o->block_len, 0, (uint8_t)(o->flags | B3REF_ROOT), v);
  for (int i = 0; i < 8; i++) store_le32(out + 4 * i, v[i] ^ v[i + 8]);
}

/* ---- hasher --------------------------------------------------------------- */

void b3ref_hasher_init(b3ref_hasher *h) {
  chunk_init(&h->chunk, 0);
  h->stack_len = 0;
}

/* Merge subtrees whose completion is proven by total_chunks: after the merge
 * the stack holds exactly one entry per 1-bit of total_chunks. */
static void merge_stack(b3ref_hasher *h, uint64_t total_chunks) {
  unsigned keep = (unsigned)__builtin_popcountll(total_chunks);
  while (h->stack_len > keep) {
    b3_output p = parent_output(h->stack[h->stack_len - 2], h->stack[h->stack_len - 1]);
    output_cv(&p, h->stack[h->stack_len - 2]);
    h->stack_len--;
  }
}

static void push_cv(b3ref_hasher *h, const uint32_t cv[8], uint64_t chunk_counter) {
  merge_stack(h, chunk_counter);
  memcpy(h->stack[h->stack_len], cv, 32);
  h->stack_len++;
}

void b3ref_hasher_update(b3ref_hasher *h, const void *data, size_t n) {
  const uint8_t *in = (const uint8_t *)data;
  while (n > 0) {
    if (chunk_len(&h->chunk) == B3REF_CHUNK_LEN) {
      /* a full chunk followed by more input is a non-root leaf */
      b3_output o = chunk_output(&h->chunk);
      uint32_t cv[8];
      output_cv(&o, cv);
      /* merge what the chunks before this one have completed, then push it */
      push_cv(h, cv, h->chunk.counter);
      chunk_init(&h->chunk, h->chunk.counter + 1);
    }
    size_t take = B3REF_CHUNK_LEN - chunk_len(&h->chunk);
    if (take > n) take = n;
    chunk_update(&h->chunk, in, take);
    in += take;
    n -= take;
  }
}

void b3ref_hasher_finalize(const b3ref_hasher *h0, uint8_t out[32]) {
  b3ref_hasher h = *h0;
  /* the stack may still hold completed-but-unmerged subtrees; merge them under
   * the final chunk's start position, then fold right-to-left */
  merge_stack(&h, h.chunk.counter);
  b3_output o = chunk_output(&h.chunk);
  for (int i = (int)h.stack_len - 1; i >= 0; i--) {
    uint32_t cv[8];
    output_cv(&o, cv);
    o = parent_output(h.stack[i], cv);
  }
  output_root_bytes(&o, out);
}

void b3ref_hash(const void *data, size_t n, uint8_t out[32]) {
  b3ref_hasher h;
  b3ref_hasher_init(&h);
  b3ref_hasher_update(&h, data, n);
  b3ref_hasher_finalize(&h, out);
}

/* parent node CV helper used by tests of subtree decompositions */
void b3ref_parent_cv(const uint32_t left[8], const uint32_t right[8], int root, uint32_t out[8]) {
  b3_output p = parent_output(left, right);
  if (root) {
    uint8_t bytes[32];
    output_root_bytes(&p, bytes);
    for (int i = 0; i < 8; i++) out[i] = load_le32(bytes + 4 * i);
  } else {
    output_cv(&p, out);
  }
}
