// b3_device.h — BLAKE3 compression for gfx950, one message block per lane.
//
// Replaces the arithmetic of the third-party `blake3` 1.5.0 crate that
// sd-core calls at core/src/object/cas.rs:24-61 and
// core/src/object/validation/hash.rs:13-22 (Hasher::update/finalize).
// Pure 32-bit integer ARX: every G step is v_add3_u32 + v_xor_b32 +
// v_alignbit_b32, the seven rounds are fully unrolled with the message
// permutation resolved at compile time, so a lane's compression is ~680 VALU
// instructions with no data movement between lanes (the CPU crate's
// `hash_many` transposes words into SIMD lanes; on CDNA every lane loads its
// own block, so no transpose exists).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace b3d {

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au;
constexpr uint32_t IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;

enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
constexpr uint32_t BLOCK_LEN = 64;
constexpr uint32_t CHUNK_LEN = 1024;

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

#define B3_G(a, b, c, d, x, y) \
  do {                         \
    a = a + b + (x);           \
    d = rotr(d ^ a, 16);       \
    c = c + d;                 \
    b = rotr(b ^ c, 12);       \
    a = a + b + (y);           \
    d = rotr(d ^ a, 8);        \
    c = c + d;                 \
    b = rotr(b ^ c, 7);        \
  } while (0)

// The same G as ONE inline-asm block: its twelve instructions issue in
// dependence order, and each v_alignbit_b32 is followed by "s_nop 0", which
// parks the issuing wave for one cycle so that the SIMD's other waves take the
// VALU. Measured on gfx950 with a register-only compression loop
// (tools/ubench_compress.hip, profiles/r02_ubench_compress.txt): the
// compiler's schedule of B3_G (the four G's of a half-round interleaved)
// sustains 58 G compressions/s, this block 67 G/s at 8 waves per SIMD, the
// block without the nops 58 G/s. Plain VALU ops on VGPRs, so no hazard needs a
// wait state inside the block.
#define B3_G_ASM(a, b, c, d, x, y)                                                           \
  asm volatile(                                                                              \
      "v_add3_u32 %0, %0, %1, %4\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 16\n"   \
      " s_nop 0\n v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n"                             \
      " v_alignbit_b32 %1, %1, %1, 12\n s_nop 0\n v_add3_u32 %0, %0, %1, %5\n"               \
      " v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 8\n s_nop 0\n"                     \
      " v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"        \
      " s_nop 0\n"                                                                          \
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)                                                   \
      : "v"(x), "v"(y))

// The first round's four column steps read c = an IV word and d = a word of
// (counter, block length, flags) only once, so they take them as inputs: c
// from an SGPR, d from the caller's VGPR, and write fresh c, d (no copies of
// the inputs into the state registers).
#define B3_G_ASM_FIRST(a, b, c, d, cin, din, x, y)                                           \
  asm volatile(                                                                              \
      "v_add3_u32 %0, %0, %1, %6\n v_xor_b32 %3, %5, %0\n v_alignbit_b32 %3, %3, %3, 16\n"   \
      " s_nop 0\n v_add_u32 %2, %4, %3\n v_xor_b32 %1, %1, %2\n"                             \
      " v_alignbit_b32 %1, %1, %1, 12\n s_nop 0\n v_add3_u32 %0, %0, %1, %7\n"               \
      " v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 8\n s_nop 0\n"                     \
      " v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"        \
      " s_nop 0\n"                                                                          \
      : "+v"(a), "+v"(b), "=&v"(c), "=&v"(d)                                                 \
      : "s"(cin), "v"(din), "v"(x), "v"(y))

// one round; s0..s15 = this round's message schedule (compile-time); G = the
// G step (B3_G or B3_G_ASM)
#define B3_ROUND_G(G, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  do {                                                                                     \
    G(v0, v4, v8, v12, m[s0], m[s1]);                                                      \
    G(v1, v5, v9, v13, m[s2], m[s3]);                                                      \
    G(v2, v6, v10, v14, m[s4], m[s5]);                                                     \
    G(v3, v7, v11, v15, m[s6], m[s7]);                                                     \
    G(v0, v5, v10, v15, m[s8], m[s9]);                                                     \
    G(v1, v6, v11, v12, m[s10], m[s11]);                                                   \
    G(v2, v7, v8, v13, m[s12], m[s13]);                                                    \
    G(v3, v4, v9, v14, m[s14], m[s15]);                                                    \
  } while (0)
#define B3_ROUND(...) B3_ROUND_G(B3_G, __VA_ARGS__)

#define B3_SIX_ROUNDS(G)                                                   \
  B3_ROUND_G(G, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);    \
  B3_ROUND_G(G, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);    \
  B3_ROUND_G(G, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);    \
  B3_ROUND_G(G, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);    \
  B3_ROUND_G(G, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);    \
  B3_ROUND_G(G, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13)

// cv <- first 8 words of compress(cv, m, counter, block_len, flags).
// For a ROOT compression these 8 words are the 32 digest bytes (LE words),
// because the root's output-block counter is 0 and every root on this path
// (a single chunk, or a parent) has counter 0 as well.
// GA = 0: compiler-scheduled G steps; GA = 1: B3_G_ASM blocks; GA = 2:
// B3_G_ASM with the first column steps as B3_G_ASM_FIRST.
#define B3_ROUND0(G) B3_ROUND_G(G, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
template <int GA = 0>
__device__ __forceinline__ void compress(uint32_t (&cv)[8], const uint32_t (&m)[16], uint64_t counter,
                                         uint32_t block_len, uint32_t flags) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3];
  uint32_t v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  if constexpr (GA == 2) {
    uint32_t v8, v9, v10, v11, v12, v13, v14, v15;
    const uint32_t c_lo = (uint32_t)counter, c_hi = (uint32_t)(counter >> 32);
    B3_G_ASM_FIRST(v0, v4, v8, v12, IV0, c_lo, m[0], m[1]);
    B3_G_ASM_FIRST(v1, v5, v9, v13, IV1, c_hi, m[2], m[3]);
    B3_G_ASM_FIRST(v2, v6, v10, v14, IV2, block_len, m[4], m[5]);
    B3_G_ASM_FIRST(v3, v7, v11, v15, IV3, flags, m[6], m[7]);
    B3_G_ASM(v0, v5, v10, v15, m[8], m[9]);
    B3_G_ASM(v1, v6, v11, v12, m[10], m[11]);
    B3_G_ASM(v2, v7, v8, v13, m[12], m[13]);
    B3_G_ASM(v3, v4, v9, v14, m[14], m[15]);
    B3_SIX_ROUNDS(B3_G_ASM);
    cv[0] = v0 ^ v8;
    cv[1] = v1 ^ v9;
    cv[2] = v2 ^ v10;
    cv[3] = v3 ^ v11;
    cv[4] = v4 ^ v12;
    cv[5] = v5 ^ v13;
    cv[6] = v6 ^ v14;
    cv[7] = v7 ^ v15;
    return;
  }
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
  uint32_t v12 = (uint32_t)counter, v13 = (uint32_t)(counter >> 32), v14 = block_len, v15 = flags;
  if constexpr (GA) {
    B3_ROUND0(B3_G_ASM);
    B3_SIX_ROUNDS(B3_G_ASM);
  } else {
    B3_ROUND0(B3_G);
    B3_SIX_ROUNDS(B3_G);
  }
  cv[0] = v0 ^ v8;
  cv[1] = v1 ^ v9;
  cv[2] = v2 ^ v10;
  cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12;
  cv[5] = v5 ^ v13;
  cv[6] = v6 ^ v14;
  cv[7] = v7 ^ v15;
}

__device__ __forceinline__ void set_iv(uint32_t (&cv)[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
  cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// parent node: message = left CV || right CV, counter 0, 64-byte block
template <int GA = 0>
__device__ __forceinline__ void parent(const uint32_t (&l)[8], const uint32_t (&r)[8], bool root,
                                       uint32_t (&out)[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  set_iv(out);
  compress<GA>(out, m, 0, BLOCK_LEN, PARENT | (root ? ROOT : 0u));
}

// ---- quad-cooperative compression, for chains that wait on each compression --
//
// One compression by the four lanes of a quad (q = lane & 3): lane q holds
// column q of the state (v[q], v[4+q], v[8+q], v[12+q]) and runs the column
// step's G for column q, then — its rows rotated within the quad by DPP
// (b from lane q+1, c from q+2, d from q+3) — the diagonal step's G for
// diagonal q, and rotates back. Every lane holds the whole message block and
// picks its round's four words by q. Per lane ~7 × (24 ARX + 6 DPP + 12
// selects) instructions, of which the dependent chain is ~7 × 26, against 680
// for one lane alone: where one compression waits on the previous one
// (k_finish_t's merges of a message's tile-crossing nodes) and nothing else
// fills the SIMD, the chain is what costs. Every lane of an active quad must
// be active (DPP reads the quad's other lanes).
template <int P>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, P, 0xF, 0xF, false);
}
// quad_perm controls: lane q reads lane (q+1)&3 / (q+2)&3 / (q+3)&3 of its quad
constexpr int kQ1 = 0x39, kQ2 = 0x4E, kQ3 = 0x93;

__device__ __forceinline__ uint32_t qsel(bool q1, bool q2, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return q2 ? (q1 ? d : c) : (q1 ? b : a);
}

#define B3_QROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  do {                                                                                 \
    const uint32_t x0 = qsel(q1, q2, m[s0], m[s2], m[s4], m[s6]);                      \
    const uint32_t y0 = qsel(q1, q2, m[s1], m[s3], m[s5], m[s7]);                      \
    const uint32_t x1 = qsel(q1, q2, m[s8], m[s10], m[s12], m[s14]);                   \
    const uint32_t y1 = qsel(q1, q2, m[s9], m[s11], m[s13], m[s15]);                   \
    B3_G(a, b, c, d, x0, y0);                                                          \
    b = qperm<kQ1>(b);                                                                 \
    c = qperm<kQ2>(c);                                                                 \
    d = qperm<kQ3>(d);                                                                 \
    B3_G(a, b, c, d, x1, y1);                                                          \
    b = qperm<kQ3>(b);                                                                 \
    c = qperm<kQ2>(c);                                                                 \
    d = qperm<kQ1>(d);                                                                 \
  } while (0)

// out <- compress(cv, m, counter, block_len, flags)'s first 8 words, in every
// lane of the quad (cv and m identical across the quad)
__device__ __forceinline__ void compress_quad(const uint32_t (&cv)[8], const uint32_t (&m)[16], uint64_t counter,
                                              uint32_t block_len, uint32_t flags, uint32_t (&out)[8]) {
  const uint32_t q = __lane_id() & 3u;
  const bool q1 = q & 1u, q2 = q & 2u;
  uint32_t a = qsel(q1, q2, cv[0], cv[1], cv[2], cv[3]);
  uint32_t b = qsel(q1, q2, cv[4], cv[5], cv[6], cv[7]);
  uint32_t c = qsel(q1, q2, IV0, IV1, IV2, IV3);
  uint32_t d = qsel(q1, q2, (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags);
  B3_QROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  B3_QROUND(2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);
  B3_QROUND(3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);
  B3_QROUND(10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);
  B3_QROUND(12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);
  B3_QROUND(9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);
  B3_QROUND(11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13);
  const uint32_t lo = a ^ c, hi = b ^ d;  // words q and 4 + q of the output
  out[0] = qperm<0x00>(lo);
  out[1] = qperm<0x55>(lo);
  out[2] = qperm<0xAA>(lo);
  out[3] = qperm<0xFF>(lo);
  out[4] = qperm<0x00>(hi);
  out[5] = qperm<0x55>(hi);
  out[6] = qperm<0xAA>(hi);
  out[7] = qperm<0xFF>(hi);
}

// The same compression with each lane's message words already picked (round
// 6, the small-batch kernel's QD 3): w[4r..4r+3] are the words lane q's G
// steps take in round r — m[s(2q)], m[s(2q+1)], m[s(8+2q)], m[s(9+2q)] for
// round r's schedule s (kQuadWord) — read from the block staged in LDS, so no
// lane selects them from the whole block (compress_quad's 84 v_cndmask per
// compression, more than a quarter of its instructions).
#define B3_QROUND_W(r)                  \
  do {                                  \
    B3_G(a, b, c, d, w[4 * (r)], w[4 * (r) + 1]);         \
    b = qperm<kQ1>(b);                  \
    c = qperm<kQ2>(c);                  \
    d = qperm<kQ3>(d);                  \
    B3_G(a, b, c, d, w[4 * (r) + 2], w[4 * (r) + 3]);     \
    b = qperm<kQ3>(b);                  \
    c = qperm<kQ2>(c);                  \
    d = qperm<kQ1>(d);                  \
  } while (0)

__device__ __forceinline__ void compress_quad_w(const uint32_t (&cv)[8], const uint32_t (&w)[28], uint64_t counter,
                                                uint32_t block_len, uint32_t flags, uint32_t (&out)[8]) {
  const uint32_t q = __lane_id() & 3u;
  const bool q1 = q & 1u, q2 = q & 2u;
  uint32_t a = qsel(q1, q2, cv[0], cv[1], cv[2], cv[3]);
  uint32_t b = qsel(q1, q2, cv[4], cv[5], cv[6], cv[7]);
  uint32_t c = qsel(q1, q2, IV0, IV1, IV2, IV3);
  uint32_t d = qsel(q1, q2, (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags);
  B3_QROUND_W(0);
  B3_QROUND_W(1);
  B3_QROUND_W(2);
  B3_QROUND_W(3);
  B3_QROUND_W(4);
  B3_QROUND_W(5);
  B3_QROUND_W(6);
  const uint32_t lo = a ^ c, hi = b ^ d;
  out[0] = qperm<0x00>(lo);
  out[1] = qperm<0x55>(lo);
  out[2] = qperm<0xAA>(lo);
  out[3] = qperm<0xFF>(lo);
  out[4] = qperm<0x00>(hi);
  out[5] = qperm<0x55>(hi);
  out[6] = qperm<0xAA>(hi);
  out[7] = qperm<0xFF>(hi);
}

// kQuadWord[q][4r + k]: the message word lane q's k-th G input of round r
// takes (the schedules of compress_quad's seven B3_QROUNDs)
struct QuadWords {
  uint8_t w[4][28];
};
constexpr QuadWords make_quad_words() {
  constexpr uint8_t s[7][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                                {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                                {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                                {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                                {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                                {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                                {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
  QuadWords t{};
  for (int q = 0; q < 4; ++q)
    for (int r = 0; r < 7; ++r) {
      t.w[q][4 * r] = s[r][2 * q];
      t.w[q][4 * r + 1] = s[r][2 * q + 1];
      t.w[q][4 * r + 2] = s[r][8 + 2 * q];
      t.w[q][4 * r + 3] = s[r][9 + 2 * q];
    }
  return t;
}
constexpr QuadWords kQuadWord = make_quad_words();

__device__ __forceinline__ void parent_quad(const uint32_t (&l)[8], const uint32_t (&r)[8], bool root,
                                            uint32_t (&out)[8]) {
  uint32_t m[16], iv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  set_iv(iv);
  compress_quad(iv, m, 0, BLOCK_LEN, PARENT | (root ? ROOT : 0u), out);
}

// 64 message bytes, 16-byte aligned, fully inside the message
__device__ __forceinline__ void load_full_block(const uint8_t* p, uint32_t (&m)[16]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  m[0] = a.x; m[1] = a.y; m[2] = a.z; m[3] = a.w;
  m[4] = b.x; m[5] = b.y; m[6] = b.z; m[7] = b.w;
  m[8] = c.x; m[9] = c.y; m[10] = c.z; m[11] = c.w;
  m[12] = d.x; m[13] = d.y; m[14] = d.z; m[15] = d.w;
}

// the same with non-temporal (streaming) loads: message bytes are read once
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load_full_block_nt(const uint8_t* p, uint32_t (&m)[16]) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  u32x4 a = __builtin_nontemporal_load(q), b = __builtin_nontemporal_load(q + 1);
  u32x4 c = __builtin_nontemporal_load(q + 2), d = __builtin_nontemporal_load(q + 3);
  m[0] = a.x; m[1] = a.y; m[2] = a.z; m[3] = a.w;
  m[4] = b.x; m[5] = b.y; m[6] = b.z; m[7] = b.w;
  m[8] = c.x; m[9] = c.y; m[10] = c.z; m[11] = c.w;
  m[12] = d.x; m[13] = d.y; m[14] = d.z; m[15] = d.w;
}

// Zero the bytes of a just-loaded block that lie past `blen` (< 64): the last
// block of a message is loaded as a full 64-byte block (the blob carries at
// least 64 readable bytes after every message, see sdcas.h) and masked here,
// so no lane ever branches into byte loads.
__device__ __forceinline__ void mask_tail(uint32_t (&m)[16], uint32_t blen) {
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const int r = (int)blen - 4 * w;
    const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : (r <= 0 ? 0u : ((1u << (8 * r)) - 1u));
    m[w] &= keep;
  }
}

// digest bytes 0..7 as a big-endian u64 (so "%016llx" == to_hex()[..16])
__device__ __forceinline__ uint64_t cas_key(const uint32_t (&d)[8]) {
  return ((uint64_t)__builtin_bswap32(d[0]) << 32) | (uint64_t)__builtin_bswap32(d[1]);
}

}  // namespace b3d
