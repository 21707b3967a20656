// b3_batch.hip — batched multi-message BLAKE3 on gfx950.
//
// One launch hashes n independent messages (cas_id messages of
// core/src/object/cas.rs:23-62, or whole files for
// core/src/object/validation/hash.rs:11-25) that sit in HBM at 16-byte aligned
// offsets of one blob.
//
// Layout: every 1 KiB chunk of every message gets one "slot" of a flat slot
// space (message m owns slots [S[m], S[m] + C[m]), C = max(1, ceil(len/1024)),
// S = exclusive scan of C). Slots are cut into TILEs of 1024; one workgroup
// owns one tile at a time (grid-stride over tiles), so every lane of every
// wave hashes a chunk — no per-message padding, no idle lanes except in the
// very last tile.
//
//   k_tile_first   which message owns each tile's first slot (lane/message)
//   k_leaf_tree    per tile: (1) each lane hashes its chunk (16 compressions,
//                  blocks straight from HBM as 4 x dwordx4 per block, next
//                  block prefetched); single-chunk messages finish here as
//                  ROOT. (2) chunk CVs go to LDS and every BLAKE3 tree node
//                  that is an aligned, complete power-of-two block lying
//                  inside the tile is reduced level by level (PARENT
//                  compressions over a compacted task list). (3) the maximal
//                  such nodes are written to `nodes` at their first slot.
//   k_finish_t     lane per tile boundary (the message crossing it first):
//                  walks its maximal nodes left to right (the decomposition is
//                  a closed-form function of (chunk index, chunk count, slot
//                  in tile)) and merges them with the BLAKE3 subtree-stack
//                  rule, the stack in LDS; the last merge is ROOT.
//
// The tree a message gets is exactly BLAKE3's left-balanced tree: complete
// aligned power-of-two subtrees are tree nodes, and the stack merge (merge
// while the stack is longer than popcount(chunks so far), then fold
// right-to-left) reassembles them in the crate's order.
//
// Only bit-exact, GPU-tested kernels are compiled into libsdcas.so. The
// layouts and block loops that lost round 1's A/B runs (and two diagnostic
// loops that skip memory reads or compressions, i.e. produce wrong digests)
// live in b3_ablate_*.inc and are compiled only with -DSDCAS_ABLATIONS into
// libsdcas_ablate.so, which only tools/ab_leaf.py loads.
#include <hip/hip_runtime.h>

#include <atomic>
#ifdef SDCAS_ABLATIONS
#include <hipcub/hipcub.hpp>  // the quad-layout ablation's scan only
#endif
#include <stdint.h>
#include <cstdio>
#include <cstring>

#include "b3_device.h"
#include "b3_batch.h"

namespace sdcas {

using namespace b3d;

constexpr int kMaxStack = 64;
constexpr int kMaxStackBig = 64;

__host__ __device__ inline uint64_t chunk_count(uint64_t len) { return len == 0 ? 1 : (len + CHUNK_LEN - 1) / CHUNK_LEN; }

// Highest level k such that the node of 2^k chunks starting at chunk j is
// (a) an aligned complete block of the message, (b) not the whole message and
// (c) inside the tile that holds chunk j at slot `s`.
// Closed form (checked against the defining loop — grow k while the node of
// 2^(k+1) chunks at j is aligned, fits the message, is not the whole message
// and fits the tile — on 2 M random cases): the largest k with 2^k dividing j,
// 2^k <= C - j, 2^k < C and 2^k <= TILE - s.
__host__ __device__ inline uint32_t floor_log2(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }  // x > 0

template <uint32_t TILE>
__host__ __device__ inline uint32_t node_level_t(uint64_t j, uint64_t C, uint32_t s) {
  if (C <= 1) return 0;
  const uint32_t a = j ? (uint32_t)__builtin_ctzll(j) : 63u;
  const uint32_t b = min(floor_log2(C - j), floor_log2(C - 1));
  return min(min(a, b), floor_log2((uint64_t)TILE - s));
}

__host__ __device__ inline uint32_t node_level(uint64_t j, uint64_t C, uint32_t s) { return node_level_t<kTile>(j, C, s); }

// Is the level-k node at (j, s) consumed by a parent computed in the same tile?
template <uint32_t TILE>
__host__ __device__ inline bool parent_in_tile_t(uint64_t j, uint64_t C, uint32_t s, uint32_t k) {
  uint64_t w = 1ull << k;
  if (!((j >> k) & 1)) return false;
  return j + w <= C && 2 * w < C && s >= w && (uint64_t)s + w <= TILE;
}

__host__ __device__ inline bool parent_in_tile(uint64_t j, uint64_t C, uint32_t s, uint32_t k) {
  uint64_t w = 1ull << k;
  if (!((j >> k) & 1)) return false;  // left children's parents start at s: not computed
  return j + w <= C && 2 * w < C && s >= w && (uint64_t)s + w <= kTile;
}


template <uint32_t TILE = kTile>
__global__ void k_tile_first(const uint64_t* __restrict__ lens, const uint64_t* __restrict__ S, uint32_t n,
                             uint64_t cap_chunks, uint32_t* __restrict__ tile_first, uint64_t* __restrict__ total) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint64_t s0 = S[m], C = chunk_count(lens[m]);
  if (m == n - 1) {
    total[0] = s0 + C;
    total[2] = 0;  // k_leaf_tree<DYN>'s tile counter
  }
  for (uint64_t t = (s0 + TILE - 1) / TILE; t * TILE < s0 + C && t * TILE < cap_chunks; ++t) tile_first[t] = m;
}

// The batch's slot plan without a library scan: S = the exclusive prefix sum
// of the messages' chunk counts, tile_first and total as k_tile_first writes
// them. (1) each workgroup sums the chunk counts of its 4096 messages, (2) one
// workgroup turns those sums into offsets (and the total), (3) each workgroup
// rescans its messages from its offset, 256 at a time, writing S and
// tile_first. Three launches at the HBM rate of reading lens twice and writing
// S once, against rocPRIM's look-back scan (two launches) + k_tile_first:
// C5 (6.25 M messages) 78 us -> ~40 us.
constexpr uint32_t kPlanWG = 256, kPlanR = 16, kPlanPer = kPlanWG * kPlanR;

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}

__global__ void __launch_bounds__(kPlanWG) k_plan_sums(const uint64_t* __restrict__ lens, uint32_t n,
                                                       uint64_t* __restrict__ bsum) {
  __shared__ uint64_t ws[kPlanWG / 64];
  const uint64_t lo = (uint64_t)blockIdx.x * kPlanPer;
  uint64_t L[kPlanR];
#pragma unroll
  for (uint32_t r = 0; r < kPlanR; ++r) {
    const uint64_t i = lo + r * kPlanWG + threadIdx.x;
    L[r] = i < n ? lens[i] : 0;
  }
  uint64_t s = 0;
#pragma unroll
  for (uint32_t r = 0; r < kPlanR; ++r)
    if (lo + r * kPlanWG + threadIdx.x < n) s += chunk_count(L[r]);
#pragma unroll
  for (uint32_t d = 32; d; d >>= 1) s += __shfl_xor(s, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
#pragma unroll
    for (uint32_t w = 0; w < kPlanWG / 64; ++w) t += ws[w];
    bsum[blockIdx.x] = t;
  }
}

// one workgroup: bsum[b] <- the exclusive prefix of the workgroup sums
__global__ void __launch_bounds__(1024) k_plan_scan(uint64_t* __restrict__ bsum, uint32_t nb,
                                                    uint64_t* __restrict__ total) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += 1024) {
    const uint32_t i = base + tid;
    const uint64_t v = i < nb ? bsum[i] : 0;
    const uint64_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += ws[w];
    if (i < nb) bsum[i] = before + inc - v;
    __syncthreads();
    if (tid == 1023) carry = before + inc;  // the last thread's inclusive total
    __syncthreads();
  }
  if (tid == 0) {
    total[0] = carry;
    total[2] = 0;  // k_leaf_tree<DYN>'s tile counter
  }
}

template <uint32_t TILE>
__global__ void __launch_bounds__(kPlanWG) k_plan_write(const uint64_t* __restrict__ lens, uint32_t n,
                                                        const uint64_t* __restrict__ boff, uint64_t cap_chunks,
                                                        uint64_t* __restrict__ S, uint32_t* __restrict__ tile_first) {
  __shared__ uint64_t ws[kPlanWG / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lo = (uint64_t)blockIdx.x * kPlanPer;
  uint64_t L[kPlanR];
#pragma unroll
  for (uint32_t r = 0; r < kPlanR; ++r) {
    const uint64_t i = lo + r * kPlanWG + tid;
    L[r] = i < n ? lens[i] : 0;
  }
  uint64_t run = boff[blockIdx.x];
#pragma unroll 1
  for (uint32_t r = 0; r < kPlanR && lo + r * kPlanWG < n; ++r) {
    const uint64_t m = lo + r * kPlanWG + tid;
    const uint64_t C = m < n ? chunk_count(L[r]) : 0;
    const uint64_t inc = wave_incl_scan(C, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t s0 = run;
    uint64_t all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kPlanWG / 64; ++w) {
      if (w < wave) s0 += ws[w];
      all += ws[w];
    }
    s0 += inc - C;
    __syncthreads();
    run += all;
    if (m < n) {
      S[m] = s0;
      for (uint64_t t = (s0 + TILE - 1) / TILE; t * TILE < s0 + C && t * TILE < cap_chunks; ++t)
        tile_first[t] = (uint32_t)m;
    }
  }
}

// Same, unrolled by two blocks with ping-pong message registers (no
// register copies between blocks; block b+1's loads fly while b compresses).
template <int GA = 0>
__device__ __forceinline__ void hash_chunk_pp(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                              uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  uint32_t m0[16], m1[16];
  load_full_block(p, m0);
#pragma unroll 1
  for (uint32_t b = 0; b < nb; b += 2) {
    load_full_block(p + min(b + 1, nb - 1) * BLOCK_LEN, m1);
    {
      const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m0, blen);
      compress<GA>(cv, m0, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));
    }
    if (b + 1 < nb) {
      load_full_block(p + min(b + 2, nb - 1) * BLOCK_LEN, m0);
      const uint32_t blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m1, blen);
      compress<GA>(cv, m1, j, blen, b + 2 == nb ? endf : 0u);
    }
  }
}

// Same two register sets as the ping-pong loop, but both 64-byte halves of a
// 128-byte line are requested together (no prefetch across lines): the second
// half never waits in L2 for a compression and cannot be evicted before it is
// read; the load latency is left to the other waves of the SIMD.
template <int GA = 0>
__device__ __forceinline__ void hash_chunk_ps(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                              uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  uint32_t m0[16], m1[16];
#pragma unroll 1
  for (uint32_t b = 0; b < nb; b += 2) {
    load_full_block(p + b * BLOCK_LEN, m0);
    load_full_block(p + min(b + 1, nb - 1) * BLOCK_LEN, m1);
    {
      const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m0, blen);
      compress<GA>(cv, m0, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));
    }
    if (b + 1 < nb) {
      const uint32_t blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m1, blen);
      compress<GA>(cv, m1, j, blen, b + 2 == nb ? endf : 0u);
    }
  }
}

// Tail masks by the length of a message's last block: row b keeps bytes
// [0, b) of a 64-byte block (word w: all ones, none, or its low 8 * (b - 4w)
// bits). Four 16-byte loads of an L1-resident 4 KiB table replace the ~100
// VALU instructions of computing the sixteen masks.
struct alignas(16) TailMasks {
  uint32_t w[BLOCK_LEN + 1][16];
};
constexpr TailMasks make_tail_masks() {
  TailMasks t{};
  for (int b = 0; b <= (int)BLOCK_LEN; ++b)
    for (int w = 0; w < 16; ++w) {
      const int r = b - 4 * w;
      t.w[b][w] = r >= 4 ? 0xFFFFFFFFu : (r <= 0 ? 0u : ((1u << (8 * r)) - 1u));
    }
  return t;
}
__device__ const TailMasks kTailMasks = make_tail_masks();

__device__ __forceinline__ void mask_tail_table(uint32_t (&m)[16], uint32_t blen) {
  const uint4* q = reinterpret_cast<const uint4*>(kTailMasks.w[blen]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = q[k];
    m[4 * k] &= v.x;
    m[4 * k + 1] &= v.y;
    m[4 * k + 2] &= v.z;
    m[4 * k + 3] &= v.w;
  }
}

// A chunk known to be whole (1024 bytes, not the root): sixteen full blocks,
// both halves of each 128-byte line requested together as in hash_chunk_ps;
// the block index is wave-uniform, so the flags are scalar selects and no
// lane computes a length or a tail mask.
template <int GA = 0>
__device__ __forceinline__ void hash_chunk_full(const uint8_t* __restrict__ p, uint64_t j, uint32_t (&cv)[8]) {
  set_iv(cv);
  uint32_t m0[16], m1[16];
#pragma unroll 1
  for (uint32_t b = 0; b < CHUNK_LEN / BLOCK_LEN; b += 2) {
    load_full_block(p + b * BLOCK_LEN, m0);
    load_full_block(p + (b + 1) * BLOCK_LEN, m1);
    compress<GA>(cv, m0, j, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
    compress<GA>(cv, m1, j, BLOCK_LEN, b + 2 == CHUNK_LEN / BLOCK_LEN ? CHUNK_END : 0u);
  }
}

// The line-pair loop with its per-block bookkeeping cut to compares against
// the chunk's last block index (computed once): a full block's length and
// flags are constants selected by one compare, the tail mask runs only on
// the last block, the second half of a line is loaded only if the chunk has
// it (no clamped address), and the block pointer advances by one add.
template <int GA = 0, int NT = 0, int LM = 0, uint32_t BS = BLOCK_LEN, int MT = 0>
__device__ __forceinline__ void hash_chunk_pl(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                              uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t lb = clen <= BLOCK_LEN ? 0u : (clen - 1) / BLOCK_LEN;  // last block index
  const uint32_t lblen = clen - lb * BLOCK_LEN;                          // its length (0 only for an empty message)
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  const uint8_t* q = p;
#pragma unroll 1
  for (uint32_t b = 0; b <= lb; b += 2, q += 2 * BS) {
    // m1 is loaded only when the chunk has the second block; left undefined
    // otherwise, the compiler zeroed its sixteen registers before the loop
    // (16 v_mov per chunk). An empty asm defines them as "whatever is there".
    uint32_t m0[16], m1[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) asm volatile("" : "=v"(m1[w]));
    const bool two = b + 1 <= lb;
    if constexpr (NT) {
      load_full_block_nt(q, m0);
      if (two) load_full_block_nt(q + BS, m1);
    } else {
      load_full_block(q, m0);
      if (two) load_full_block(q + BS, m1);
    }
    {
      const bool last = b == lb;
      if (last && lblen < BLOCK_LEN) {
        uint32_t L = lblen;
        if constexpr (LM) asm volatile("" : "+v"(L));  // keeps the mask inside the branch
        if constexpr (MT) mask_tail_table(m0, L);
        else mask_tail(m0, L);
      }
      compress<GA>(cv, m0, j, last ? lblen : BLOCK_LEN, (b == 0 ? CHUNK_START : 0u) | (last ? endf : 0u));
    }
    if (two) {
      const bool last = b + 1 == lb;
      if (last && lblen < BLOCK_LEN) {
        uint32_t L = lblen;
        if constexpr (LM) asm volatile("" : "+v"(L));
        if constexpr (MT) mask_tail_table(m1, L);
        else mask_tail(m1, L);
      }
      compress<GA>(cv, m1, j, last ? lblen : BLOCK_LEN, last ? endf : 0u);
    }
  }
}

#ifdef SDCAS_ABLATIONS
#include "b3_ablate_loops.inc"
#endif

// One chunk by the four lanes of a quad (compress_quad), for batches whose
// chunks are so few that each chunk's 16-compression chain is the kernel's
// time (a lone file of the watcher or of browse): every lane loads the same
// block, the chain is ~1/3 of one lane's.
__device__ __forceinline__ void hash_chunk_quad(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                                uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t lb = clen <= BLOCK_LEN ? 0u : (clen - 1) / BLOCK_LEN;  // last block index
  const uint32_t lblen = clen - lb * BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  const uint8_t* q = p;
#pragma unroll 1
  for (uint32_t b = 0; b <= lb; ++b, q += BLOCK_LEN) {
    uint32_t m[16], o[8];
    load_full_block(q, m);
    const bool last = b == lb;
    if (last && lblen < BLOCK_LEN) mask_tail_table(m, lblen);
    compress_quad(cv, m, j, last ? lblen : BLOCK_LEN, (b == 0 ? CHUNK_START : 0u) | (last ? endf : 0u), o);
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = o[i];
  }
}

// The same chain with four blocks in flight (round 6): a lone chunk's loop
// above waits for each block's load before its compression, so a one-file
// call's kernel was the sum of 16 load latencies (the blocks arrive from L2
// or HBM right after their upload) and 16 compressions. Here block b + 4 is
// requested as soon as block b has been compressed, from a ring of four
// register sets (64 VGPRs: the quad kernel holds few waves), so a load has
// four compressions (~2 us) to land.
__device__ __forceinline__ void quad_block(const uint32_t (&m)[16], uint32_t b, uint32_t lb, uint32_t lblen,
                                           uint32_t endf, uint64_t j, uint32_t (&cv)[8]) {
  uint32_t mm[16], o[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) mm[i] = m[i];
  const bool last = b == lb;
  if (last && lblen < BLOCK_LEN) mask_tail_table(mm, lblen);
  compress_quad(cv, mm, j, last ? lblen : BLOCK_LEN, (b == 0 ? CHUNK_START : 0u) | (last ? endf : 0u), o);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = o[i];
}

__device__ __forceinline__ void hash_chunk_quad4(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                                 uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t lb = clen <= BLOCK_LEN ? 0u : (clen - 1) / BLOCK_LEN;  // last block index
  const uint32_t lblen = clen - lb * BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  uint32_t r0[16], r1[16], r2[16], r3[16];
  // blocks past the last are not loaded: their registers are "whatever is
  // there" (an empty asm defines them, as in hash_chunk_pl) and never read
#pragma unroll
  for (int w = 0; w < 16; ++w) asm volatile("" : "=v"(r1[w]), "=v"(r2[w]), "=v"(r3[w]));
  load_full_block(p, r0);
  if (lb >= 1) load_full_block(p + BLOCK_LEN, r1);
  if (lb >= 2) load_full_block(p + 2 * BLOCK_LEN, r2);
  if (lb >= 3) load_full_block(p + 3 * BLOCK_LEN, r3);
  const uint8_t* q = p + 4 * BLOCK_LEN;
#pragma unroll 1
  for (uint32_t b = 0;; b += 4, q += 4 * BLOCK_LEN) {
    quad_block(r0, b, lb, lblen, endf, j, cv);
    if (b + 4 <= lb) load_full_block(q, r0);
    if (b + 1 > lb) break;
    quad_block(r1, b + 1, lb, lblen, endf, j, cv);
    if (b + 5 <= lb) load_full_block(q + BLOCK_LEN, r1);
    if (b + 2 > lb) break;
    quad_block(r2, b + 2, lb, lblen, endf, j, cv);
    if (b + 6 <= lb) load_full_block(q + 2 * BLOCK_LEN, r2);
    if (b + 3 > lb) break;
    quad_block(r3, b + 3, lb, lblen, endf, j, cv);
    if (b + 7 <= lb) load_full_block(q + 3 * BLOCK_LEN, r3);
    if (b + 4 > lb) break;
  }
}

// QD 3 (round 6): a quad's block staged in LDS. Lane q loads only its
// quarter of each block (one dwordx4, four blocks in flight), writes it to the
// quad's 64-byte LDS buffer (qbuf[qslot..qslot+16)), and reads back the 28
// words its rounds take (word indices wi: kQuadWord for its q, with qslot
// added) for compress_quad_w — a lone quad's chain without the 84 selects per
// compression. The quad's lanes are one wave, whose LDS operations run in
// issue order, so a lane reads its quad's block after the write that holds it
// and the next block's write lands after these reads; the empty asm keeps the
// compiler from moving them across each other.
__device__ __forceinline__ void quad_lds_words(uint32_t* __restrict__ qbuf, uint32_t qslot, uint4 v,
                                               const uint32_t (&wi)[28], uint32_t (&w)[28]) {
  const uint32_t q = __lane_id() & 3u;
  asm volatile("" ::: "memory");
  *reinterpret_cast<uint4*>(&qbuf[qslot + 4 * q]) = v;
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < 28; ++k) w[k] = qbuf[wi[k]];
}

__device__ __forceinline__ void quad_lds_block(uint4 v, uint32_t b, uint32_t lb, uint32_t lblen, uint32_t endf,
                                               uint64_t j, uint32_t* __restrict__ qbuf, uint32_t qslot,
                                               const uint32_t (&wi)[28], uint32_t (&cv)[8]) {
  const bool last = b == lb;
  if (last && lblen < BLOCK_LEN) {
    const uint4 mk = reinterpret_cast<const uint4*>(kTailMasks.w[lblen])[__lane_id() & 3u];
    v.x &= mk.x;
    v.y &= mk.y;
    v.z &= mk.z;
    v.w &= mk.w;
  }
  uint32_t w[28], o[8];
  quad_lds_words(qbuf, qslot, v, wi, w);
  compress_quad_w(cv, w, j, last ? lblen : BLOCK_LEN, (b == 0 ? CHUNK_START : 0u) | (last ? endf : 0u), o);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = o[i];
}

__device__ __forceinline__ void hash_chunk_quad_lds(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j,
                                                    bool root, uint32_t* __restrict__ qbuf, uint32_t qslot,
                                                    const uint32_t (&wi)[28], uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t lb = clen <= BLOCK_LEN ? 0u : (clen - 1) / BLOCK_LEN;  // last block index
  const uint32_t lblen = clen - lb * BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  const uint4* src = reinterpret_cast<const uint4*>(p) + (__lane_id() & 3u);  // this lane's quarter of block 0
  uint4 g0, g1, g2, g3;
  // quarters of blocks past the last are not loaded (never read)
  asm volatile("" : "=v"(g1.x), "=v"(g1.y), "=v"(g1.z), "=v"(g1.w));
  asm volatile("" : "=v"(g2.x), "=v"(g2.y), "=v"(g2.z), "=v"(g2.w));
  asm volatile("" : "=v"(g3.x), "=v"(g3.y), "=v"(g3.z), "=v"(g3.w));
  g0 = src[0];
  if (lb >= 1) g1 = src[4];
  if (lb >= 2) g2 = src[8];
  if (lb >= 3) g3 = src[12];
#pragma unroll 1
  for (uint32_t b = 0;; b += 4) {
    quad_lds_block(g0, b, lb, lblen, endf, j, qbuf, qslot, wi, cv);
    if (b + 4 <= lb) g0 = src[4 * (b + 4)];
    if (b + 1 > lb) break;
    quad_lds_block(g1, b + 1, lb, lblen, endf, j, qbuf, qslot, wi, cv);
    if (b + 5 <= lb) g1 = src[4 * (b + 5)];
    if (b + 2 > lb) break;
    quad_lds_block(g2, b + 2, lb, lblen, endf, j, qbuf, qslot, wi, cv);
    if (b + 6 <= lb) g2 = src[4 * (b + 6)];
    if (b + 3 > lb) break;
    quad_lds_block(g3, b + 3, lb, lblen, endf, j, qbuf, qslot, wi, cv);
    if (b + 7 <= lb) g3 = src[4 * (b + 7)];
    if (b + 4 > lb) break;
  }
}

// Block loop of a leaf chunk: PF 8 = hash_chunk_ps, 9 = hash_chunk_pl, 4 =
// hash_chunk_pp, 59 = hash_chunk_full for a whole non-root chunk (per lane)
// else hash_chunk_ps, 69 = hash_chunk_full when every active lane of the wave
// holds a whole non-root chunk else hash_chunk_pl; PF + 100 = the same loop
// with the asm G blocks (B3_G_ASM, b3_device.h), PF + 200 = with the
// copy-free first column steps too (compress<2>); any other PF names an
// ablation loop.
template <int PF>
constexpr int kGA = PF / 100;
template <int PF>
__device__ __forceinline__ void leaf_hash(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                          uint32_t (&cv)[8]) {
  constexpr int L = PF % 100, GA = kGA<PF>;
  if constexpr (L == 8) {
    hash_chunk_ps<GA>(p, clen, j, root, cv);
  } else if constexpr (L == 9) {
    hash_chunk_pl<GA>(p, clen, j, root, cv);
  } else if constexpr (L == 4) {
    hash_chunk_pp<GA>(p, clen, j, root, cv);
  } else if constexpr (L == 59) {
    if (clen == CHUNK_LEN && !root) hash_chunk_full<GA>(p, j, cv);
    else hash_chunk_ps<GA>(p, clen, j, root, cv);
  } else if constexpr (L == 79) {
    hash_chunk_pl<GA, 0, 0, BLOCK_LEN, 1>(p, clen, j, root, cv);
  } else if constexpr (L == 89) {
    if (__all(clen == CHUNK_LEN && !root)) hash_chunk_full<GA>(p, j, cv);
    else hash_chunk_pl<GA, 0, 0, BLOCK_LEN, 1>(p, clen, j, root, cv);
  } else if constexpr (L == 69) {
    // a wave whose active lanes all hold whole non-root chunks takes the
    // full-chunk loop; any other wave the last-block-index loop
    if (__all(clen == CHUNK_LEN && !root)) hash_chunk_full<GA>(p, j, cv);
    else hash_chunk_pl<GA>(p, clen, j, root, cv);
  } else {
#ifdef SDCAS_ABLATIONS
    leaf_hash_ablation<PF>(p, clen, j, root, cv);  // b3_ablate_loops.inc
#else
    static_assert(L == 8 || L == 9 || L == 4 || L == 59 || L == 69 || L == 79 || L == 89, "ablation block loops need -DSDCAS_ABLATIONS");
#endif
  }
}

// the message address of a leaf chunk (an ablation loop may fold it)
template <int PF>
__device__ __forceinline__ const uint8_t* leaf_ptr(const uint8_t* blob, const uint8_t* p) {
#ifdef SDCAS_ABLATIONS
  return leaf_ptr_ablation<PF>(blob, p);
#else
  (void)blob;
  return p;
#endif
}

__device__ __forceinline__ void store_digest(uint32_t m, const uint32_t (&d)[8], uint8_t* out32, uint64_t* out_keys) {
  if (out32) {
    uint4* o = reinterpret_cast<uint4*>(out32 + 32ull * m);
    o[0] = make_uint4(d[0], d[1], d[2], d[3]);
    o[1] = make_uint4(d[4], d[5], d[6], d[7]);
  }
  if (out_keys) out_keys[m] = cas_key(d);
}

// per-level task regions of the in-tile tree: level k (1..10) holds at most
// 2 * (kTile >> k) tasks (regular level-k nodes are disjoint 2^k blocks, spine
// steps consume disjoint maximal 2^(k-1) blocks), 2046 entries in all
template <uint32_t TL = kTile>
__host__ __device__ constexpr uint32_t task_base(uint32_t k) { return 2 * (TL - (TL >> (k - 1))); }
template <uint32_t TL = kTile>
constexpr uint32_t kTaskCap = 2 * (TL - 1);
constexpr uint16_t kNoMsg = 0xFFFF;

__device__ __forceinline__ uint32_t enc_task(uint32_t l, uint32_t r, uint32_t msg, bool root) {
  return l | (r << 10) | (msg << 20) | (root ? 0x80000000u : 0u);
}

// leaf-order bin of chunk j of a message of `len` bytes: 16 - blocks (full
// chunks first), 0..15
__device__ __forceinline__ uint32_t leaf_bin(uint64_t len, uint64_t j) {
  const uint64_t rest = len - j * CHUNK_LEN;
  const uint32_t clen = len == 0 ? 0u : (uint32_t)min<uint64_t>(CHUNK_LEN, rest);
  const uint32_t nb = clen == 0 ? 1u : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  return 16u - nb;
}

// Leaf order of a tile by block count (ORD): the lanes of a wave run their
// chunks in lockstep, so a wave holding full chunks next to partial last
// chunks idles the short lanes (C5's small files: 13 % of lane time). Slots
// are ranked by bin (16 - blocks; past-the-end slots last) with one ballot
// per bin per 64-slot group, the 17 x 16 group counts are scanned by one wave,
// and lane i of the leaf loop takes slot order[i]. The tree and the node
// layout do not change: a leaf still writes its CV at its own slot.

template <int WG, uint32_t NB = 17, uint32_t TL = kTile>
__device__ __forceinline__ void leaf_order(uint32_t tid, const uint32_t (&bin)[TL / WG], uint16_t* __restrict__ order,
                                           uint16_t* __restrict__ gcnt) {
  constexpr uint32_t kGroups = TL / 64;
  const uint32_t lane = tid & 63;
  uint32_t rk[TL / WG];
#pragma unroll
  for (uint32_t r = 0; r < TL / WG; ++r) {
    const uint32_t g = (tid + r * WG) >> 6;
    uint32_t mine = 0, cnt_l = 0;
#pragma unroll 1
    for (uint32_t b = 0; b < NB; ++b) {
      const uint64_t m = __ballot(bin[r] == b);
      if (bin[r] == b) mine = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == b) cnt_l = (uint32_t)__popcll(m);
    }
    rk[r] = mine;
    if (lane < NB) gcnt[lane * kGroups + g] = (uint16_t)cnt_l;
  }
  __syncthreads();
  if (tid < 64) {
    // exclusive scan of the NB x kGroups counts in bin-major order
    constexpr uint32_t kPer = (NB * kGroups + 63) / 64;
    uint32_t v[kPer], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t e = tid * kPer + q;
      v[q] = e < NB * kGroups ? gcnt[e] : 0u;
      sum += v[q];
    }
    uint32_t inc = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    uint32_t acc = inc - sum;
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t e = tid * kPer + q;
      if (e < NB * kGroups) gcnt[e] = (uint16_t)acc;
      acc += v[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < TL / WG; ++r) {
    const uint32_t s = tid + r * WG;
    order[gcnt[bin[r] * kGroups + (s >> 6)] + rk[r]] = (uint16_t)s;
  }
  __syncthreads();
}

// MINW: waves per SIMD the register allocation must allow (0: 6 with the
// leaf order, else 1)
// TL: chunk slots per tile (kTile; kSmallTile for the small-batch kernel)
// QD: a quad of lanes per slot (WG = 4 x the slots a pass covers): each
// chunk and each tree node by compress_quad; the quad's lead lane alone
// writes shared state (task lists, chaining values, digests). Needs ORD 0 and
// CA 0. QD 2 (round 6): the same with four blocks of a chunk in flight
// (hash_chunk_quad4); QD 3: and each quad's block staged in LDS, every lane
// reading its rounds' words (hash_chunk_quad_lds, the tree's parents too).
// XT (round 5), bit 1: a tree level of at most 32 tasks — levels 5-10 in C2's
// tiles (30, 14, 7 ... tasks), each one wave of mostly idle lanes — runs its
// parents by quads of lanes (parent_quad: ~310 instructions per lane for a
// task, against 680 for a lone lane; two waves at most). Bit 2: phase 1 marks
// in a bit per slot which nodes of tile-crossing messages go to HBM, so that
// phase 4 reads one bit per slot instead of recomputing the message's shape.
// Bit 4: phase 1 appends a wave's tree tasks level by level with one LDS
// atomic per wave (a ballot and a lane count place each task).
template <int WG, int PF, int TR = 1, int ORD = 0, int DYN = 0, int CA = 0, int MINW = 0, uint32_t TL = kTile,
          int QD = 0, int XT = 0>
__global__ void __launch_bounds__(WG, MINW ? MINW : (ORD ? 6 : 1)) k_leaf_tree(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offs,
                                                   const uint64_t* __restrict__ lens, uint32_t n,
                                                   const uint64_t* __restrict__ S,
                                                   const uint32_t* __restrict__ tile_first,
                                                   const uint64_t* __restrict__ total_p, uint64_t cap_chunks,
                                                   uint32_t* __restrict__ nodes, uint8_t* __restrict__ out32,
                                                   uint64_t* __restrict__ out_keys, const uint32_t* __restrict__ perm) {
  __shared__ uint32_t cvs[TL][8];   // chunk / node chaining values, by slot
  __shared__ uint64_t sS[TL + 1];   // S[] of the tile's messages
  __shared__ uint16_t smsg[TL];     // slot -> message index in the tile (kNoMsg: past the end)
  __shared__ uint32_t task[kTaskCap<TL>];  // tree tasks by level (enc_task)
  __shared__ uint32_t ntask[12];
  __shared__ uint16_t order[ORD ? TL : 1];  // leaf loop position -> slot
  __shared__ uint32_t sexp[(XT & 2) ? TL / 32 : 1];  // XT 2: slots whose node goes to HBM (phase 4)
  __shared__ uint64_t next_tile;
  __shared__ uint32_t qbuf[QD == 3 ? 16 * (WG / 4) : 1];  // QD 3: each quad's 64-byte block buffer

  // XT bits 3-5 (ablation): that many s_nop at the entry, shifting the
  // kernel's code by 4-byte steps (code placement A/B, cdna_hip_programming.md
  // rule 27)
  if constexpr (((XT >> 3) & 7) != 0) asm volatile(".rept %c0\n s_nop 0\n .endr" ::"i"((XT >> 3) & 7));
  const uint64_t total = *total_p;
  if (total > cap_chunks) return;  // reported by sdcas_dev_sync
  const uint64_t ntiles = (total + TL - 1) / TL;
  const uint32_t tid = threadIdx.x;
  static_assert(!QD || (ORD == 0 && CA == 0 && WG % 4 == 0), "quad slots: no leaf order, no cached chunk");
  constexpr uint32_t SW = QD ? WG / 4 : WG;  // slot workers: lanes, or quads of lanes
  const uint32_t sid = QD ? tid >> 2 : tid;
  const bool lead = !QD || (tid & 3u) == 0;
  // QD 3: the LDS word indices of this lane's 28 round inputs in its quad's
  // block buffer (kQuadWord for lane q, fixed for the kernel)
  const uint32_t qslot = 16 * sid;
  uint32_t wi[QD == 3 ? 28 : 1];
  if constexpr (QD == 3) {
    const uint32_t q = tid & 3u;
    const bool q1 = q & 1u, q2 = q & 2u;
#pragma unroll
    for (int k = 0; k < 28; ++k)
      wi[k] = qslot + qsel(q1, q2, kQuadWord.w[0][k], kQuadWord.w[1][k], kQuadWord.w[2][k], kQuadWord.w[3][k]);
  }
  // DYN 1: tiles after the first are handed out by a global counter
  // (total_p[2], zeroed by k_tile_first) instead of round-robin, so a
  // workgroup that drew cheap tiles takes more and the grid drains within
  // about one tile; the next tile is claimed at the start of the current one
  // (the atomic's latency hides behind the tile) and read after its last
  // barrier. DYN 2: one tile per workgroup (the grid covers every tile the
  // workspace can hold; the hardware dispatcher is the schedule).
  unsigned long long* tile_ctr = reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(total_p) + 2);
  for (uint64_t tile = blockIdx.x; tile < ntiles;) {
    const uint64_t tbase = tile * TL;
    const uint32_t m0 = tile_first[tile];
    const uint32_t m1 = (tile + 1 < ntiles) ? tile_first[tile + 1] : n - 1;
    const uint32_t cnt = m1 - m0 + 1;  // <= TL + 1
    for (uint32_t i = tid; i < cnt; i += WG) sS[i] = S[m0 + i];
    if (tid < 12) ntask[tid] = 0;
    if constexpr ((XT & 2) != 0)
      for (uint32_t i = tid; i < TL / 32; i += WG) sexp[i] = 0;
    if (DYN == 1 && tid == 0) next_tile = gridDim.x + atomicAdd(tile_ctr, 1ull);
    __syncthreads();

    // (1) slot -> message, and the tree schedule: every aligned complete
    // power-of-two node inside the tile (level k task at its first slot), plus
    // the spine of each message lying wholly in the tile — the right-to-left
    // fold over its binary decomposition, one step per part, scheduled in the
    // level after that part's node is complete; the last step is the ROOT.
    // CA: the leaf phase takes the same two slots per lane as this loop (unless
    // the leaf order permutes them), so their chunk's address, length and
    // counter (CA 2: the first slot's only) are kept in registers from here — the message's offset is
    // loaded now, its latency hidden behind the schedule and the barrier,
    // instead of on the leaf phase's critical path
    constexpr uint32_t R = TL / SW;
    const uint8_t* c_p[R];
    uint64_t c_j[R];
    uint32_t c_clen[R], c_m[R];
    bool c_ok[R], c_root[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) c_ok[r] = false;
    constexpr uint32_t kPhase1Unroll = CA ? R : 1;
#pragma unroll kPhase1Unroll
    for (uint32_t s = sid; s < TL; s += SW) {
      const uint64_t g = tbase + s;
      uint32_t K = 0;  // levels of the tree tasks this slot starts (0: none)
      if (g >= total) {
        smsg[s] = kNoMsg;
      } else {
        uint32_t lo = 0, hi = cnt - 1;  // last message with S <= g
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (sS[mid] <= g) lo = mid;
          else hi = mid - 1;
        }
        smsg[s] = (uint16_t)lo;
        if (TR || CA) {
          const uint64_t j = g - sS[lo];
          const uint64_t len = lens[m0 + lo];
          const uint64_t C = chunk_count(len);
          if (CA && (CA == 1 || s == tid)) {
            const uint32_t r = (s - tid) / WG;
            c_ok[r] = true;
            c_m[r] = m0 + lo;
            c_j[r] = j;
            c_clen[r] = len == 0 ? 0u : (uint32_t)min<uint64_t>(CHUNK_LEN, len - j * CHUNK_LEN);
            c_root[r] = C == 1;
            c_p[r] = blob + offs[m0 + lo] + j * CHUNK_LEN;
          }
          if (TR && C != 1 && lead) {
            K = node_level_t<TL>(j, C, s);
            if constexpr ((XT & 4) == 0)
              for (uint32_t k = 1; k <= K; ++k)
                task[task_base<TL>(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s, s + (1u << (k - 1)), 0, false);
            if constexpr ((XT & 2) != 0) {
              // phase 4's test, here where the message's shape is at hand: a
              // node of a message crossing the tile whose parent is not in it
              const uint64_t S0 = g - j;
              if ((S0 < tbase || S0 + C > tbase + TL) && !parent_in_tile_t<TL>(j, C, s, K))
                atomicOr(&sexp[s >> 5], 1u << (s & 31));
            }
          }
        }
      }
      if constexpr ((XT & 4) != 0) {
        // the wave's tasks appended level by level with one LDS atomic per
        // wave and level (64 lanes adding to one counter serialise in LDS)
        for (uint32_t k = 1;; ++k) {
          const bool want = K >= k;
          const uint64_t bal = __ballot(want);
          if (!bal) break;
          const uint32_t first = (uint32_t)__ffsll((long long)bal) - 1;
          uint32_t base = 0;
          if (__lane_id() == first) base = atomicAdd(&ntask[k], (uint32_t)__popcll(bal));
          base = __shfl(base, (int)first);
          const uint32_t below =
              __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (want) task[task_base<TL>(k) + base + below] = enc_task(s, s + (1u << (k - 1)), 0, false);
        }
      }
    }
#pragma unroll 1
    for (uint32_t i = sid; TR && lead && i < cnt; i += SW) {
      const uint64_t S0 = sS[i];
      if (S0 < tbase) continue;
      const uint64_t C = chunk_count(lens[m0 + i]);
      if (C == 1 || S0 + C > tbase + TL) continue;
      const uint32_t s0 = (uint32_t)(S0 - tbase), c = (uint32_t)C;
      if (!(c & (c - 1))) {
        const uint32_t k = 31 - __clz(c);
        task[task_base<TL>(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s0, s0 + (c >> 1), i, true);
      } else {
        uint32_t rem = c, part = rem & (0u - rem);
        uint32_t pos = c - part, acc = pos;
        rem -= part;
        while (rem) {
          part = rem & (0u - rem);
          pos -= part;
          const uint32_t k = 32 - __clz(part);  // log2(part) + 1
          task[task_base<TL>(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s0 + pos, s0 + acc, i, rem == part);
          acc = pos;
          rem -= part;
        }
      }
    }

    // (2) leaves
    // Ordering pays only where a tile holds more partial chunks (one per
    // message) than a wave has lanes — fewer cannot fill a wave of their own —
    // and not in a run of single-chunk messages, which the shape sort already
    // grouped by block count. The test is uniform over the workgroup.
    // ORD 2: every other tile is put in a two-bin order — whole non-root
    // chunks first, then the rest, then past-the-end slots — so that the
    // waves over whole chunks take the full-chunk loop (PF % 100 == 6)
    const bool ord17 = ORD && cnt > 64 && chunk_count(lens[m0 + cnt - 1]) > 1;
    const bool ord = ord17 || ORD == 2;
    if constexpr (ORD != 0) if (ord) {
      uint32_t bin[TL / WG];
#pragma unroll
      for (uint32_t r = 0; r < TL / WG; ++r) {
        const uint32_t s = tid + r * WG;
        const uint32_t mi = smsg[s];
        if (ord17) {
          bin[r] = mi == kNoMsg ? 16u : leaf_bin(lens[m0 + mi], tbase + s - sS[mi]);
        } else if (mi == kNoMsg) {
          bin[r] = 2u;
        } else {
          const uint64_t len = lens[m0 + mi], j = tbase + s - sS[mi];
          bin[r] = (len - j * CHUNK_LEN >= CHUNK_LEN && len > CHUNK_LEN) ? 0u : 1u;
        }
      }
      // the per (bin, 64-slot group) counts borrow cvs, which no one reads
      // between the previous tile's last barrier and this tile's leaves
      if (ord17) leaf_order<WG, 17, TL>(tid, bin, order, reinterpret_cast<uint16_t*>(&cvs[0][0]));
      else leaf_order<WG, 3, TL>(tid, bin, order, reinterpret_cast<uint16_t*>(&cvs[0][0]));
    }
    if (CA && !ord) {
#pragma unroll
      for (uint32_t r = 0; r < (CA == 1 ? R : 1); ++r) {
        if (!c_ok[r]) continue;
        uint32_t cv[8];
        leaf_hash<PF>(leaf_ptr<PF>(blob, c_p[r]), c_clen[r], c_j[r], c_root[r], cv);
        if (c_root[r]) {
          store_digest(perm ? perm[c_m[r]] : c_m[r], cv, out32, out_keys);
        } else {
          const uint32_t s = tid + r * WG;
#pragma unroll
          for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
        }
      }
    }
    // (CA 2 keeps the first slot only: the second one's state would live in
    // registers across the first one's block loop, where they spill)
#pragma unroll 1
    for (uint32_t i = (CA == 2 && !ord) ? tid + WG : sid; (CA != 1 || ord) && i < TL; i += SW) {
      const uint32_t s = ord ? order[i] : i;
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint32_t m = m0 + mi;
      const uint64_t j = tbase + s - sS[mi];
      const uint64_t len = lens[m];
      const uint64_t C = chunk_count(len);
      const uint32_t clen = len == 0 ? 0u : (uint32_t)min<uint64_t>(CHUNK_LEN, len - j * CHUNK_LEN);
      const bool root = (C == 1);
      uint32_t cv[8];
      if constexpr (QD == 3) hash_chunk_quad_lds(blob + offs[m] + j * CHUNK_LEN, clen, j, root, qbuf, qslot, wi, cv);
      else if constexpr (QD == 2) hash_chunk_quad4(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if constexpr (QD) hash_chunk_quad(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else leaf_hash<PF>(leaf_ptr<PF>(blob, blob + offs[m] + j * CHUNK_LEN), clen, j, root, cv);
      if (!lead) continue;
      if (root) {
        store_digest(perm ? perm[m] : m, cv, out32, out_keys);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
      }
    }
    __syncthreads();
    // the next tile, read between two barriers: thread 0 overwrites next_tile
    // only after this tile's last barrier, which every thread has passed the
    // read by then
    const uint64_t nt = DYN == 2 ? ntiles : (DYN ? next_tile : tile + gridDim.x);

    // (3) the tree, level by level: every task of a level is independent
    // (TR 3: DIAGNOSTIC, wrong digests — levels 5-10 skipped, what they cost)
    for (uint32_t k = 1; TR && (1u << k) <= TL && k <= (TR == 3 ? 4u : 10u); ++k) {
      const uint32_t T = ntask[k];
      if (T == 0) continue;
      if constexpr ((XT & 1) != 0 && !QD) {
        if (T <= 32) {
          // a few tasks: one quad of lanes per task (all four lanes of a
          // task's quad run it together, as parent_quad's DPP needs)
#pragma unroll 1
          for (uint32_t t = tid >> 2; t < T; t += WG / 4) {
            const uint32_t e = task[task_base<TL>(k) + t];
            const uint32_t l = e & 1023u, r = (e >> 10) & 1023u;
            const bool root = e >> 31;
            uint32_t a[8], b[8], o[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              a[q] = cvs[l][q];
              b[q] = cvs[r][q];
            }
            parent_quad(a, b, root, o);
            if (tid & 3u) continue;
            if (root) {
              const uint32_t mm = m0 + ((e >> 20) & 2047u);
              store_digest(perm ? perm[mm] : mm, o, out32, out_keys);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) cvs[l][q] = o[q];
            }
          }
          __syncthreads();
          continue;
        }
      }
      // TR 2 (diagnostic, still bit-exact): every lane of a wave that holds
      // tasks computes one — lanes past the level's last task repeat it and
      // do not store — to price masked lanes against active ones
      const uint32_t TT = TR == 2 ? (T + 63u) & ~63u : T;
#pragma unroll 1
      for (uint32_t t = sid; t < TT; t += SW) {
        const uint32_t e = task[task_base<TL>(k) + (TR == 2 ? min(t, T - 1) : t)];
        const uint32_t l = e & 1023u, r = (e >> 10) & 1023u;
        const bool root = e >> 31;
        uint32_t o[8];
        if constexpr (QD == 3) {
          // lane q's quarter of the parent block: words 4q..4q+3 of l's CV
          // (q < 2) or of r's (q >= 2), staged as a leaf block is
          const uint32_t q = tid & 3u;
          const uint32_t* src = q < 2 ? &cvs[l][4 * q] : &cvs[r][4 * (q - 2)];
          uint32_t w[28], iv[8];
          quad_lds_words(qbuf, qslot, make_uint4(src[0], src[1], src[2], src[3]), wi, w);
          set_iv(iv);
          compress_quad_w(iv, w, 0, BLOCK_LEN, PARENT | (root ? ROOT : 0u), o);
        } else {
          uint32_t a[8], b[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            a[q] = cvs[l][q];
            b[q] = cvs[r][q];
          }
          if constexpr (QD) parent_quad(a, b, root, o);
          else parent<kGA<PF>>(a, b, root, o);
        }
        if ((TR == 2 && t >= T) || !lead) continue;
        if (root) {
          const uint32_t mm = m0 + ((e >> 20) & 2047u);
          store_digest(perm ? perm[mm] : mm, o, out32, out_keys);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) cvs[l][q] = o[q];
        }
      }
      __syncthreads();
    }

    // (4) messages crossing a tile boundary: their maximal in-tile nodes go to
    // HBM at their first slot, for k_finish
#pragma unroll 1
    for (uint32_t s = sid; TR && lead && s < TL; s += SW) {
      if constexpr ((XT & 2) != 0) {
        if (!((sexp[s >> 5] >> (s & 31)) & 1u)) continue;
        uint4* o = reinterpret_cast<uint4*>(nodes + 8ull * (tbase + s));
        o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
        o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
        continue;
      }
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t S0 = sS[mi];
      const uint64_t C = chunk_count(lens[m0 + mi]);
      if (C == 1 || (S0 >= tbase && S0 + C <= tbase + TL)) continue;  // single chunk / spine done in (3)
      const uint64_t j = tbase + s - S0;
      const uint32_t k = node_level_t<TL>(j, C, s);
      if (parent_in_tile_t<TL>(j, C, s, k)) continue;
      uint4* o = reinterpret_cast<uint4*>(nodes + 8ull * (tbase + s));
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
    __syncthreads();
    tile = nt;
  }
}


// Messages crossing tile boundaries: one lane per tile boundary t (the
// message holding slot t*kTile, when it started in tile t-1 — its first
// crossing), so the launch is dense (~ one active lane per tile) instead of a
// lane per message. The lane walks the message's maximal nodes left to right
// (a closed-form function of (chunk index, chunk count, slot in tile)) and
// merges them with the BLAKE3 subtree-stack rule; the last merge is ROOT.
// The subtree-stack merge of one message's maximal nodes (left to right),
// the last merge ROOT. `at(d)` is the d-th stack entry (8 words).
template <uint32_t TILE, class At>
__device__ __forceinline__ void merge_nodes(const uint32_t* __restrict__ nodes, uint64_t s0, uint64_t C, At at,
                                            uint32_t (&cv)[8]) {
  int depth = 0;
  uint64_t j = 0;
  while (j < C) {
    const uint64_t g = s0 + j;
    const uint32_t k = node_level_t<TILE>(j, C, (uint32_t)(g % TILE));
    const uint4* p = reinterpret_cast<const uint4*>(nodes + 8ull * g);
    uint4 a = p[0], b = p[1];
    uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    // subtrees completed by the first j chunks are merged before going on
    const int keep = __popcll(j);
    while (depth > keep) {
      uint32_t l[8], r[8], o[8];
      uint32_t *pl = at(depth - 2), *pr = at(depth - 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        l[i] = pl[i];
        r[i] = pr[i];
      }
      parent(l, r, false, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) pl[i] = o[i];
      --depth;
    }
    j += 1ull << k;
    if (j == C) {
      for (int d = depth - 1; d >= 0; --d) {
        uint32_t l[8], o[8];
        const uint32_t* pl = at(d);
#pragma unroll
        for (int i = 0; i < 8; ++i) l[i] = pl[i];
        parent(l, v, d == 0, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = o[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) cv[i] = v[i];
      return;
    }
    uint32_t* pp = at(depth);
#pragma unroll
    for (int i = 0; i < 8; ++i) pp[i] = v[i];
    ++depth;
  }
}

// merge_nodes without divergence between lanes: every lane runs the same
// bookkeeping (loads and pushes, no compression) up to its next compression,
// then the wave issues ONE parent compression for all lanes that need one —
// the merge of the stack's top two nodes or a fold of the final node into
// the stack. merge_nodes' nested loops, run by 64 lanes whose node lists
// differ, execute the union of their compression sequences instead.
// QUAD: the four lanes of a quad run the same message's merges (identical
// bookkeeping) and each parent compression together (compress_quad)
template <uint32_t TILE, bool QUAD = false, class At>
__device__ __forceinline__ void merge_nodes_flat(const uint32_t* __restrict__ nodes, uint64_t s0, uint64_t C, At at,
                                                 uint32_t (&cv)[8]) {
  int depth = 0, keep = 0;
  uint64_t j = 0;
  uint32_t k = 0;
  bool have = false, done = false;
  uint32_t v[8];
  for (;;) {
    int op = 0;  // 1: merge the stack's top two; 2: fold the final node into the top
    while (!done) {
      if (!have) {
        const uint64_t g = s0 + j;
        k = node_level_t<TILE>(j, C, (uint32_t)(g % TILE));
        const uint4* p = reinterpret_cast<const uint4*>(nodes + 8ull * g);
        const uint4 a = p[0], b = p[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        keep = __popcll(j);  // subtrees completed by the first j chunks merge first
        have = true;
      }
      if (depth > keep) {
        op = 1;
        break;
      }
      if (j + (1ull << k) < C) {
        uint32_t* pp = at(depth);
#pragma unroll
        for (int i = 0; i < 8; ++i) pp[i] = v[i];
        ++depth;
        j += 1ull << k;
        have = false;
        continue;
      }
      if (depth == 0) {  // the final node has absorbed the whole stack: it is the root's output
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = v[i];
        done = true;
        break;
      }
      op = 2;
      break;
    }
    if (__builtin_amdgcn_ballot_w64(op != 0) == 0) return;
    if (op) {
      uint32_t l[8], r[8], o[8];
      const uint32_t* pl = at(op == 1 ? depth - 2 : depth - 1);
      const uint32_t* pr = at(depth - 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        l[i] = pl[i];
        r[i] = op == 1 ? pr[i] : v[i];
      }
      if constexpr (QUAD) parent_quad(l, r, op == 2 && depth == 1, o);
      else parent(l, r, op == 2 && depth == 1, o);
      if (op == 1) {
        uint32_t* po = at(depth - 2);
#pragma unroll
        for (int i = 0; i < 8; ++i) po[i] = o[i];
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = o[i];
      }
      --depth;
    }
  }
}

// rare: a message of 2^22+ chunks (4 GiB+) needs a deeper stack than LDS holds
template <uint32_t TILE>
__device__ __noinline__ void merge_nodes_deep(const uint32_t* __restrict__ nodes, uint64_t s0, uint64_t C,
                                              uint32_t (&cv)[8]) {
  uint32_t stack[kMaxStack][8];
  merge_nodes<TILE>(nodes, s0, C, [&](int d) { return &stack[d][0]; }, cv);
}

// Messages crossing tile boundaries: one lane per tile boundary t (the
// message holding slot t*TILE, when it started in tile t-1 — its first
// crossing); the merge stack lives in LDS (a private array would live in
// scratch memory, a round trip to HBM per merge).
constexpr int kFinishWG = 64, kFinishDepth = 24;
template <uint32_t TILE>
__global__ void __launch_bounds__(kFinishWG) k_finish_t(const uint64_t* __restrict__ lens, uint32_t n,
                                                       const uint64_t* __restrict__ S,
                                                       const uint32_t* __restrict__ tile_first,
                                                       const uint64_t* __restrict__ total_p, uint64_t cap_slots,
                                                       const uint32_t* __restrict__ nodes,
                                                       const uint32_t* __restrict__ perm, uint8_t* __restrict__ out32,
                                                       uint64_t* __restrict__ out_keys) {
  // one lane's stack per row, rows an odd number of words apart: lane l's
  // word w sits in bank (l * kFinishRow + w) mod 64, so a wave's stack
  // accesses are conflict-free (a 192-word row put all 64 lanes in one bank)
  constexpr uint32_t kFinishRow = kFinishDepth * 8 + 1;
  __shared__ uint32_t lstack[kFinishWG][kFinishRow];
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = *total_p;
  if (total > cap_slots || t == 0 || t * TILE >= total) return;
  const uint32_t m = tile_first[t];
  const uint64_t s0 = S[m];
  if (s0 >= t * TILE || s0 / TILE != t - 1) return;  // starts on the boundary / crossed an earlier one first
  const uint64_t C = chunk_count(lens[m]);
  if (s0 + C <= t * TILE) return;  // (quad layout) only its padding reaches the boundary
  uint32_t cv[8];
  // stack depth <= popcount(j) + 1 <= log2(C) + 1
  if (C < (1ull << (kFinishDepth - 2)))
    merge_nodes_flat<TILE>(nodes, s0, C, [&](int d) { return &lstack[threadIdx.x][8 * d]; }, cv);
  else
    merge_nodes_deep<TILE>(nodes, s0, C, cv);
  store_digest(perm ? perm[m] : m, cv, out32, out_keys);
}

// The same with a quad per tile boundary: the boundary's merges run on four
// lanes (merge_nodes_flat<QUAD>), each parent compression a quad's chain of
// ~180 dependent instructions instead of one lane's 680, and four times the
// lanes in flight. C2's 50 K boundaries: 0.07 ms as k_finish_t.
constexpr int kFinishQWG = 64, kFinishQPerWG = kFinishQWG / 4;
template <uint32_t TILE>
__global__ void __launch_bounds__(kFinishQWG) k_finish_q(const uint64_t* __restrict__ lens, uint32_t n,
                                                        const uint64_t* __restrict__ S,
                                                        const uint32_t* __restrict__ tile_first,
                                                        const uint64_t* __restrict__ total_p, uint64_t cap_slots,
                                                        const uint32_t* __restrict__ nodes,
                                                        const uint32_t* __restrict__ perm, uint8_t* __restrict__ out32,
                                                        uint64_t* __restrict__ out_keys) {
  constexpr uint32_t kFinishRow = kFinishDepth * 8 + 1;
  __shared__ uint32_t lstack[kFinishQPerWG][kFinishRow];
  const uint32_t b = threadIdx.x >> 2;  // the quad's boundary in the workgroup
  const uint64_t t = (uint64_t)blockIdx.x * kFinishQPerWG + b;
  const uint64_t total = *total_p;
  // every test below depends on t only: a quad's lanes leave together
  if (total > cap_slots || t == 0 || t * TILE >= total) return;
  const uint32_t m = tile_first[t];
  const uint64_t s0 = S[m];
  if (s0 >= t * TILE || s0 / TILE != t - 1) return;
  const uint64_t C = chunk_count(lens[m]);
  if (s0 + C <= t * TILE) return;
  uint32_t cv[8];
  if (C < (1ull << (kFinishDepth - 2)))
    merge_nodes_flat<TILE, true>(nodes, s0, C, [&](int d) { return &lstack[b][8 * d]; }, cv);
  else
    merge_nodes_deep<TILE>(nodes, s0, C, cv);
  if ((threadIdx.x & 3) == 0) store_digest(perm ? perm[m] : m, cv, out32, out_keys);
}

// SDCAS_FINISH=lane: k_finish_t (a lane per boundary) instead of k_finish_q (A/B)
static bool finish_by_quad() {
  const char* v = getenv("SDCAS_FINISH");
  return !(v && strcmp(v, "lane") == 0);
}

template <uint32_t TILE>
static void launch_finish(uint64_t tiles, hipStream_t st, const uint64_t* lens, uint32_t n, const uint64_t* S,
                          const uint32_t* tile_first, const uint64_t* total, uint64_t cap_slots, const uint32_t* nodes,
                          const uint32_t* perm, uint8_t* out32, uint64_t* out_keys) {
  if (finish_by_quad())
    hipLaunchKernelGGL(k_finish_q<TILE>, dim3((uint32_t)((tiles + kFinishQPerWG - 1) / kFinishQPerWG)),
                       dim3(kFinishQWG), 0, st, lens, n, S, tile_first, total, cap_slots, nodes, perm, out32,
                       out_keys);
  else
    hipLaunchKernelGGL(k_finish_t<TILE>, dim3((uint32_t)((tiles + kFinishWG - 1) / kFinishWG)), dim3(kFinishWG), 0,
                       st, lens, n, S, tile_first, total, cap_slots, nodes, perm, out32, out_keys);
}

#ifdef SDCAS_ABLATIONS
#include "b3_ablate_kernels.inc"
#endif

// Slot order by message shape: key = min(chunks, 15) << 4 | (blocks in the
// last chunk - 1). Single-chunk messages — whose lanes otherwise run 1..16
// blocks side by side in one wave — end up grouped by block count;
// multi-chunk messages have one short chunk each and are merely clustered.
// A counting sort over the 256 shape bins in three launches and no global
// atomics: (1) each workgroup's histogram of its 4096 messages, stored
// bin-major (wcnt[bin][wg]); (2) one workgroup per bin: the bin's total and
// each workgroup's start inside the bin; (3) the scatter: each workgroup
// scans the bin totals, orders its messages by shape in LDS and writes them
// run by run. Round 3's version reserved each workgroup's range per bin with
// a global atomicAdd on one counter per bin — on C5, ~300 K atomics on ~200
// addresses, serialised at their L2 channels (hist 20 us + scatter 104 us).
// Order inside a bin: by workgroup, then unspecified — it changes nothing
// but the slot a message lands in.
constexpr uint32_t kShapeBins = 256;
constexpr uint32_t kScatterPerWG = 4096;
constexpr uint32_t kScatterR = kScatterPerWG / 256;  // messages per scatter thread
constexpr uint32_t kShapeManyChunks = 15 << 4;  // first shape key of messages of 15+ chunks
static_assert(kSortTotalsWords == kShapeBins && kSortPerWG == kScatterPerWG, "ws.sort_keys layout");

__device__ __forceinline__ uint32_t shape_key(uint64_t L) {
  const uint64_t C = chunk_count(L);
  const uint64_t last = L - (C - 1) * CHUNK_LEN;  // 0..1024
  const uint32_t blocks = last == 0 ? 1u : (uint32_t)((last + BLOCK_LEN - 1) / BLOCK_LEN);
  return ((uint32_t)min<uint64_t>(C, 15) << 4) | (blocks - 1);
}

// (1) wcnt[bin * nwg + wg] = messages of workgroup wg's 4096 in bin
__global__ void __launch_bounds__(256) k_shape_hist(const uint64_t* __restrict__ lens, uint32_t n,
                                                    uint32_t* __restrict__ wcnt) {
  __shared__ uint32_t h[kShapeBins];
  const uint32_t t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const uint64_t lo = (uint64_t)blockIdx.x * kScatterPerWG;
  uint64_t L[kScatterR];
#pragma unroll
  for (uint32_t r = 0; r < kScatterR; ++r) {
    const uint64_t i = lo + r * 256 + t;
    L[r] = i < n ? lens[i] : 0;
  }
#pragma unroll
  for (uint32_t r = 0; r < kScatterR; ++r)
    if (lo + r * 256 + t < n) atomicAdd(&h[shape_key(L[r])], 1u);
  __syncthreads();
  wcnt[(uint64_t)t * gridDim.x + blockIdx.x] = h[t];
}

// (2) one workgroup per bin: totals[bin], and wcnt[bin][wg] <- the exclusive
// prefix over the workgroups (the workgroup's first position inside the bin)
__global__ void __launch_bounds__(256) k_shape_bins(uint32_t* __restrict__ wcnt, uint32_t nwg,
                                                    uint32_t* __restrict__ totals) {
  __shared__ uint32_t ws[4];
  __shared__ uint32_t carry;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t* col = wcnt + (uint64_t)blockIdx.x * nwg;
  if (t == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nwg; base += 256) {
    const uint32_t i = base + t;
    const uint32_t v = i < nwg ? col[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= d) inc += x;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += ws[w];
    if (i < nwg) col[i] = before + inc - v;
    __syncthreads();
    if (t == 255) carry = before + inc;
    __syncthreads();
  }
  if (t == 0) totals[blockIdx.x] = carry;
}

// (3) Scatter in two steps so that the global writes are coalesced: the
// workgroup's 4096 messages are first ordered by shape in LDS (2-byte local
// indices), then written run by run — consecutive threads to consecutive
// addresses of a bin's range. The second read of offs/lens (in LDS order) hits
// the L2 lines the first read brought in. Each thread's kScatterR global
// loads of a pass are issued together, ahead of their use.
__global__ void __launch_bounds__(256) k_shape_scatter(const uint64_t* __restrict__ offs,
                                                       const uint64_t* __restrict__ lens, uint32_t n,
                                                       const uint32_t* __restrict__ totals,
                                                       const uint32_t* __restrict__ wstart,
                                                       uint32_t* __restrict__ perm, uint64_t* __restrict__ soffs,
                                                       uint64_t* __restrict__ slens) {
  __shared__ uint32_t gstart[kShapeBins], lstart[kShapeBins], h[kShapeBins];
  __shared__ uint16_t order[kScatterPerWG];
  __shared__ uint8_t keyof[kScatterPerWG];
  __shared__ uint32_t few_chunks;
  const uint32_t t = threadIdx.x;
  // exclusive scan of the bin totals (256 entries, one per thread)
  const uint32_t bin_count = totals[t];
  gstart[t] = bin_count;
  h[t] = 0;
  __syncthreads();
  for (uint32_t d = 1; d < kShapeBins; d <<= 1) {
    const uint32_t v = t >= d ? gstart[t - d] : 0u;
    __syncthreads();
    gstart[t] += v;
    __syncthreads();
  }
  if (t == kShapeManyChunks - 1) few_chunks = gstart[t];  // messages of < 15 chunks
  const uint32_t excl = gstart[t] - bin_count;
  __syncthreads();
  gstart[t] = excl;
  const uint32_t lo = blockIdx.x * kScatterPerWG, hi = min(n, lo + kScatterPerWG), m = hi - lo;
  // When most messages span 15+ chunks (C2's 1-100 KiB files: 86 %), their
  // chunks are full whatever the order and sorting gains nothing (measured:
  // C2 leaf 15.34 ms unsorted vs 15.38 sorted, C3 / C5 2-3 % faster sorted):
  // keep the caller's order, as a coalesced copy. Every workgroup decides the
  // same from the same totals.
  if ((uint64_t)(n - few_chunks) * 10 > (uint64_t)n * 6) {
    uint64_t o[kScatterR], l[kScatterR];
#pragma unroll
    for (uint32_t r = 0; r < kScatterR; ++r) {
      const uint32_t k = t + r * 256;
      o[r] = k < m ? offs[lo + k] : 0;
      l[r] = k < m ? lens[lo + k] : 0;
    }
#pragma unroll
    for (uint32_t r = 0; r < kScatterR; ++r) {
      const uint32_t k = t + r * 256;
      if (k >= m) continue;
      perm[lo + k] = lo + k;
      soffs[lo + k] = o[r];
      slens[lo + k] = l[r];
    }
    return;
  }
  {
    uint64_t l[kScatterR];
#pragma unroll
    for (uint32_t r = 0; r < kScatterR; ++r) {
      const uint32_t k = t + r * 256;
      l[r] = k < m ? lens[lo + k] : 0;
    }
#pragma unroll
    for (uint32_t r = 0; r < kScatterR; ++r) {
      const uint32_t k = t + r * 256;
      if (k >= m) continue;
      const uint32_t key = shape_key(l[r]);
      keyof[k] = (uint8_t)key;
      atomicAdd(&h[key], 1u);
    }
  }
  __syncthreads();
  // this workgroup's range in bin t (from k_shape_bins), and the bin's start
  // in the local order
  const uint32_t cnt = h[t];
  gstart[t] += wstart[(uint64_t)t * gridDim.x + blockIdx.x];
  lstart[t] = cnt;
  __syncthreads();
  for (uint32_t d = 1; d < kShapeBins; d <<= 1) {
    const uint32_t v = t >= d ? lstart[t - d] : 0u;
    __syncthreads();
    lstart[t] += v;
    __syncthreads();
  }
  lstart[t] -= cnt;  // exclusive
  h[t] = 0;          // becomes the per-bin fill cursor
  __syncthreads();
  for (uint32_t k = t; k < m; k += 256) {
    const uint32_t key = keyof[k];
    order[lstart[key] + atomicAdd(&h[key], 1u)] = (uint16_t)k;
  }
  __syncthreads();
  uint32_t kk[kScatterR];
  uint64_t o[kScatterR], l[kScatterR];
#pragma unroll
  for (uint32_t r = 0; r < kScatterR; ++r) {
    const uint32_t p = t + r * 256;
    kk[r] = p < m ? order[p] : 0u;
    o[r] = p < m ? offs[lo + kk[r]] : 0;
    l[r] = p < m ? lens[lo + kk[r]] : 0;
  }
#pragma unroll
  for (uint32_t r = 0; r < kScatterR; ++r) {
    const uint32_t p = t + r * 256;
    if (p >= m) continue;
    const uint32_t key = keyof[kk[r]];
    const uint32_t pos = gstart[key] + (p - lstart[key]);
    perm[pos] = lo + kk[r];
    soffs[pos] = o[r];
    slens[pos] = l[r];
  }
}


// ---- big files: 1 MiB pieces -----------------------------------------------
//
// A file of C > kTile chunks is cut at 1 MiB boundaries of the FILE into
// pieces; piece q holds chunks [1024q, 1024q + 1024) and the last piece the
// r = C mod 1024 remaining chunks (if any). One workgroup hashes one piece:
// its 1024 chunks fill exactly one tile, so a full piece reduces to its
// level-10 subtree CV (a node of the file's tree, never the root since
// C > 1024), and a tail piece to the binary decomposition of r (one node per
// 1-bit of r). These nodes go to a per-file node list: full piece q at index
// q, tail nodes after the Q full pieces in decreasing size. Pieces of one file
// may arrive over many launches (streamed windows); k_bigfile_finish merges a
// file's list once all of it is there.

// One workgroup's pass over its pieces (the body of k_piece_tree and
// k_piece_l4). DEFER: a full piece stops at tree level 4 and writes its 64
// level-4 nodes to l4[64 pi ..] for k_piece_top, which runs the one-wave
// levels 5-10 of eight pieces at once; a tail piece completes here.
template <int PF, int DIRECT, int ROT, int TOP, int DEFER>
__device__ __forceinline__ void piece_pass(const uint8_t* __restrict__ blob, const PieceDesc* __restrict__ pieces,
                                           uint32_t npieces, uint32_t* __restrict__ file_nodes,
                                           uint32_t* __restrict__ l4) {
  __shared__ uint32_t cvs[kTile][8];
  __shared__ uint16_t task[kTile / 2];
  __shared__ uint32_t ntask[16];
  const uint32_t tid = threadIdx.x;
  for (uint32_t pi = blockIdx.x; pi < npieces; pi += gridDim.x) {
    const PieceDesc pd = pieces[pi];
    const uint32_t nchunks = (pd.len + CHUNK_LEN - 1) / CHUNK_LEN;
    if (tid < 16) ntask[tid] = 0;
    // ROT: co-resident workgroups start at different 64-chunk offsets of
    // their pieces, so the chip's concurrent reads do not all sit at the
    // same offset of 1 MiB-aligned pieces
    const uint32_t rot = ROT ? (uint32_t)((pi * 7u * 64u) % nchunks) & ~63u : 0u;
#pragma unroll 1
    for (uint32_t s0 = tid; s0 < nchunks; s0 += kWG) {
      uint32_t s = s0 + rot;
      if (ROT && s >= nchunks) s -= nchunks;
      const uint32_t clen = min(CHUNK_LEN, pd.len - s * CHUNK_LEN);
      uint32_t cv[8];
      leaf_hash<PF>(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv);
#pragma unroll
      for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
    }
    __syncthreads();
    const bool defer = DEFER && nchunks == kTile;
    const uint32_t top = defer ? kPieceDeferLevel : TOP;
    for (uint32_t k = 1; (1u << k) <= kTile && k <= top; ++k) {  // TOP < 10: DIAGNOSTIC (wrong digests)
      const uint32_t w = 1u << k;
      uint32_t T;
      if (DIRECT) {
        // the complete aligned level-k nodes of a piece are its first
        // nchunks >> k multiples of 2^k: task t is node t, no list needed
        T = nchunks >> k;
        if (T == 0) break;
      } else {
        for (uint32_t s = tid; s < nchunks; s += kWG)
          if (!(s & (w - 1)) && s + w <= nchunks) task[atomicAdd(&ntask[k], 1u)] = (uint16_t)s;
        __syncthreads();
        T = ntask[k];
        if (T == 0) break;
      }
#pragma unroll 1
      for (uint32_t t = tid; t < T; t += kWG) {
        const uint32_t s = DIRECT ? t << k : task[t];
        uint32_t l[8], r[8], o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          l[i] = cvs[s][i];
          r[i] = cvs[s + (w >> 1)][i];
        }
        parent<kGA<PF>>(l, r, false, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = o[i];
      }
      __syncthreads();
    }
    if (defer) {
      for (uint32_t t = tid; t < kTile >> kPieceDeferLevel; t += kWG) {
        const uint32_t s = t << kPieceDeferLevel;
        uint4* o = reinterpret_cast<uint4*>(l4 + 8ull * ((uint64_t)pi * (kTile >> kPieceDeferLevel) + t));
        o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
        o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
      }
      __syncthreads();
      continue;
    }
    // maximal nodes: the binary decomposition of nchunks (one node for a full piece)
    for (uint32_t s = tid; s < nchunks; s += kWG) {
      const uint32_t rest = nchunks - s;
      // s starts a maximal node iff s is the sum of the higher bits of nchunks
      const uint32_t k = 31 - __clz(rest);  // node size = highest power of two <= rest
      if ((s & ((1u << k) - 1)) || (s != (nchunks & ~((2u << k) - 1)))) continue;
      const uint64_t idx = pd.node_base + (nchunks == kTile ? pd.j0 / kTile : pd.j0 / kTile + __popc(nchunks >> (k + 1)));
      uint4* o = reinterpret_cast<uint4*>(file_nodes + 8ull * idx);
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
    __syncthreads();
  }
}

template <int PF, int MINW, int DIRECT = 0, int ROT = 0, int TOP = 10>
__global__ void __launch_bounds__(kWG, MINW) k_piece_tree(const uint8_t* __restrict__ blob,
                                                          const PieceDesc* __restrict__ pieces, uint32_t npieces,
                                                          uint32_t* __restrict__ file_nodes) {
  piece_pass<PF, DIRECT, ROT, TOP, 0>(blob, pieces, npieces, file_nodes, nullptr);
}

// k_piece_tree whose full pieces stop at level 4 (piece_pass DEFER)
template <int PF, int MINW>
__global__ void __launch_bounds__(kWG, MINW) k_piece_l4(const uint8_t* __restrict__ blob,
                                                        const PieceDesc* __restrict__ pieces, uint32_t npieces,
                                                        uint32_t* __restrict__ file_nodes, uint32_t* __restrict__ l4) {
  piece_pass<PF, 1, 0, 10, 1>(blob, pieces, npieces, file_nodes, l4);
}

// Levels 5-10 of kTopPieces full pieces per workgroup, one thread per level-4
// node: the levels' tasks (256, 128, 64, 32, 16, 8) fill 10 wave-issues for
// the 504 parents of 8 pieces, where one piece per workgroup spends 6 nearly
// empty wave-issues on its 63. A piece's 64 nodes are 64-aligned in the
// group's array, so the in-place levels never cross pieces. Pieces of fewer
// than kTile chunks have no l4 entries and no result here.
constexpr uint32_t kTopPieces = kWG / (kTile >> kPieceDeferLevel);
static_assert(kTopPieces * (kTile >> kPieceDeferLevel) == kWG, "k_piece_top: one thread per level-4 node");
static_assert(kPieceDeferLevel < 10 && (kTile >> kPieceDeferLevel) <= kWG, "a piece's level-4 nodes fit one workgroup");
template <int PF>
__global__ void __launch_bounds__(kWG) k_piece_top(const PieceDesc* __restrict__ pieces, uint32_t npieces,
                                                   const uint32_t* __restrict__ l4, uint32_t* __restrict__ file_nodes) {
  constexpr uint32_t kN = kTile >> kPieceDeferLevel;  // level-4 nodes per piece
  __shared__ uint32_t cvs[kTopPieces * kN][8];
  const uint32_t tid = threadIdx.x;
  const uint32_t p0 = blockIdx.x * kTopPieces;
  if (p0 + tid / kN < npieces) {
    const uint4* src = reinterpret_cast<const uint4*>(l4 + 8ull * ((uint64_t)p0 * kN + tid));
    const uint4 a = src[0], b = src[1];
    cvs[tid][0] = a.x; cvs[tid][1] = a.y; cvs[tid][2] = a.z; cvs[tid][3] = a.w;
    cvs[tid][4] = b.x; cvs[tid][5] = b.y; cvs[tid][6] = b.z; cvs[tid][7] = b.w;
  }
  __syncthreads();
#pragma unroll 1
  for (uint32_t k = 1; (1u << k) <= kN; ++k) {
    if (tid < (kTopPieces * kN) >> k) {
      const uint32_t s = tid << k, h = 1u << (k - 1);
      uint32_t l[8], r[8], o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        l[i] = cvs[s][i];
        r[i] = cvs[s + h][i];
      }
      parent<kGA<PF>>(l, r, false, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) cvs[s][i] = o[i];
    }
    __syncthreads();
  }
  if (tid < kTopPieces && p0 + tid < npieces) {
    const PieceDesc pd = pieces[p0 + tid];
    if ((pd.len + CHUNK_LEN - 1) / CHUNK_LEN == kTile) {  // piece_pass deferred it (a file's last piece too)
      const uint32_t s = tid * kN;
      uint4* o = reinterpret_cast<uint4*>(file_nodes + 8ull * (pd.node_base + pd.j0 / kTile));
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
  }
}

// hash_chunk_ps whose first line (blocks 0 and min(1, nb-1)) the caller has
// already loaded into m0 / m1
__device__ __forceinline__ void hash_chunk_ps_loaded(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j,
                                                     uint32_t (&cv)[8], uint32_t (&m0)[16], uint32_t (&m1)[16]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
#pragma unroll 1
  for (uint32_t b = 0;; b += 2) {
    {
      const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m0, blen);
      compress(cv, m0, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? CHUNK_END : 0u));
    }
    if (b + 1 < nb) {
      const uint32_t blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m1, blen);
      compress(cv, m1, j, blen, b + 2 == nb ? CHUNK_END : 0u);
    }
    if (b + 2 >= nb) break;
    load_full_block(p + (b + 2) * BLOCK_LEN, m0);
    load_full_block(p + min(b + 3, nb - 1) * BLOCK_LEN, m1);
  }
}

// k_piece_tree on the leaf kernel's schedule: a persistent grid whose
// workgroups claim pieces from a global counter (`ctr`, zeroed before the
// launch; the next piece is claimed at the start of the current one, so the
// atomic's latency hides behind it), and — PRE — each lane loads the first
// line of its first chunk of the NEXT piece before the current piece's tree
// levels, whose few active waves would otherwise leave the CU's load path
// idle while the next piece starts cold. Full pieces only reduce to their
// level-10 node; tail pieces to the binary decomposition of their chunks, as
// in k_piece_tree.
template <int MINW, int PRE>
__global__ void __launch_bounds__(kWG, MINW) k_piece_dyn(const uint8_t* __restrict__ blob,
                                                         const PieceDesc* __restrict__ pieces, uint32_t npieces,
                                                         uint32_t* __restrict__ file_nodes,
                                                         uint32_t* __restrict__ ctr) {
  __shared__ uint32_t cvs[kTile][8];
  __shared__ uint32_t next_piece;
  const uint32_t tid = threadIdx.x;
  uint32_t pm0[16], pm1[16];
  bool have = false;  // PRE: pm0 / pm1 hold chunk `tid` of piece pi
#pragma unroll 1
  for (uint32_t pi = blockIdx.x; pi < npieces;) {
    if (tid == 0) next_piece = gridDim.x + atomicAdd(ctr, 1u);
    const PieceDesc pd = pieces[pi];
    const uint32_t nchunks = (pd.len + CHUNK_LEN - 1) / CHUNK_LEN;
#pragma unroll 1
    for (uint32_t s = tid; s < nchunks; s += kWG) {
      const uint32_t clen = min(CHUNK_LEN, pd.len - s * CHUNK_LEN);
      const uint8_t* p = blob + pd.off + (uint64_t)s * CHUNK_LEN;
      uint32_t cv[8];
      if (PRE && have && s == tid) {
        hash_chunk_ps_loaded(p, clen, pd.j0 + s, cv, pm0, pm1);
      } else {
        hash_chunk_ps(p, clen, pd.j0 + s, false, cv);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
    }
    __syncthreads();
    // read between two barriers: thread 0 rewrites it after this piece's last one
    const uint32_t nx = next_piece;
    if (PRE) {
      have = false;
      if (nx < npieces) {
        const PieceDesc nd = pieces[nx];
        if (tid * CHUNK_LEN < nd.len) {
          const uint32_t clen = min(CHUNK_LEN, nd.len - tid * CHUNK_LEN);
          const uint32_t nb = (clen + BLOCK_LEN - 1) / BLOCK_LEN;
          const uint8_t* p = blob + nd.off + (uint64_t)tid * CHUNK_LEN;
          load_full_block(p, pm0);
          load_full_block(p + min(1u, nb - 1) * BLOCK_LEN, pm1);
          have = true;
        }
      }
    }
    // the complete aligned level-k nodes of a piece are its first
    // nchunks >> k multiples of 2^k
#pragma unroll 1
    for (uint32_t k = 1; k <= 10; ++k) {
      const uint32_t T = nchunks >> k;
      if (T == 0) break;
      const uint32_t half = 1u << (k - 1);
#pragma unroll 1
      for (uint32_t t = tid; t < T; t += kWG) {
        const uint32_t s = t << k;
        uint32_t l[8], r[8], o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          l[i] = cvs[s][i];
          r[i] = cvs[s + half][i];
        }
        parent(l, r, false, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = o[i];
      }
      __syncthreads();
    }
    // maximal nodes: the binary decomposition of nchunks (one node for a full piece)
    for (uint32_t s = tid; s < nchunks; s += kWG) {
      const uint32_t k = 31 - __clz(nchunks - s);
      if ((s & ((1u << k) - 1)) || (s != (nchunks & ~((2u << k) - 1)))) continue;
      const uint64_t idx = pd.node_base + (nchunks == kTile ? pd.j0 / kTile : pd.j0 / kTile + __popc(nchunks >> (k + 1)));
      uint4* o = reinterpret_cast<uint4*>(file_nodes + 8ull * idx);
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
    __syncthreads();
    pi = nx;
  }
}

// one workgroup per big file: merge its node list (Q level-10 piece CVs, then
// the tail decomposition) into the root. The Q piece CVs are reduced
// 1024 at a time in LDS (complete aligned groups of pieces are tree nodes);
// the maximal groups and the tail nodes are merged by lane 0 with the
// subtree-stack rule, the last merge being ROOT.
__global__ void __launch_bounds__(kWG) k_bigfile_finish(const FileDesc* __restrict__ files, uint32_t nfiles,
                                                        const uint32_t* __restrict__ file_nodes,
                                                        uint8_t* __restrict__ out32) {
  __shared__ uint32_t cvs[kTile][8];
  __shared__ uint16_t task[kTile / 2];
  __shared__ uint32_t ntask[16];
  __shared__ uint32_t stack[kMaxStackBig][8];
  __shared__ uint32_t depth_s;
  const uint32_t tid = threadIdx.x;
  const uint32_t fi = blockIdx.x;
  if (fi >= nfiles) return;
  const FileDesc fd = files[fi];
  const uint64_t C = fd.C;
  const uint64_t Q = C / kTile;
  const uint32_t r = (uint32_t)(C % kTile);
  if (tid == 0) depth_s = 0;
  // lane 0 pushes node (chunk position j, cv) after merging what j completes
  auto push = [&](uint64_t j, const uint32_t (&cv)[8]) {
    uint32_t depth = depth_s;
    const uint32_t keep = __popcll(j);
    while (depth > keep) {
      uint32_t a[8], b[8], o[8];
      for (int i = 0; i < 8; ++i) { a[i] = stack[depth - 2][i]; b[i] = stack[depth - 1][i]; }
      parent(a, b, false, o);
      for (int i = 0; i < 8; ++i) stack[depth - 2][i] = o[i];
      --depth;
    }
    for (int i = 0; i < 8; ++i) stack[depth][i] = cv[i];
    depth_s = depth + 1;
  };
  for (uint64_t b0 = 0; b0 < Q; b0 += kTile) {
    const uint32_t nb = (uint32_t)min<uint64_t>(kTile, Q - b0);
    if (tid < 16) ntask[tid] = 0;
    for (uint32_t s = tid; s < nb; s += kWG) {
      const uint4* p = reinterpret_cast<const uint4*>(file_nodes + 8ull * (fd.node_base + b0 + s));
      uint4 a = p[0], b = p[1];
      cvs[s][0] = a.x; cvs[s][1] = a.y; cvs[s][2] = a.z; cvs[s][3] = a.w;
      cvs[s][4] = b.x; cvs[s][5] = b.y; cvs[s][6] = b.z; cvs[s][7] = b.w;
    }
    __syncthreads();
    // groups of 2^k pieces: aligned, complete, and not the whole file
    for (uint32_t k = 1; (1u << k) <= kTile; ++k) {
      const uint32_t w = 1u << k;
      for (uint32_t s = tid; s < nb; s += kWG)
        if (!(s & (w - 1)) && s + w <= nb && (uint64_t)w * kTile < C) task[atomicAdd(&ntask[k], 1u)] = (uint16_t)s;
      __syncthreads();
      const uint32_t T = ntask[k];
      if (T == 0) break;
#pragma unroll 1
      for (uint32_t t = tid; t < T; t += kWG) {
        const uint32_t s = task[t];
        uint32_t l[8], rr[8], o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          l[i] = cvs[s][i];
          rr[i] = cvs[s + (w >> 1)][i];
        }
        parent(l, rr, false, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = o[i];
      }
      __syncthreads();
    }
    if (tid == 0) {
      // maximal groups in order: greedy largest computed group at each position
      uint32_t s = 0;
      while (s < nb) {
        uint32_t k = 0;
        while (true) {
          const uint32_t w = 2u << k;
          if ((s & (w - 1)) || s + w > nb || (uint64_t)w * kTile >= C) break;
          ++k;
        }
        uint32_t cv[8];
        for (int i = 0; i < 8; ++i) cv[i] = cvs[s][i];
        const uint64_t j = (b0 + s) * kTile;
        const uint64_t jn = j + ((uint64_t)kTile << k);
        if (jn == C) {
          // whole remainder done: fold (only when r == 0 and this is the last group)
          uint32_t depth = depth_s;
          const uint32_t keep = __popcll(j);
          while (depth > keep) {
            uint32_t a[8], bb[8], o[8];
            for (int i = 0; i < 8; ++i) { a[i] = stack[depth - 2][i]; bb[i] = stack[depth - 1][i]; }
            parent(a, bb, false, o);
            for (int i = 0; i < 8; ++i) stack[depth - 2][i] = o[i];
            --depth;
          }
          for (int d = (int)depth - 1; d >= 0; --d) {
            uint32_t a[8], o[8];
            for (int i = 0; i < 8; ++i) a[i] = stack[d][i];
            parent(a, cv, d == 0, o);
            for (int i = 0; i < 8; ++i) cv[i] = o[i];
          }
          uint4* o = reinterpret_cast<uint4*>(out32 + 32ull * fd.out_index);
          o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
          o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
          depth_s = 0;
        } else {
          push(j, cv);
        }
        s += 1u << k;
      }
    }
    __syncthreads();
  }
  if (r && tid == 0) {
    // tail nodes, decreasing sizes, at file_nodes[node_base + Q + t]
    uint64_t j = Q * kTile;
    uint32_t t = 0;
    for (int k = 9; k >= 0; --k) {
      if (!((r >> k) & 1)) continue;
      const uint4* p = reinterpret_cast<const uint4*>(file_nodes + 8ull * (fd.node_base + Q + t));
      uint4 a = p[0], b = p[1];
      uint32_t cv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint64_t jn = j + (1ull << k);
      if (jn == C) {
        uint32_t depth = depth_s;
        const uint32_t keep = __popcll(j);
        while (depth > keep) {
          uint32_t aa[8], bb[8], o[8];
          for (int i = 0; i < 8; ++i) { aa[i] = stack[depth - 2][i]; bb[i] = stack[depth - 1][i]; }
          parent(aa, bb, false, o);
          for (int i = 0; i < 8; ++i) stack[depth - 2][i] = o[i];
          --depth;
        }
        for (int d = (int)depth - 1; d >= 0; --d) {
          uint32_t aa[8], o[8];
          for (int i = 0; i < 8; ++i) aa[i] = stack[d][i];
          parent(aa, cv, d == 0, o);
          for (int i = 0; i < 8; ++i) cv[i] = o[i];
        }
        uint4* o = reinterpret_cast<uint4*>(out32 + 32ull * fd.out_index);
        o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
        o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
      } else {
        push(j, cv);
      }
      j = jn;
      ++t;
    }
  }
}

// ---------------------------------------------------------------------------

#ifdef SDCAS_ABLATIONS
using QuadIt = hipcub::TransformInputIterator<uint64_t, QuadSlotsOp, hipcub::CountingInputIterator<uint32_t>>;
#endif

size_t batch_scan_temp_bytes(uint32_t max_msgs) {
  size_t qbytes = 0;
#ifdef SDCAS_ABLATIONS
  QuadIt qit(hipcub::CountingInputIterator<uint32_t>(0), QuadSlotsOp{nullptr, max_msgs});
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, qbytes, qit, (uint64_t*)nullptr, (int)max_msgs);
#endif
  // the slot plan's workgroup sums (k_plan_sums)
  const size_t plan = sizeof(uint64_t) * ((size_t)max_msgs / kPlanPer + 2);
  return std::max(qbytes, plan);
}

// Leaf/tree kernel variants, numbered as in the A/B runs of rounds 1-2
//  so that profiles/ and tools/ keep their meaning. libsdcas.so
// holds only the bit-exact, GPU-tested product kernels (PROD: the default,
// 52, and 51, the same without its copy-free first column steps); every other
// entry is compiled only into the ablation library (ABL), and the stagger /
// priority experiments (8, 9, 11, 12, 37) are retired (RET).
struct LeafVariant {
  const void* fn;
  int wg;
  int quad = 0;      // 1: quad slot layout (k_leaf_quad / k_finish_t<kQTile>, needs the shape-sorted order)
  int one_tile = 0;  // 1: one tile per workgroup (DYN 2): the grid covers the workspace's tiles
  uint32_t tile = kTile;  // chunk slots per tile (kSmallTile: the small-batch kernel)
};
#define PROD(wg, ...) {(const void*)__VA_ARGS__, wg}
#define PROD1(wg, ...) {(const void*)__VA_ARGS__, wg, 0, 1}
#define PRODS(wg, ...) {(const void*)__VA_ARGS__, wg, 0, 1, kSmallTile}
#ifdef SDCAS_ABLATIONS
#define ABLS(wg, ...) {(const void*)__VA_ARGS__, wg, 0, 1, kSmallTile}
#else
#define ABLS(wg, ...) {nullptr, wg, 0, 1, kSmallTile}
#endif
#ifdef SDCAS_ABLATIONS
#define ABL(wg, ...) {(const void*)__VA_ARGS__, wg}
#define ABLQ(wg, ...) {(const void*)__VA_ARGS__, wg, 1}
#else
#define ABL(wg, ...) {nullptr, wg}
#define ABLQ(wg, ...) {nullptr, wg, 1}
#endif
#define RET {nullptr, 512}
#ifdef SDCAS_ABLATIONS
#define ABL1(wg, ...) {(const void*)__VA_ARGS__, wg, 0, 1}
#else
#define ABL1(wg, ...) {nullptr, wg, 0, 1}
#endif
static const LeafVariant kLeafVariants[] = {
    ABL(512, k_leaf_tree<512, 0>),   // 0: plain block loop
    ABL(512, k_leaf_tree<512, 1>),   // 1: next block prefetched
    ABL(256, k_leaf_tree<256, 1>),   // 2, 3: 256 / 1024 threads per workgroup
    ABL(1024, k_leaf_tree<1024, 1>),
    ABL(512, k_leaf_tree<512, 2>),   // 4 DIAGNOSTIC (wrong digests): no memory reads
    ABL(512, k_leaf_tree<512, 3>),   // 5 DIAGNOSTIC (wrong digests): no compression
    ABL(512, k_leaf_tree<512, 1, 0>),  // 6, 7 DIAGNOSTIC (wrong digests): no in-tile tree; neither tree nor loads
    ABL(512, k_leaf_tree<512, 2, 0>),
    RET, RET,                          // 8, 9: workgroups staggered by a fraction of a tile
    ABL(512, k_leaf_tree<512, 4>),   // 10: ping-pong block loop
    RET, RET,                          // 11, 12: tree waves at priority 1
    ABL(512, k_leaf_tree<512, 5>),   // 13: non-temporal message loads
    ABL(512, k_leaf_slim<512, 1, 8>),  // 14-16: compact LDS (4 workgroups per CU)
    ABL(512, k_leaf_slim<512, 1, 6>),
    ABL(512, k_leaf_slim<512, 0, 8>),
    ABL(512, k_leaf_tree<512, 6>),   // 17: prefetch distance two blocks
    ABL(512, k_leaf_tree<512, 7>),   // 18: 128-byte pair loads
    ABL(512, k_leaf_slim<512, 1, 6, 1>),  // 19, 20: compact LDS + leaf order by block count
    ABL(512, k_leaf_slim<512, 0, 6, 1>),
    ABLQ(512, k_leaf_quad<1>),        // 21, 22: quad layout (four chunks per lane)
    ABLQ(512, k_leaf_quad<0>),
    ABL(512, k_leaf_slim<512, 4, 6>),  // 23, 24: compact LDS + ping-pong under a 6 / 5 wave register cap
    ABL(512, k_leaf_slim<512, 4, 5>),
    ABL(512, k_leaf_tree<512, 1, 1, 1>),     // 25: leaf order by block count
    ABL(512, k_leaf_tree<512, 2, 1, 1>),     // 26-28 DIAGNOSTIC (wrong digests): 25 without loads / tree / both
    ABL(512, k_leaf_tree<512, 1, 0, 1>),
    ABL(512, k_leaf_tree<512, 2, 0, 1>),
    ABL(512, k_leaf_tree<512, 1, 1, 1, 1>),  // 29: 25 + tiles from a global counter (dynamic schedule)
    ABL(512, k_leaf_slim<512, 1, 8, 0, 1>),  // 30-33: compact LDS with the dynamic schedule
    ABL(512, k_leaf_slim<512, 1, 6, 1, 1>),
    ABL(512, k_leaf_slim<512, 1, 8, 1, 1>),
    ABL(512, k_leaf_slim<512, 0, 8, 0, 1>),
    ABL(1024, k_leaf_tree<1024, 1, 1, 1, 1>),  // 34: 29 at 1024 threads
    ABL(512, k_leaf_tree<512, 1, 1, 0, 1>),    // 35: 29 without the leaf order
    ABL(512, k_leaf_tree<512, 4, 1, 1, 1>),    // 36: 29 with the ping-pong block loop
    RET,                                        // 37: 29 with tree waves at priority 1
    ABL(512, k_leaf_tree<512, 6, 1, 1, 1>),    // 38: 29 with prefetch distance two
    ABL(512, k_leaf_tree<512, 4, 0, 1, 1>),    // 39-41 DIAGNOSTIC (wrong digests): 36 without tree / loads / both
    ABL(512, k_leaf_tree<512, 2, 1, 1, 1>),
    ABL(512, k_leaf_tree<512, 2, 0, 1, 1>),
    ABL(512, k_leaf_tree<512, 7, 1, 1, 1>),    // 42: 29 with 128-byte pair loads
    ABL(512, k_leaf_tree<512, 8, 1, 1, 1>),    // 43 (round 1's default): 36 with both halves of a line loaded together
    ABL1(512, k_leaf_tree<512, 8, 1, 1, 2>),   // 44: 43 with one tile per workgroup (hardware dispatch)
    ABL1(512, k_leaf_tree<512, 4, 1, 1, 2>),   // 45: 36 with one tile per workgroup
    ABL1(512, k_leaf_tree<512, 9, 1, 1, 2>),   // 46: 44 with the last-block-index loop (hash_chunk_pl)
    ABL(512, k_leaf_tree<512, 9, 1, 1, 1>),    // 47: 43 with the last-block-index loop
    ABL(512, k_leaf_tree<512, 9, 1, 1, 1, 1>),    // 48: 47 with the leaf's chunk kept in registers from phase 1
    ABL1(512, k_leaf_tree<512, 9, 1, 1, 2, 1>),   // 49: 46 with the same
    ABL1(512, k_leaf_tree<512, 9, 1, 1, 2, 2>),   // 50: 49 keeping only the first slot's chunk (no spills)
    ABL1(512, k_leaf_tree<512, 109, 1, 1, 2, 2>),   // 51: 50 with the asm G blocks (B3_G_ASM)
    PROD1(512, k_leaf_tree<512, 209, 1, 1, 2, 2>),  // 52 (round 2's default): 51 with copy-free first column steps (compress<2>)
    ABL1(512, k_leaf_tree<512, 119, 1, 1, 2, 2>),   // 53: 51 with non-temporal message loads (1.7x slower)
    ABL1(512, k_leaf_tree<512, 129, 1, 1, 2, 2>),   // 54: 51 with the tail mask computed in its branch
    ABL1(512, k_leaf_tree<512, 229, 1, 1, 2, 2>),   // 55: 52 with the same
    ABL1(512, k_leaf_tree<512, 102, 1, 1, 2, 2>),   // 56 DIAGNOSTIC (wrong digests): 51's compression, no memory reads
    ABL1(512, k_leaf_tree<512, 139, 1, 1, 2, 2>),   // 57 DIAGNOSTIC (wrong digests): 51 reading a wave-transposed image
    ABL1(512, k_leaf_tree<512, 149, 1, 1, 2, 2>),   // 58 DIAGNOSTIC (wrong digests): 51 reading an L2-resident 2 MiB
    ABL1(512, k_leaf_tree<512, 209, 0, 1, 2, 2>),   // 59 DIAGNOSTIC (wrong digests): 52 without the in-tile tree
    ABL1(512, k_leaf_tree<512, 209, 2, 1, 2, 2>),   // 60: 52 with every lane of a tree wave computing (prices masked lanes)
    ABL1(1024, k_leaf_tree<1024, 229, 1, 1, 2, 2, 8>),  // 61: 55 at 1024 threads, one slot per lane, 8 waves/SIMD
    ABL1(1024, k_leaf_tree<1024, 209, 1, 1, 2, 2, 8>),  // 62: 52 at 1024 threads, one slot per lane, 8 waves/SIMD
    ABL1(1024, k_leaf_tree<1024, 229, 1, 1, 2, 2, 6>),  // 63: 61 at 6 waves/SIMD (register budget of 52)
    ABL1(512, k_leaf_tree<512, 269, 1, 2, 2, 2>),   // 64: 52 with whole chunks first in every tile and waves of whole chunks through hash_chunk_full
    ABL1(512, k_leaf_tree<512, 269, 1, 1, 2, 2>),   // 65: 64 without the two-bin order (the full-chunk loop where a wave happens to hold only whole chunks)
    ABL1(512, k_leaf_tree<512, 209, 1, 2, 2, 2>),   // 66: 52 with the two-bin order only (its cost)
    PROD1(512, k_leaf_tree<512, 279, 1, 1, 2, 2>),  // 67 (default since round 3): 52 with the tail masks from a table
    ABL1(512, k_leaf_tree<512, 289, 1, 1, 2, 2>),   // 68: 65 with the tail masks from a table
    ABL1(512, k_leaf_tree<512, 279, 3, 1, 2, 2>),   // 69 DIAGNOSTIC (wrong digests): 67 without the tree levels 5-10
    ABL1(512, k_leaf_tree<512, 279, 0, 1, 2, 2>),   // 70 DIAGNOSTIC (wrong digests): 67 without the in-tile tree
    // 71 (product, the small-batch kernel): tiles of kSmallTile slots, one
    // slot per lane, the compiler-scheduled G (a lone wave issues the four
    // independent G chains of a half-round together; the asm blocks issue one
    // chain at a time) and the tail-mask table
    PRODS(kSmallTile, k_leaf_tree<kSmallTile, 79, 1, 1, 2, 2, 0, kSmallTile>),
    ABLS(kSmallTile, k_leaf_tree<kSmallTile, 279, 1, 1, 2, 2, 0, kSmallTile>),  // 72: 71 with the asm G blocks (slower: 1-100 files +6-12 %)
    // 73 (product): 71 with a quad of lanes per slot (compress_quad), no leaf
    // order, 512 threads for the 128 slots
    PRODS(4 * kSmallTile, k_leaf_tree<4 * kSmallTile, 79, 1, 0, 2, 0, 0, kSmallTile, 1>),
    ABL1(512, k_leaf_tree<512, 299, 1, 1, 2, 2>),  // 74: 67 with the split line-pair loop (hash_chunk_split)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 3>),  // 75: 67 with quad tree levels and phase-4 bits (XT 3)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 1>),  // 76: 67 with quad tree levels (XT 1)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 2>),  // 77: 67 with phase-4 bits (XT 2)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 7>),  // 78: 75 with the tree tasks appended per wave (XT 7)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 8>),   // 79-82: 67 with its code shifted by 4, 8, 12, 16 bytes
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 16>),  //   (s_nop at the entry: code placement A/B)
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 24>),
    ABL1(512, k_leaf_tree<512, 279, 1, 1, 2, 2, 0, kTile, 0, 32>),
    // 83 (round 6): 73 with four blocks of each chunk in flight
    // (hash_chunk_quad4): a one-file call's kernel -4 %, superseded by 84
    ABLS(4 * kSmallTile, k_leaf_tree<4 * kSmallTile, 79, 1, 0, 2, 0, 0, kSmallTile, 2>),
    // 84 (product, the small-batch default since round 6): 83 with each
    // quad's block staged in LDS and every lane reading its rounds' 28 words
    // from it (hash_chunk_quad_lds, compress_quad_w: no per-round word
    // selects, 453 -> 141 v_cndmask in the kernel)
    PRODS(4 * kSmallTile, k_leaf_tree<4 * kSmallTile, 79, 1, 0, 2, 0, 0, kSmallTile, 3>),
};
#undef PROD
#undef PROD1
#undef PRODS
#undef ABLS
#undef ABL1
#undef ABL
#undef ABLQ
#undef RET
constexpr int kNumLeafVariants = sizeof(kLeafVariants) / sizeof(kLeafVariants[0]);
constexpr int kDefaultLeafVariant = 67;

int leaf_variant_count() { return kNumLeafVariants; }
// SDCAS_LEAF_VARIANT names a variant this build holds (then every batch runs it)
bool leaf_variant_forced() {
  static const bool f = [] {  // read once, thread-safe (the path calls run on the callers' threads)
    const char* e = getenv("SDCAS_LEAF_VARIANT");
    return e && leaf_variant_available(atoi(e));
  }();
  return f;
}
bool leaf_variant_available(int v) { return v >= 0 && v < kNumLeafVariants && kLeafVariants[v].fn != nullptr; }

// SDCAS_LEAF_VARIANT selects a variant for A/B runs; a variant this build
// does not hold (every diagnostic one in libsdcas.so) falls back to the default
int leaf_variant() {
  static const int v = [] {
    const char* e = getenv("SDCAS_LEAF_VARIANT");
    const int x = e ? atoi(e) : kDefaultLeafVariant;
    return leaf_variant_available(x) ? x : kDefaultLeafVariant;
  }();
  return v;
}

int batch_grid(int device, int variant) {
  static std::atomic<int> cached[64][kNumLeafVariants];  // zero-initialised (static storage)
  const bool cacheable = device >= 0 && device < 64 && variant >= 0 && variant < kNumLeafVariants;
  if (cacheable && cached[device][variant].load(std::memory_order_relaxed))
    return cached[device][variant].load(std::memory_order_relaxed);
  int cus = 256, per = 1;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kLeafVariants[variant].fn, kLeafVariants[variant].wg, 0);
  if (per < 1) per = 1;
  if (getenv("SDCAS_DEBUG_GRID")) fprintf(stderr, "leaf variant %d: %d workgroups/CU\n", variant, per);
  int g = cus * per;
  if (cacheable) cached[device][variant].store(g, std::memory_order_relaxed);
  return g;
}

uint64_t batch_plan_host(const uint64_t* lens, uint32_t n, uint32_t tile, uint64_t cap_slots, uint64_t* S,
                         uint32_t* tile_first, uint64_t* total, bool* crossing) {
  uint64_t s = 0, tiles = 0;
  bool cross = false;
  for (uint32_t m = 0; m < n; ++m) {
    const uint64_t C = chunk_count(lens[m]);
    S[m] = s;
    for (uint64_t t = (s + tile - 1) / tile; t * tile < s + C && t * tile < cap_slots; ++t) tile_first[t] = m;
    cross |= s / tile != (s + C - 1) / tile;
    s += C;
  }
  tiles = (s + tile - 1) / tile;
  total[0] = s;
  total[1] = total[2] = total[3] = 0;
  *crossing = cross;
  return tiles;
}

hipError_t batch_hash(const BatchWorkspace& ws, const uint8_t* blob, const uint64_t* offs, const uint64_t* lens,
                      uint32_t n, uint8_t* out32, uint64_t* out_keys, hipStream_t st, uint64_t max_chunks,
                      hipEvent_t ev0, hipEvent_t ev1, const BatchPlan* plan) {
  if (n == 0) return hipSuccess;
  if (n > ws.cap_msgs) return hipErrorInvalidValue;
  [[maybe_unused]] hipError_t e;  // (the quad-layout ablation's scan)
  const uint32_t* perm = nullptr;
  // A batch of a few messages fills a tile or two whatever their order: its
  // three sort launches would only add latency (the reference's 100-file step).
  if (ws.sort && n >= kSortMinMsgs && ws.perm) {
    // the bin totals, then each workgroup's count per bin (bin-major)
    const uint32_t nwg = (n + kScatterPerWG - 1) / kScatterPerWG;
    uint32_t* totals = ws.sort_keys;
    uint32_t* wcnt = ws.sort_keys + kSortTotalsWords;
    hipLaunchKernelGGL(k_shape_hist, dim3(nwg), dim3(256), 0, st, lens, n, wcnt);
    hipLaunchKernelGGL(k_shape_bins, dim3(kShapeBins), dim3(256), 0, st, wcnt, nwg, totals);
    hipLaunchKernelGGL(k_shape_scatter, dim3(nwg), dim3(256), 0, st, offs, lens, n, totals, wcnt, ws.perm, ws.soffs,
                       ws.slens);
    offs = ws.soffs;
    lens = ws.slens;
    perm = ws.perm;
  }
  const bool forced = leaf_variant_available(ws.variant) || leaf_variant_forced();
  int v = leaf_variant_available(ws.variant) ? ws.variant : leaf_variant();
  bool quad = false;
#ifdef SDCAS_ABLATIONS
  quad = kLeafVariants[v].quad && (perm || n == 1);
  if (kLeafVariants[v].quad && !quad) v = kDefaultLeafVariant;  // the quad layout needs the shape-sorted order
#endif
  // slots the batch may fill: a grid sized to the workspace instead costs a
  // small batch ~45 us of empty workgroups (8449 of them at 256 MiB staging)
  const uint64_t slots =
      max_chunks ? std::min<uint64_t>(ws.cap_slots, max_chunks + (quad ? 3ull * n + 8 : 0)) : ws.cap_slots;
  // A small batch fills a few 1 MiB tiles, each hashed by one CU while the
  // rest idle: unless a variant was chosen, it takes the small-batch kernel,
  // whose tiles of kSmallTile slots spread it over the chip.
  if (!forced && !quad && slots <= ws.small_slots && slots / kSmallTile + 2 <= ws.cap_small_tiles)
    v = leaf_variant_available(ws.small_variant) && kLeafVariants[ws.small_variant].tile == kSmallTile ? ws.small_variant
                                                                                                        : kSmallVariant;
  // a small-tile kernel chosen by hand (A/B) for a batch whose 128-slot tiles
  // outnumber the workspace's tile_first entries runs the default instead
  if (kLeafVariants[v].tile == kSmallTile && slots / kSmallTile + 2 > ws.cap_small_tiles) v = kDefaultLeafVariant;
  const uint32_t tile = kLeafVariants[v].tile;
  // the caller's host plan stands in for the scan and k_tile_first when it
  // was made for this order and tile size
  const bool planned = plan && !perm && !quad && plan->tile == tile;
  uint64_t* const S = planned ? const_cast<uint64_t*>(plan->S) : ws.S;
  uint32_t* const tile_first = planned ? const_cast<uint32_t*>(plan->tile_first) : ws.tile_first;
  uint64_t* const total = planned ? plan->total : ws.total;
  size_t tmp = ws.scan_tmp_bytes;
  if (planned) {
  } else if (quad) {
#ifdef SDCAS_ABLATIONS
    QuadIt qit(hipcub::CountingInputIterator<uint32_t>(0), QuadSlotsOp{lens, n});
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tmp, qit, ws.S, (int)n, st))) return e;
    hipLaunchKernelGGL(k_tile_first_q, dim3((n + 255) / 256), dim3(256), 0, st, lens, ws.S, n, ws.cap_slots,
                       ws.tile_first, ws.total);
#endif
  } else {
    // the workgroup sums live in the scan's temp space (batch_scan_temp_bytes)
    const uint32_t nb = (n + kPlanPer - 1) / kPlanPer;
    if ((size_t)(nb + 1) * sizeof(uint64_t) > tmp) return hipErrorInvalidValue;
    uint64_t* bsum = static_cast<uint64_t*>(ws.scan_tmp);
    hipLaunchKernelGGL(k_plan_sums, dim3(nb), dim3(kPlanWG), 0, st, lens, n, bsum);
    hipLaunchKernelGGL(k_plan_scan, dim3(1), dim3(1024), 0, st, bsum, nb, ws.total);
    if (tile == kSmallTile)
      hipLaunchKernelGGL(k_plan_write<kSmallTile>, dim3(nb), dim3(kPlanWG), 0, st, lens, n, bsum, ws.cap_slots, ws.S,
                         ws.tile_first);
    else
      hipLaunchKernelGGL(k_plan_write<kTile>, dim3(nb), dim3(kPlanWG), 0, st, lens, n, bsum, ws.cap_slots, ws.S,
                         ws.tile_first);
  }
  if (ev0) (void)hipEventRecord(ev0, st);
  {
    int dev = 0;
    (void)hipGetDevice(&dev);
    const int grid = kLeafVariants[v].one_tile ? (int)std::min<uint64_t>(slots / tile + 1, 0x7FFFFFFF)
                                               : batch_grid(dev, v);
    void* args[] = {(void*)&blob,     (void*)&offs,       (void*)&lens,     (void*)&n,
                    (void*)&S,        (void*)&tile_first, (void*)&total,    (void*)&ws.cap_slots,
                    (void*)&ws.nodes, (void*)&out32,      (void*)&out_keys, (void*)&perm};
    hipError_t le = hipLaunchKernel(kLeafVariants[v].fn, dim3(grid), dim3(kLeafVariants[v].wg), args, 0, st);
    if (le != hipSuccess) return le;
  }
  if (ev1) (void)hipEventRecord(ev1, st);
  if (quad) {
#ifdef SDCAS_ABLATIONS
    const uint64_t tiles = slots / kQTile + 1;
    hipLaunchKernelGGL(k_finish_t<kQTile>, dim3((uint32_t)((tiles + kFinishWG - 1) / kFinishWG)), dim3(kFinishWG), 0,
                       st, lens, n, ws.S, ws.tile_first, ws.total, ws.cap_slots, ws.nodes, perm, out32, out_keys);
#endif
  } else if (planned && !plan->crossing) {
    // every message ended inside its tile: the leaf kernel wrote them all
  } else if (tile == kSmallTile) {
    launch_finish<kSmallTile>(slots / kSmallTile + 1, st, lens, n, S, tile_first, total, ws.cap_slots, ws.nodes, perm,
                              out32, out_keys);
  } else {
    launch_finish<kTile>(slots / kTile + 1, st, lens, n, S, tile_first, total, ws.cap_slots, ws.nodes, perm, out32,
                         out_keys);
  }
  return hipGetLastError();
}

// Piece kernel variants. Product: 17 = one workgroup per 1 MiB piece, whole
// chunks through hash_chunk_full (no per-block length, flag or tail-mask work
// on a lane; the block index is wave-uniform), partial chunks through the
// leaf kernel's line-pair block loop, 6 waves/SIMD, every G step a B3_G_ASM
// block with the copy-free first column steps (b3_device.h, compress<2>);
// 19 (default since round 3) = 17 whose full pieces stop at tree level 4
// (k_piece_l4) and k_piece_top runs levels 5-10 of eight pieces per
// workgroup: those levels are one nearly empty wave-issue each when one
// piece owns the workgroup (1.0 % faster in a same-process A/B, bit-exact,
// profiles/r03_ab_piece_17_19.txt; the DIAGNOSTIC 18 bounded the gain at
// 1.1 %). Ablation library only: 15 = 17 with whole chunks through the
// line-pair loop (round 3's first-session product pair, 1.7 % slower,
// profiles/r03_ab_piece_15_17.txt), 14 = 15 without
// the copy-free first column steps (round 2's product pair), 4 = ping-pong
// block loop (round 1's default), 6 = 14 with the compiler-scheduled G (round
// 2's default before B3_G_ASM: 10 % slower), 11 = persistent grid on a global
// piece counter (k_piece_dyn), 12 = 11 with the next piece's first line loaded
// before the current piece's tree levels, 13 = 11 at 8 waves/SIMD (11-13 lost
// to the hardware dispatcher), the older plain / prefetch loops, rotated chunk
// orders, a round-robin persistent grid, and the DIAGNOSTIC 7 (no memory
// reads), 16 and 18 (15 and 17 without the in-piece tree levels 5-10: what
// the one-wave levels cost).
constexpr int kDefaultPieceVariant = 19;

bool piece_variant_available(int v) {
  if (v == 17 || v == 19) return true;
#ifdef SDCAS_ABLATIONS
  if (v >= 0 && v <= 20) return true;
#endif
  return false;
}

int piece_variant() {
  static const int v = [] {
    const char* e = getenv("SDCAS_PIECE_VARIANT");
    const int x = e ? atoi(e) : kDefaultPieceVariant;
    return piece_variant_available(x) ? x : kDefaultPieceVariant;
  }();
  return v;
}

#ifdef SDCAS_ABLATIONS
static int piece_grid(const void* fn) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kWG, 0);
  return (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
}

template <int MINW, int PRE>
static hipError_t launch_piece_dyn(const uint8_t* blob, const PieceDesc* pieces, uint32_t npieces,
                                   uint32_t* file_nodes, uint32_t* ctr, hipStream_t st) {
  static int grid = 0;  // the same on every MI355X of the node
  if (!grid) grid = piece_grid((const void*)k_piece_dyn<MINW, PRE>);
  hipError_t e = hipMemsetAsync(ctr, 0, sizeof(uint32_t), st);
  if (e) return e;
  hipLaunchKernelGGL((k_piece_dyn<MINW, PRE>), dim3(std::min<uint32_t>(npieces, (uint32_t)grid)), dim3(kWG), 0, st,
                     blob, pieces, npieces, file_nodes, ctr);
  return hipGetLastError();
}

static hipError_t piece_hash_ablation(int v, const uint8_t* blob, const PieceDesc* pieces, uint32_t npieces,
                                      uint32_t* file_nodes, uint32_t* ctr, uint32_t* l4, hipStream_t st) {
  if (v == 20) {  // 19 at 8 waves/SIMD (64 VGPRs; the spills are outside the full-chunk loop)
    if (!l4) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_piece_l4<259, 8>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes, l4);
    hipLaunchKernelGGL((k_piece_top<259>), dim3((npieces + kTopPieces - 1) / kTopPieces), dim3(kWG), 0, st, pieces,
                       npieces, l4, file_nodes);
    return hipGetLastError();
  }
  if (v == 11) return launch_piece_dyn<6, 0>(blob, pieces, npieces, file_nodes, ctr, st);
  if (v == 12) return launch_piece_dyn<6, 1>(blob, pieces, npieces, file_nodes, ctr, st);
  if (v == 13) return launch_piece_dyn<8, 0>(blob, pieces, npieces, file_nodes, ctr, st);
  if (v == 16)  // DIAGNOSTIC (wrong digests): 15 without the in-piece tree levels 5-10
    hipLaunchKernelGGL((k_piece_tree<208, 6, 1, 0, 4>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces,
                       file_nodes);
  else if (v == 14)  // 15 without the copy-free first column steps
    hipLaunchKernelGGL((k_piece_tree<108, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 18)  // DIAGNOSTIC (wrong digests): 17 without the in-piece tree levels 5-10
    hipLaunchKernelGGL((k_piece_tree<259, 6, 1, 0, 4>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces,
                       file_nodes);
  else if (v == 15)  // 17 with whole chunks through the line-pair loop
    hipLaunchKernelGGL((k_piece_tree<208, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  if (v >= 14) return hipGetLastError();
  if (v == 0) hipLaunchKernelGGL((k_piece_tree<0, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 1)
    hipLaunchKernelGGL((k_piece_tree<1, 8>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 2)
    hipLaunchKernelGGL((k_piece_tree<1, 8, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 3)
    hipLaunchKernelGGL((k_piece_tree<1, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 5)
    hipLaunchKernelGGL((k_piece_tree<4, 8, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 6)
    hipLaunchKernelGGL((k_piece_tree<8, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 7)  // DIAGNOSTIC (wrong digests): 4's loop without memory reads
    hipLaunchKernelGGL((k_piece_tree<2, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 8)  // 4 with per-workgroup rotated chunk order
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 9)  // 6 with per-workgroup rotated chunk order
    hipLaunchKernelGGL((k_piece_tree<8, 6, 1, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 10) {  // 4 as a persistent grid dealing pieces round-robin
    static int grid = 0;
    if (!grid) grid = piece_grid((const void*)k_piece_tree<4, 6, 1>);
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1>), dim3(std::min<uint32_t>(npieces, (uint32_t)grid)), dim3(kWG), 0, st,
                       blob, pieces, npieces, file_nodes);
  } else  // 4
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  return hipGetLastError();
}
#endif

hipError_t piece_hash(const uint8_t* blob, const PieceDesc* pieces, uint32_t npieces, uint32_t* file_nodes,
                      uint32_t* ctr, uint32_t* l4, int variant, hipStream_t st) {
  if (!npieces) return hipSuccess;
  const int v = piece_variant_available(variant) ? variant : piece_variant();
  if (v == 19) {
    if (!l4) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_piece_l4<259, 6>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes, l4);
    hipLaunchKernelGGL((k_piece_top<259>), dim3((npieces + kTopPieces - 1) / kTopPieces), dim3(kWG), 0, st, pieces,
                       npieces, l4, file_nodes);
    return hipGetLastError();
  }
#ifdef SDCAS_ABLATIONS
  if (v != 17) return piece_hash_ablation(v, blob, pieces, npieces, file_nodes, ctr, l4, st);
#else
  (void)ctr;
#endif
  hipLaunchKernelGGL((k_piece_tree<259, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  return hipGetLastError();
}

// One thread per piece: its segment by binary search over the segments'
// first pieces (a few hundred at most, L2-resident), then the piece's
// descriptor. 32 B written per piece (8 MiB for C4's 256 Ki pieces).
__global__ void __launch_bounds__(256) k_expand_pieces(const SegDesc* __restrict__ segs, uint32_t nseg,
                                                       PieceDesc* __restrict__ pieces, uint32_t npieces) {
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;
  if (p >= npieces) return;
  uint32_t lo = 0, hi = nseg;  // segs[lo].piece_first <= p < segs[hi].piece_first
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].piece_first <= p) lo = mid;
    else hi = mid;
  }
  const SegDesc sg = segs[lo];
  const uint64_t o = (uint64_t)(p - sg.piece_first) * (1024ull * kTile);
  PieceDesc pd;
  pd.off = sg.off + o;
  pd.j0 = sg.j0 + o / 1024;
  pd.node_base = sg.node_base;
  pd.len = (uint32_t)(sg.len - o < 1024ull * kTile ? sg.len - o : 1024ull * kTile);
  pd.pad = 0;
  pieces[p] = pd;
}

hipError_t expand_pieces(const SegDesc* segs, uint32_t nseg, PieceDesc* pieces, uint32_t npieces, hipStream_t st) {
  if (!npieces) return hipSuccess;
  if (!nseg) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_expand_pieces, dim3((npieces + 255) / 256), dim3(256), 0, st, segs, nseg, pieces, npieces);
  return hipGetLastError();
}

hipError_t bigfile_finish(const FileDesc* files, uint32_t nfiles, const uint32_t* file_nodes, uint8_t* out32,
                          hipStream_t st) {
  if (!nfiles) return hipSuccess;
  hipLaunchKernelGGL(k_bigfile_finish, dim3(nfiles), dim3(kWG), 0, st, files, nfiles, file_nodes, out32);
  return hipGetLastError();
}


}  // namespace sdcas
