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
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <cstdio>

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
__host__ __device__ inline uint32_t node_level(uint64_t j, uint64_t C, uint32_t s) {
  uint32_t k = 0;
  for (;;) {
    uint64_t w = 2ull << k;
    if ((j & (w - 1)) || j + w > C || w >= C || (uint64_t)s + w > kTile) break;
    ++k;
  }
  return k;
}

// Is the level-k node at (j, s) consumed by a parent computed in the same tile?
__host__ __device__ inline bool parent_in_tile(uint64_t j, uint64_t C, uint32_t s, uint32_t k) {
  uint64_t w = 1ull << k;
  if (!((j >> k) & 1)) return false;  // left children's parents start at s: not computed
  return j + w <= C && 2 * w < C && s >= w && (uint64_t)s + w <= kTile;
}

struct ChunkCountOp {
  __host__ __device__ uint64_t operator()(uint64_t len) const { return chunk_count(len); }
};

__global__ void k_tile_first(const uint64_t* __restrict__ lens, const uint64_t* __restrict__ S, uint32_t n,
                             uint64_t cap_chunks, uint32_t* __restrict__ tile_first, uint64_t* __restrict__ total) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  uint64_t s0 = S[m], C = chunk_count(lens[m]);
  if (m == n - 1) {
    total[0] = s0 + C;
    total[2] = 0;  // k_leaf_tree<DYN>'s tile counter
  }
  for (uint64_t t = (s0 + kTile - 1) / kTile; t * kTile < s0 + C && t * kTile < cap_chunks; ++t) tile_first[t] = m;
}

// Hash one chunk (`clen` bytes at p, 0 <= clen <= 1024) with chunk counter j.
__device__ __forceinline__ void hash_chunk(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                           uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
#pragma unroll 1
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
    uint32_t m[16];
    load_full_block(p + b * BLOCK_LEN, m);
    if (blen < BLOCK_LEN) mask_tail(m, blen);
    const uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? (CHUNK_END | (root ? ROOT : 0u)) : 0u);
    compress(cv, m, j, blen, flags);
  }
}

// Same, with the next block's loads issued before the current block is
// compressed (software pipelining: one 64-byte block per lane in flight while
// the VALU works). The load address is clamped to the chunk's last block, so
// the final iteration re-reads it harmlessly instead of running off the end.
template <bool NT = false>
__device__ __forceinline__ void hash_chunk_pf(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                              uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  uint32_t m[16];
  if (NT) load_full_block_nt(p, m);
  else load_full_block(p, m);
#pragma unroll 1
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t nx[16];
    if (NT) load_full_block_nt(p + min(b + 1, nb - 1) * BLOCK_LEN, nx);
    else load_full_block(p + min(b + 1, nb - 1) * BLOCK_LEN, nx);
    const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
    if (blen < BLOCK_LEN) mask_tail(m, blen);
    const uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? (CHUNK_END | (root ? ROOT : 0u)) : 0u);
    compress(cv, m, j, blen, flags);
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = nx[i];
  }
}

// Same, unrolled by two blocks with ping-pong message registers (no
// register copies between blocks; block b+1's loads fly while b compresses).
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
      compress(cv, m0, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));
    }
    if (b + 1 < nb) {
      load_full_block(p + min(b + 2, nb - 1) * BLOCK_LEN, m0);
      const uint32_t blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m1, blen);
      compress(cv, m1, j, blen, b + 2 == nb ? endf : 0u);
    }
  }
}

// Same, two blocks of prefetch distance (three rotating message register
// sets, unrolled by three): block b+2's loads fly while b compresses.
#define B3_PF2_STEP(cur, nxt_blk)                                                              \
  {                                                                                            \
    const uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);                                \
    if (blen < BLOCK_LEN) mask_tail(cur, blen);                                                \
    compress(cv, cur, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));       \
    if (++b >= nb) break;                                                                      \
    load_full_block(p + min(nxt_blk, nb - 1) * BLOCK_LEN, cur);                                \
  }
__device__ __forceinline__ void hash_chunk_pf2(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                               uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  uint32_t x[16], y[16], z[16];
  load_full_block(p, x);
  load_full_block(p + min(1u, nb - 1) * BLOCK_LEN, y);
  load_full_block(p + min(2u, nb - 1) * BLOCK_LEN, z);
  uint32_t b = 0;
#pragma unroll 1
  for (;;) {
    B3_PF2_STEP(x, b + 2)
    B3_PF2_STEP(y, b + 2)
    B3_PF2_STEP(z, b + 2)
  }
}
#undef B3_PF2_STEP

// Same, loading 128 bytes (two blocks, one L2 line of a 128-byte aligned
// chunk) per step into one register set while the previous pair compresses.
// The pair load at an odd last block is cut to 64 bytes so nothing past the
// guaranteed 64-byte tail is read.
__device__ __forceinline__ void load_pair(const uint8_t* p, uint32_t b, uint32_t nb, uint32_t (&m)[32]) {
  const uint4* q = reinterpret_cast<const uint4*>(p + b * BLOCK_LEN);
  uint4 r[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = q[i];
  if (b + 1 < nb) {
#pragma unroll
    for (int i = 4; i < 8; ++i) r[i] = q[i];
  } else {
#pragma unroll
    for (int i = 4; i < 8; ++i) r[i] = r[i - 4];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[4 * i] = r[i].x; m[4 * i + 1] = r[i].y; m[4 * i + 2] = r[i].z; m[4 * i + 3] = r[i].w;
  }
}
__device__ __forceinline__ void hash_chunk_pair(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                                uint32_t (&cv)[8]) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
  const uint32_t endf = CHUNK_END | (root ? ROOT : 0u);
  uint32_t cur[32];
  load_pair(p, 0, nb, cur);
#pragma unroll 1
  for (uint32_t b = 0; b < nb; b += 2) {
    uint32_t nx[32];
    load_pair(p, min(b + 2, (nb - 1) & ~1u), nb, nx);
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = cur[i];
    uint32_t blen = min(BLOCK_LEN, clen - b * BLOCK_LEN);
    if (blen < BLOCK_LEN) mask_tail(m, blen);
    compress(cv, m, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));
    if (b + 1 < nb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = cur[16 + i];
      blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m, blen);
      compress(cv, m, j, blen, b + 2 == nb ? endf : 0u);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) cur[i] = nx[i];
  }
}

// Same two register sets as the ping-pong loop, but both 64-byte halves of a
// 128-byte line are requested together (no prefetch across lines): the second
// half never waits in L2 for a compression and cannot be evicted before it is
// read; the load latency is left to the other waves of the SIMD.
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
      compress(cv, m0, j, blen, (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? endf : 0u));
    }
    if (b + 1 < nb) {
      const uint32_t blen = min(BLOCK_LEN, clen - (b + 1) * BLOCK_LEN);
      if (blen < BLOCK_LEN) mask_tail(m1, blen);
      compress(cv, m1, j, blen, b + 2 == nb ? endf : 0u);
    }
  }
}

// DIAGNOSTIC ONLY (wrong digests, never the default): PF=2 compresses
// register-made blocks without touching memory (pure VALU rate); PF=3 streams
// the chunk's blocks and folds them with XOR, no compression (pure load rate).
__device__ __forceinline__ void hash_chunk_diag(const uint8_t* __restrict__ p, uint32_t clen, uint64_t j, bool root,
                                                uint32_t (&cv)[8], int mode) {
  set_iv(cv);
  const uint32_t nb = clen == 0 ? 1 : (clen + BLOCK_LEN - 1) / BLOCK_LEN;
#pragma unroll 1
  for (uint32_t b = 0; b < nb; ++b) {
    uint32_t m[16];
    if (mode == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = (uint32_t)(uintptr_t)p + b * 64 + i;
      compress(cv, m, j, 64, b == 0 ? CHUNK_START : 0u);
    } else if (mode == 3) {
      load_full_block(p + b * BLOCK_LEN, m);
#pragma unroll
      for (int i = 0; i < 16; ++i) cv[i & 7] ^= m[i];
    }
  }
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
__host__ __device__ constexpr uint32_t task_base(uint32_t k) { return 2 * (kTile - (kTile >> (k - 1))); }
constexpr uint32_t kTaskCap = 2 * (kTile - 1);
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
constexpr uint32_t kGroups = kTile / 64;

template <int WG>
__device__ __forceinline__ void leaf_order(uint32_t tid, const uint32_t (&bin)[kTile / WG], uint16_t* __restrict__ order,
                                           uint16_t* __restrict__ gcnt) {
  const uint32_t lane = tid & 63;
  uint32_t rk[kTile / WG];
#pragma unroll
  for (uint32_t r = 0; r < kTile / WG; ++r) {
    const uint32_t g = (tid + r * WG) >> 6;
    uint32_t mine = 0, cnt_l = 0;
#pragma unroll 1
    for (uint32_t b = 0; b < 17; ++b) {
      const uint64_t m = __ballot(bin[r] == b);
      if (bin[r] == b) mine = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == b) cnt_l = (uint32_t)__popcll(m);
    }
    rk[r] = mine;
    if (lane < 17) gcnt[lane * kGroups + g] = (uint16_t)cnt_l;
  }
  __syncthreads();
  if (tid < 64) {
    // exclusive scan of the 17 x kGroups counts in bin-major order
    constexpr uint32_t kPer = (17 * kGroups + 63) / 64;
    uint32_t v[kPer], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t e = tid * kPer + q;
      v[q] = e < 17 * kGroups ? gcnt[e] : 0u;
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
      if (e < 17 * kGroups) gcnt[e] = (uint16_t)acc;
      acc += v[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kTile / WG; ++r) {
    const uint32_t s = tid + r * WG;
    order[gcnt[bin[r] * kGroups + (s >> 6)] + rk[r]] = (uint16_t)s;
  }
  __syncthreads();
}

template <int WG, int PF, int TR = 1, int STAGGER = 0, int PRIO = 0, int ORD = 0, int DYN = 0>
__global__ void __launch_bounds__(WG, ORD ? 6 : 1) k_leaf_tree(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offs,
                                                   const uint64_t* __restrict__ lens, uint32_t n,
                                                   const uint64_t* __restrict__ S,
                                                   const uint32_t* __restrict__ tile_first,
                                                   const uint64_t* __restrict__ total_p, uint64_t cap_chunks,
                                                   uint32_t* __restrict__ nodes, uint8_t* __restrict__ out32,
                                                   uint64_t* __restrict__ out_keys, const uint32_t* __restrict__ perm) {
  __shared__ uint32_t cvs[kTile][8];   // chunk / node chaining values, by slot
  __shared__ uint64_t sS[kTile + 1];   // S[] of the tile's messages
  __shared__ uint16_t smsg[kTile];     // slot -> message index in the tile (kNoMsg: past the end)
  __shared__ uint32_t task[kTaskCap];  // tree tasks by level (enc_task)
  __shared__ uint32_t ntask[12];
  __shared__ uint16_t order[ORD ? kTile : 1];  // leaf loop position -> slot
  __shared__ uint64_t next_tile;

  const uint64_t total = *total_p;
  if (total > cap_chunks) return;  // reported by sdcas_dev_sync
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t tid = threadIdx.x;
  if (STAGGER) {
    // Co-resident workgroups run identical tiles in lockstep, so their
    // barrier-bound tree phases coincide and leave the CU's SIMDs idle.
    // Offset them once by a fraction of a tile (speed only).
    const uint32_t phase = (blockIdx.x / (gridDim.x / (STAGGER ? STAGGER : 1))) % (STAGGER ? STAGGER : 1);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t wait = (uint64_t)phase * 25000 / STAGGER;  // 100 MHz ticks: ~250 us per tile
    while (__builtin_amdgcn_s_memrealtime() - t0 < wait) __builtin_amdgcn_s_sleep(100);
  }

  // DYN: tiles after the first are handed out by a global counter (total_p[2],
  // zeroed by k_tile_first) instead of round-robin, so a workgroup that drew
  // cheap tiles takes more and the grid drains within about one tile; the
  // next tile is claimed at the start of the current one (the atomic's
  // latency hides behind the tile) and read after its last barrier
  unsigned long long* tile_ctr = reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(total_p) + 2);
  for (uint64_t tile = blockIdx.x; tile < ntiles;) {
    const uint64_t tbase = tile * kTile;
    const uint32_t m0 = tile_first[tile];
    const uint32_t m1 = (tile + 1 < ntiles) ? tile_first[tile + 1] : n - 1;
    const uint32_t cnt = m1 - m0 + 1;  // <= kTile + 1
    for (uint32_t i = tid; i < cnt; i += WG) sS[i] = S[m0 + i];
    if (tid < 12) ntask[tid] = 0;
    if (DYN && tid == 0) next_tile = gridDim.x + atomicAdd(tile_ctr, 1ull);
    __syncthreads();

    // (1) slot -> message, and the tree schedule: every aligned complete
    // power-of-two node inside the tile (level k task at its first slot), plus
    // the spine of each message lying wholly in the tile — the right-to-left
    // fold over its binary decomposition, one step per part, scheduled in the
    // level after that part's node is complete; the last step is the ROOT.
#pragma unroll 1
    for (uint32_t s = tid; s < kTile; s += WG) {
      const uint64_t g = tbase + s;
      if (g >= total) {
        smsg[s] = kNoMsg;
        continue;
      }
      uint32_t lo = 0, hi = cnt - 1;  // last message with S <= g
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (sS[mid] <= g) lo = mid;
        else hi = mid - 1;
      }
      smsg[s] = (uint16_t)lo;
      if (!TR) continue;
      const uint64_t j = g - sS[lo];
      const uint64_t C = chunk_count(lens[m0 + lo]);
      if (C == 1) continue;
      const uint32_t K = node_level(j, C, s);
      for (uint32_t k = 1; k <= K; ++k)
        task[task_base(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s, s + (1u << (k - 1)), 0, false);
    }
#pragma unroll 1
    for (uint32_t i = tid; TR && i < cnt; i += WG) {
      const uint64_t S0 = sS[i];
      if (S0 < tbase) continue;
      const uint64_t C = chunk_count(lens[m0 + i]);
      if (C == 1 || S0 + C > tbase + kTile) continue;
      const uint32_t s0 = (uint32_t)(S0 - tbase), c = (uint32_t)C;
      if (!(c & (c - 1))) {
        const uint32_t k = 31 - __clz(c);
        task[task_base(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s0, s0 + (c >> 1), i, true);
      } else {
        uint32_t rem = c, part = rem & (0u - rem);
        uint32_t pos = c - part, acc = pos;
        rem -= part;
        while (rem) {
          part = rem & (0u - rem);
          pos -= part;
          const uint32_t k = 32 - __clz(part);  // log2(part) + 1
          task[task_base(k) + atomicAdd(&ntask[k], 1u)] = enc_task(s0 + pos, s0 + acc, i, rem == part);
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
    const bool ord = ORD && cnt > 64 && chunk_count(lens[m0 + cnt - 1]) > 1;
    if (ord) {
      uint32_t bin[kTile / WG];
#pragma unroll
      for (uint32_t r = 0; r < kTile / WG; ++r) {
        const uint32_t s = tid + r * WG;
        const uint32_t mi = smsg[s];
        bin[r] = mi == kNoMsg ? 16u : leaf_bin(lens[m0 + mi], tbase + s - sS[mi]);
      }
      // the per (bin, 64-slot group) counts borrow cvs, which no one reads
      // between the previous tile's last barrier and this tile's leaves
      leaf_order<WG>(tid, bin, order, reinterpret_cast<uint16_t*>(&cvs[0][0]));
    }
#pragma unroll 1
    for (uint32_t i = tid; i < kTile; i += WG) {
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
      if (PF == 8) hash_chunk_ps(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF == 6) hash_chunk_pf2(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF == 7) hash_chunk_pair(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF == 4) hash_chunk_pp(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF == 5) hash_chunk_pf<true>(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF >= 2) hash_chunk_diag(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv, PF);
      else if (PF) hash_chunk_pf(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else hash_chunk(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      if (root) {
        store_digest(perm ? perm[m] : m, cv, out32, out_keys);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
      }
    }
    __syncthreads();

    // (3) the tree, level by level: every task of a level is independent
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);  // the few tree waves gate the barrier: let them issue first
    for (uint32_t k = 1; TR && k <= 10; ++k) {
      const uint32_t T = ntask[k];
      if (T == 0) continue;
#pragma unroll 1
      for (uint32_t t = tid; t < T; t += WG) {
        const uint32_t e = task[task_base(k) + t];
        const uint32_t l = e & 1023u, r = (e >> 10) & 1023u;
        const bool root = e >> 31;
        uint32_t a[8], b[8], o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          a[q] = cvs[l][q];
          b[q] = cvs[r][q];
        }
        parent(a, b, root, o);
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
    if (PRIO) __builtin_amdgcn_s_setprio(0);

    // (4) messages crossing a tile boundary: their maximal in-tile nodes go to
    // HBM at their first slot, for k_finish
#pragma unroll 1
    for (uint32_t s = tid; TR && s < kTile; s += WG) {
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t S0 = sS[mi];
      const uint64_t C = chunk_count(lens[m0 + mi]);
      if (C == 1 || (S0 >= tbase && S0 + C <= tbase + kTile)) continue;  // single chunk / spine done in (3)
      const uint64_t j = tbase + s - S0;
      const uint32_t k = node_level(j, C, s);
      if (parent_in_tile(j, C, s, k)) continue;
      uint4* o = reinterpret_cast<uint4*>(nodes + 8ull * (tbase + s));
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
    __syncthreads();
    tile = DYN ? next_tile : tile + gridDim.x;
  }
}

// k_leaf_slim: k_leaf_tree's algorithm with a 39 KB LDS image, so four
// 512-thread workgroups (8 waves per SIMD) fit in a CU's 160 KB when the
// kernel also fits 64 VGPRs (__launch_bounds__ MINW = 8):
//   * message starts relative to the tile as u16 (a message other than the
//     tile's first starts inside it: 1..1024); the first message's start is
//     the uniform S[m0];
//   * tree tasks as u16 (left slot | ROOT << 15): the right child of a level-k
//     task is always 2^(k-1) slots further and a root's message is the owner
//     of its left slot; tasks are counted per level first, then written
//     compacted (a tile holds at most kTile - 1 parent compressions).
constexpr uint16_t kTaskRoot = 0x8000;

template <int WG, int PF, int MINW, int ORD = 0, int DYN = 0>
__global__ void __launch_bounds__(WG, MINW) k_leaf_slim(const uint8_t* __restrict__ blob,
                                                        const uint64_t* __restrict__ offs,
                                                        const uint64_t* __restrict__ lens, uint32_t n,
                                                        const uint64_t* __restrict__ S,
                                                        const uint32_t* __restrict__ tile_first,
                                                        const uint64_t* __restrict__ total_p, uint64_t cap_chunks,
                                                        uint32_t* __restrict__ nodes, uint8_t* __restrict__ out32,
                                                        uint64_t* __restrict__ out_keys,
                                                        const uint32_t* __restrict__ perm) {
  __shared__ uint32_t cvs[kTile][8];
  __shared__ uint16_t srel[kTile + 2];
  __shared__ uint16_t smsg[kTile];
  __shared__ uint16_t task[kTile];
  __shared__ uint32_t ntask[12], tbase_k[12];
  // ORD: leaf order by block count (slots whose chunks have the same number
  // of blocks share waves, so a partial last chunk does not idle 63 lanes)
  __shared__ uint16_t order[ORD ? kTile : 1];
  __shared__ uint32_t obin[ORD ? 17 : 1];
  __shared__ uint64_t next_tile;  // DYN: k_leaf_tree's global tile counter

  const uint64_t total = *total_p;
  if (total > cap_chunks) return;
  const uint64_t ntiles = (total + kTile - 1) / kTile;
  const uint32_t tid = threadIdx.x;
  unsigned long long* tile_ctr = reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(total_p) + 2);

  for (uint64_t tile = blockIdx.x; tile < ntiles;) {
    const uint64_t tbase = tile * kTile;
    const uint32_t m0 = tile_first[tile];
    const uint32_t m1 = (tile + 1 < ntiles) ? tile_first[tile + 1] : n - 1;
    const uint32_t cnt = m1 - m0 + 1;  // <= kTile + 1
    const uint64_t lead = tbase - S[m0];  // chunks of the first message before this tile
    for (uint32_t i = tid + 1; i < cnt; i += WG) srel[i] = (uint16_t)(S[m0 + i] - tbase);
    if (tid < 12) ntask[tid] = 0;
    if (ORD && tid < 17) obin[tid] = 0;
    if (DYN && tid == 0) next_tile = gridDim.x + atomicAdd(tile_ctr, 1ull);
    __syncthreads();

    // (1a) slot -> message; count the tree tasks of every level
#pragma unroll 1
    for (uint32_t s = tid; s < kTile; s += WG) {
      if (tbase + s >= total) {
        smsg[s] = kNoMsg;
        continue;
      }
      uint32_t lo = 0, hi = cnt - 1;  // last message starting at or before slot s
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (srel[mid] <= s) lo = mid;
        else hi = mid - 1;
      }
      smsg[s] = (uint16_t)lo;
      const uint64_t j = lo ? (uint64_t)(s - srel[lo]) : lead + s;
      const uint64_t len = lens[m0 + lo];
      const uint64_t C = chunk_count(len);
      if (ORD) atomicAdd(&obin[leaf_bin(len, j)], 1u);
      if (C == 1) continue;
      const uint32_t K = node_level(j, C, s);
      for (uint32_t k = 1; k <= K; ++k) atomicAdd(&ntask[k], 1u);
      // a message lying wholly in the tile starts here: its spine steps
      if (j == 0 && (lo || lead == 0) && s + C <= kTile) {
        const uint32_t c = (uint32_t)C;
        if (!(c & (c - 1))) {
          atomicAdd(&ntask[31 - __clz(c)], 1u);
        } else {
          uint32_t rem = c & (c - 1);  // the lowest part is not a step of its own
          while (rem) {
            const uint32_t part = rem & (0u - rem);
            atomicAdd(&ntask[32 - __clz(part)], 1u);
            rem -= part;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int k = 1; k <= 10; ++k) {
        tbase_k[k] = acc;
        acc += ntask[k];
        ntask[k] = 0;
      }
      tbase_k[11] = acc;
      if (ORD) {
        uint32_t o = 0;
        for (int b = 0; b < 17; ++b) {
          const uint32_t c = obin[b];
          obin[b] = o;
          o += c;
        }
      }
    }
    __syncthreads();
    // (1b) write the tasks, compacted by level
#pragma unroll 1
    for (uint32_t s = tid; s < kTile; s += WG) {
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t j = mi ? (uint64_t)(s - srel[mi]) : lead + s;
      const uint64_t len1 = lens[m0 + mi];
      const uint64_t C = chunk_count(len1);
      if (ORD) order[atomicAdd(&obin[leaf_bin(len1, j)], 1u)] = (uint16_t)s;
      if (C == 1) continue;
      const uint32_t K = node_level(j, C, s);
      for (uint32_t k = 1; k <= K; ++k) task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)s;
      if (j == 0 && (mi || lead == 0) && s + C <= kTile) {
        const uint32_t c = (uint32_t)C;
        if (!(c & (c - 1))) {
          const uint32_t k = 31 - __clz(c);
          task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)(s | kTaskRoot);
        } else {
          // right-to-left fold over the binary decomposition of c
          uint32_t rem = c, part = rem & (0u - rem);
          uint32_t pos = c - part;
          rem -= part;
          while (rem) {
            part = rem & (0u - rem);
            pos -= part;
            const uint32_t k = 32 - __clz(part);
            task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)((s + pos) | (rem == part ? kTaskRoot : 0u));
            rem -= part;
          }
        }
      }
    }

    // (2) leaves
    if (ORD) __syncthreads();  // order[] is complete
    const uint32_t nleaf = ORD ? obin[16] : kTile;
#pragma unroll 1
    for (uint32_t i = tid; i < nleaf; i += WG) {
      const uint32_t s = ORD ? order[i] : i;
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint32_t m = m0 + mi;
      const uint64_t j = mi ? (uint64_t)(s - srel[mi]) : lead + s;
      const uint64_t len = lens[m];
      const uint32_t clen = len == 0 ? 0u : (uint32_t)min<uint64_t>(CHUNK_LEN, len - j * CHUNK_LEN);
      const bool root = len <= CHUNK_LEN;
      uint32_t cv[8];
      if (PF == 4) hash_chunk_pp(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else if (PF) hash_chunk_pf(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      else hash_chunk(blob + offs[m] + j * CHUNK_LEN, clen, j, root, cv);
      if (root) {
        store_digest(perm ? perm[m] : m, cv, out32, out_keys);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
      }
    }
    __syncthreads();

    // (3) the tree, level by level
    for (uint32_t k = 1; k <= 10; ++k) {
      const uint32_t T = ntask[k];
      if (T == 0) continue;
      const uint32_t base = tbase_k[k], half = 1u << (k - 1);
#pragma unroll 1
      for (uint32_t t = tid; t < T; t += WG) {
        const uint32_t e = task[base + t];
        const uint32_t l = e & 1023u, r = l + half;
        const bool root = e & kTaskRoot;
        uint32_t a[8], b[8], o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          a[q] = cvs[l][q];
          b[q] = cvs[r][q];
        }
        parent(a, b, root, o);
        if (root) {
          const uint32_t mm = m0 + smsg[l];
          store_digest(perm ? perm[mm] : mm, o, out32, out_keys);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) cvs[l][q] = o[q];
        }
      }
      __syncthreads();
    }

    // (4) maximal in-tile nodes of messages crossing a tile boundary
#pragma unroll 1
    for (uint32_t s = tid; s < kTile; s += WG) {
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t C = chunk_count(lens[m0 + mi]);
      if (C == 1) continue;
      const bool inside = mi ? (srel[mi] + C <= kTile) : (lead == 0 && C <= kTile);
      if (inside) continue;
      const uint64_t j = mi ? (uint64_t)(s - srel[mi]) : lead + s;
      const uint32_t k = node_level(j, C, s);
      if (parent_in_tile(j, C, s, k)) continue;
      uint4* o = reinterpret_cast<uint4*>(nodes + 8ull * (tbase + s));
      o[0] = make_uint4(cvs[s][0], cvs[s][1], cvs[s][2], cvs[s][3]);
      o[1] = make_uint4(cvs[s][4], cvs[s][5], cvs[s][6], cvs[s][7]);
    }
    __syncthreads();
    tile = DYN ? next_tile : tile + gridDim.x;
  }
}

// ---- quad layout: four consecutive chunks per lane ----------------------------
//
// The in-tile tree of k_leaf_tree parks a workgroup's waves at one barrier per
// level while a few waves compress (profiles/r01_pmc_sq_variants_c2.json: 18 %
// of wave time). Here every lane owns an aligned group of four chunk slots of
// one message and reduces it in registers — P(P(c0,c1), P(c2,c3)), a BLAKE3
// tree node because the group is aligned inside the message — so levels 1 and
// 2 need no barrier, a tile holds 2048 slots for the same 32 KB of node LDS,
// and the barrier-bound levels start at 3 (8 chunks). The leaf phase per lane
// grows to 64 compressions + 3 parents, the tree phase keeps its length, so
// the parked share of a tile halves.
//
// Slot layout (requires the shape-sorted order, single-chunk messages first):
// a single-chunk message takes one slot; the last of them is padded so the
// first multi-chunk message starts on a multiple of 4; a multi-chunk message
// takes its chunk count rounded up to 4 (the padding slots are dead). Every
// node starts on an even slot, so node CVs live at cvs[slot / 2].
constexpr uint32_t kQTile = 2048;

template <uint32_t TILE>
__host__ __device__ inline uint32_t node_level_t(uint64_t j, uint64_t C, uint32_t s) {
  uint32_t k = 0;
  for (;;) {
    uint64_t w = 2ull << k;
    if ((j & (w - 1)) || j + w > C || w >= C || (uint64_t)s + w > TILE) break;
    ++k;
  }
  return k;
}

template <uint32_t TILE>
__host__ __device__ inline bool parent_in_tile_t(uint64_t j, uint64_t C, uint32_t s, uint32_t k) {
  uint64_t w = 1ull << k;
  if (!((j >> k) & 1)) return false;
  return j + w <= C && 2 * w < C && s >= w && (uint64_t)s + w <= TILE;
}

__host__ __device__ inline uint64_t quad_slots(const uint64_t* lens, uint32_t n, uint32_t i) {
  const uint64_t C = chunk_count(lens[i]);
  if (C > 1) return (C + 3) & ~3ull;
  if (i + 1 < n && chunk_count(lens[i + 1]) > 1) return 1 + ((4 - ((i + 1) & 3)) & 3);
  return 1;
}

struct QuadSlotsOp {
  const uint64_t* lens;
  uint32_t n;
  __host__ __device__ uint64_t operator()(uint32_t i) const { return quad_slots(lens, n, i); }
};

__global__ void k_tile_first_q(const uint64_t* __restrict__ lens, const uint64_t* __restrict__ S, uint32_t n,
                               uint64_t cap_slots, uint32_t* __restrict__ tile_first, uint64_t* __restrict__ total) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const uint64_t s0 = S[m], Q = quad_slots(lens, n, m);
  if (m == n - 1) *total = s0 + Q;
  for (uint64_t t = (s0 + kQTile - 1) / kQTile; t * kQTile < s0 + Q && t * kQTile < cap_slots; ++t) tile_first[t] = m;
}

template <int PF>
__device__ __forceinline__ void quad_chunk(const uint8_t* __restrict__ base, uint64_t len, uint64_t j, bool root,
                                           uint32_t (&cv)[8]) {
  const uint32_t clen = len == 0 ? 0u : (uint32_t)min<uint64_t>(CHUNK_LEN, len - j * CHUNK_LEN);
  if (PF) hash_chunk_pf(base + j * CHUNK_LEN, clen, j, root, cv);
  else hash_chunk(base + j * CHUNK_LEN, clen, j, root, cv);
}

__device__ __forceinline__ void lds_get(const uint32_t (*cvs)[8], uint32_t i, uint32_t (&o)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = cvs[i][q];
}
__device__ __forceinline__ void lds_put(uint32_t (*cvs)[8], uint32_t i, const uint32_t (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) cvs[i][q] = v[q];
}

template <int PF>
__global__ void __launch_bounds__(512, 6) k_leaf_quad(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offs,
                                                   const uint64_t* __restrict__ lens, uint32_t n,
                                                   const uint64_t* __restrict__ S,
                                                   const uint32_t* __restrict__ tile_first,
                                                   const uint64_t* __restrict__ total_p, uint64_t cap_slots,
                                                   uint32_t* __restrict__ nodes, uint8_t* __restrict__ out32,
                                                   uint64_t* __restrict__ out_keys,
                                                   const uint32_t* __restrict__ perm) {
  constexpr uint32_t T = kQTile, WG = 512;
  __shared__ uint32_t cvs[T / 2][8];  // node CVs by first slot / 2
  __shared__ uint16_t srel[T + 2];    // message starts relative to the tile (messages 1..)
  __shared__ uint16_t smsg[T];        // slot -> message in the tile
  __shared__ uint16_t task[T / 4];    // level >= 3 merges of group nodes: < T / 4
  __shared__ uint32_t ntask[13], tbase_k[13];

  const uint64_t total = *total_p;
  if (total > cap_slots) return;
  const uint64_t ntiles = (total + T - 1) / T;
  const uint32_t tid = threadIdx.x;

  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t tbase = tile * T;
    const uint32_t m0 = tile_first[tile];
    const uint32_t m1 = (tile + 1 < ntiles) ? tile_first[tile + 1] : n - 1;
    const uint32_t cnt = m1 - m0 + 1;
    const uint64_t lead = tbase - S[m0];
    for (uint32_t i = tid + 1; i < cnt; i += WG) srel[i] = (uint16_t)(S[m0 + i] - tbase);
    if (tid < 13) ntask[tid] = 0;
    __syncthreads();

    // (1a) slot -> message; count the level >= 3 merges: regular nodes of 8+
    // chunks, and the spine of every multi-group message lying in the tile
#pragma unroll 1
    for (uint32_t s = tid; s < T; s += WG) {
      if (tbase + s >= total) {
        smsg[s] = kNoMsg;
        continue;
      }
      uint32_t lo = 0, hi = cnt - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (srel[mid] <= s) lo = mid;
        else hi = mid - 1;
      }
      smsg[s] = (uint16_t)lo;
      const uint64_t j = lo ? (uint64_t)(s - srel[lo]) : lead + s;
      const uint64_t C = chunk_count(lens[m0 + lo]);
      if (C <= 4 || j >= C) continue;
      const uint32_t K = node_level_t<T>(j, C, s);
      for (uint32_t k = 3; k <= K; ++k) atomicAdd(&ntask[k], 1u);
      if (j == 0 && (lo || lead == 0) && s + C <= T) {
        const uint32_t c = (uint32_t)C;
        if (!(c & (c - 1))) {
          atomicAdd(&ntask[31 - __clz(c)], 1u);
        } else {
          uint32_t rem = c & ~3u;
          if (!(c & 3)) rem &= rem - 1;  // the lowest 4+ part is the fold's start, not a step
          while (rem) {
            const uint32_t part = rem & (0u - rem);
            atomicAdd(&ntask[32 - __clz(part)], 1u);
            rem -= part;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int k = 3; k <= 11; ++k) {
        tbase_k[k] = acc;
        acc += ntask[k];
        ntask[k] = 0;
      }
    }
    __syncthreads();
    // (1b) write the merges, compacted by level
#pragma unroll 1
    for (uint32_t s = tid; s < T; s += WG) {
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t j = mi ? (uint64_t)(s - srel[mi]) : lead + s;
      const uint64_t C = chunk_count(lens[m0 + mi]);
      if (C <= 4 || j >= C) continue;
      const uint32_t K = node_level_t<T>(j, C, s);
      for (uint32_t k = 3; k <= K; ++k) task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)s;
      if (j == 0 && (mi || lead == 0) && s + C <= T) {
        const uint32_t c = (uint32_t)C;
        if (!(c & (c - 1))) {
          const uint32_t k = 31 - __clz(c);
          task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)(s | kTaskRoot);
        } else {
          // right-to-left fold: the tail (< 4 chunks, folded in its group)
          // or the lowest part is the accumulator; each higher part merges in
          uint32_t rem = c & ~3u, pos;
          if (c & 3) {
            pos = c & ~3u;
          } else {
            pos = c - (rem & (0u - rem));
            rem &= rem - 1;
          }
          while (rem) {
            const uint32_t part = rem & (0u - rem);
            pos -= part;
            const uint32_t k = 32 - __clz(part);
            task[tbase_k[k] + atomicAdd(&ntask[k], 1u)] = (uint16_t)((s + pos) | (rem == part ? kTaskRoot : 0u));
            rem -= part;
          }
        }
      }
    }

    // (2) groups: four chunk slots per lane, reduced in registers
#pragma unroll 1
    for (uint32_t g = tid; g < T / 4; g += WG) {
      const uint32_t s = 4 * g;
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint32_t m = m0 + mi;
      const uint64_t len = lens[m];
      const uint64_t C = chunk_count(len);
      if (C == 1) {
        // up to four single-chunk messages (or the padding after the last)
#pragma unroll 1
        for (uint32_t q = 0; q < 4; ++q) {
          const uint32_t mq = smsg[s + q];
          if (mq == kNoMsg) break;
          const uint64_t jq = mq ? (uint64_t)(s + q - srel[mq]) : lead + s + q;
          if (jq != 0) continue;
          const uint32_t mm = m0 + mq;
          uint32_t cv[8];
          quad_chunk<PF>(blob + offs[mm], lens[mm], 0, true, cv);
          store_digest(perm ? perm[mm] : mm, cv, out32, out_keys);
        }
        continue;
      }
      const uint64_t rel0 = mi ? srel[mi] : 0;
      const uint64_t j0 = mi ? (uint64_t)s - rel0 : lead + s;
      const uint32_t nv = (uint32_t)min<uint64_t>(4, C - j0);
      // the last three chunks of a message lying in the tile are folded here
      // (the spine's first step); a crossing message keeps P(c0,c1) and c2
      const bool fold3 = nv == 3 && (C == 3 || ((mi || lead == 0) && rel0 + C <= T));
      const uint8_t* base = blob + offs[m];
      // chunks one by one; the group's nodes stack up in cvs[2g], cvs[2g+1]
      // and merge as pairs complete (one hash and one parent call site keep
      // the register footprint of a single chunk)
      uint32_t depth = 0;
#pragma unroll 1
      for (uint32_t q = 0; q < nv; ++q) {
        uint32_t cv[8];
        quad_chunk<PF>(base, len, j0 + q, false, cv);
        uint32_t merges = q == 1 ? 1u : (q == 3 ? 2u : 0u);
        if (q == 2 && fold3) merges = 1;
        bool root = false;
#pragma unroll 1
        for (uint32_t t = 0; t < merges; ++t) {
          uint32_t a[8];
          lds_get(cvs, 2 * g + depth - 1, a);
          root = depth == 1 && j0 == 0 && q + 1 == C;  // the merge that completes the whole message
          parent(a, cv, root, cv);
          --depth;
        }
        if (root) {
          store_digest(perm ? perm[m] : m, cv, out32, out_keys);
          break;
        }
        lds_put(cvs, 2 * g + depth, cv);
        ++depth;
      }
    }
    __syncthreads();

    // (3) the tree above the groups, level by level
    for (uint32_t k = 3; k <= 11; ++k) {
      const uint32_t Tk = ntask[k];
      if (Tk == 0) continue;
      const uint32_t base = tbase_k[k], half = 1u << (k - 1);
#pragma unroll 1
      for (uint32_t t = tid; t < Tk; t += WG) {
        const uint32_t e = task[base + t];
        const uint32_t l = e & (T - 1), r = l + half;
        const bool root = e & kTaskRoot;
        uint32_t a[8], b[8], o[8];
        lds_get(cvs, l >> 1, a);
        lds_get(cvs, r >> 1, b);
        parent(a, b, root, o);
        if (root) {
          const uint32_t mm = m0 + smsg[l];
          store_digest(perm ? perm[mm] : mm, o, out32, out_keys);
        } else {
          lds_put(cvs, l >> 1, o);
        }
      }
      __syncthreads();
    }

    // (4) maximal in-tile nodes of messages crossing a tile boundary
#pragma unroll 1
    for (uint32_t s = tid; s < T; s += WG) {
      const uint32_t mi = smsg[s];
      if (mi == kNoMsg) continue;
      const uint64_t C = chunk_count(lens[m0 + mi]);
      if (C <= 4) continue;
      const uint64_t rel0 = mi ? srel[mi] : 0;
      if ((mi || lead == 0) && rel0 + C <= T) continue;
      const uint64_t j = mi ? (uint64_t)s - rel0 : lead + s;
      if (j >= C) continue;
      const uint32_t k = node_level_t<T>(j, C, s);
      if (parent_in_tile_t<T>(j, C, s, k)) continue;
      uint4* o = reinterpret_cast<uint4*>(nodes + 8ull * (tbase + s));
      const uint32_t i = s >> 1;
      o[0] = make_uint4(cvs[i][0], cvs[i][1], cvs[i][2], cvs[i][3]);
      o[1] = make_uint4(cvs[i][4], cvs[i][5], cvs[i][6], cvs[i][7]);
    }
    __syncthreads();
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
template <uint32_t TILE, class At>
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
      parent(l, r, op == 2 && depth == 1, o);
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
  __shared__ uint32_t lstack[kFinishWG][kFinishDepth][8];
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
    merge_nodes_flat<TILE>(nodes, s0, C, [&](int d) { return &lstack[threadIdx.x][d][0]; }, cv);
  else
    merge_nodes_deep<TILE>(nodes, s0, C, cv);
  store_digest(perm ? perm[m] : m, cv, out32, out_keys);
}

// Slot order by message shape: key = min(chunks, 15) << 4 | (blocks in the
// last chunk - 1). Single-chunk messages — whose lanes otherwise run 1..16
// blocks side by side in one wave — end up grouped by block count;
// multi-chunk messages have one short chunk each and are merely clustered.
// A counting sort over the 256 shape bins (histogram, then a scatter that
// reserves each workgroup's range per bin): order inside a bin is not
// specified, which changes nothing but the slot a message lands in.
constexpr uint32_t kShapeBins = 256;
constexpr uint32_t kScatterPerWG = 4096;

__device__ __forceinline__ uint32_t shape_key(uint64_t L) {
  const uint64_t C = chunk_count(L);
  const uint64_t last = L - (C - 1) * CHUNK_LEN;  // 0..1024
  const uint32_t blocks = last == 0 ? 1u : (uint32_t)((last + BLOCK_LEN - 1) / BLOCK_LEN);
  return ((uint32_t)min<uint64_t>(C, 15) << 4) | (blocks - 1);
}

__global__ void __launch_bounds__(256) k_shape_hist(const uint64_t* __restrict__ lens, uint32_t n,
                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[kShapeBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) atomicAdd(&h[shape_key(lens[i])], 1u);
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ void __launch_bounds__(256) k_shape_scatter(const uint64_t* __restrict__ offs,
                                                       const uint64_t* __restrict__ lens, uint32_t n,
                                                       const uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm,
                                                       uint64_t* __restrict__ soffs, uint64_t* __restrict__ slens) {
  __shared__ uint32_t start[kShapeBins], h[kShapeBins], rank[kShapeBins];
  const uint32_t t = threadIdx.x;
  // exclusive scan of the global bin counts (256 entries, one per thread)
  start[t] = counts[t];
  h[t] = 0;
  rank[t] = 0;
  __syncthreads();
  for (uint32_t d = 1; d < kShapeBins; d <<= 1) {
    const uint32_t v = t >= d ? start[t - d] : 0u;
    __syncthreads();
    start[t] += v;
    __syncthreads();
  }
  const uint32_t excl = start[t] - counts[t];
  __syncthreads();
  start[t] = excl;
  const uint32_t lo = blockIdx.x * kScatterPerWG, hi = min(n, lo + kScatterPerWG);
  for (uint32_t i = lo + t; i < hi; i += 256) atomicAdd(&h[shape_key(lens[i])], 1u);
  __syncthreads();
  if (h[t]) start[t] += atomicAdd(&cursor[t], h[t]);  // this workgroup's range in bin t
  __syncthreads();
  for (uint32_t i = lo + t; i < hi; i += 256) {
    const uint64_t L = lens[i];
    const uint32_t k = shape_key(L);
    const uint32_t pos = start[k] + atomicAdd(&rank[k], 1u);
    perm[pos] = i;
    soffs[pos] = offs[i];
    slens[pos] = L;
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

template <int PF, int MINW, int DIRECT = 0, int ROT = 0>
__global__ void __launch_bounds__(kWG, MINW) k_piece_tree(const uint8_t* __restrict__ blob,
                                                          const PieceDesc* __restrict__ pieces, uint32_t npieces,
                                                          uint32_t* __restrict__ file_nodes) {
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
      if (PF == 8) hash_chunk_ps(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv);
      else if (PF == 2) hash_chunk_diag(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv, 2);
      else if (PF == 4) hash_chunk_pp(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv);
      else if (PF) hash_chunk_pf(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv);
      else hash_chunk(blob + pd.off + (uint64_t)s * CHUNK_LEN, clen, pd.j0 + s, false, cv);
#pragma unroll
      for (int i = 0; i < 8; ++i) cvs[s][i] = cv[i];
    }
    __syncthreads();
    for (uint32_t k = 1; (1u << k) <= kTile; ++k) {
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
        parent(l, r, false, o);
#pragma unroll
        for (int i = 0; i < 8; ++i) cvs[s][i] = o[i];
      }
      __syncthreads();
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

using QuadIt = hipcub::TransformInputIterator<uint64_t, QuadSlotsOp, hipcub::CountingInputIterator<uint32_t>>;

size_t batch_scan_temp_bytes(uint32_t max_msgs) {
  size_t bytes = 0, qbytes = 0;
  hipcub::TransformInputIterator<uint64_t, ChunkCountOp, const uint64_t*> it(nullptr, ChunkCountOp());
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, it, (uint64_t*)nullptr, (int)max_msgs);
  QuadIt qit(hipcub::CountingInputIterator<uint32_t>(0), QuadSlotsOp{nullptr, max_msgs});
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, qbytes, qit, (uint64_t*)nullptr, (int)max_msgs);
  return std::max(bytes, qbytes);
}

// leaf/tree kernel variants (workgroup size x block prefetch); the default is
// what bench measurements picked, SDCAS_LEAF_VARIANT overrides for A/B runs
struct LeafVariant {
  const void* fn;
  int wg;
  int quad = 0;  // 1: quad slot layout (k_leaf_quad / k_finish_t<kQTile>, needs the shape-sorted order)
};
static const LeafVariant kLeafVariants[] = {
    {(const void*)k_leaf_tree<512, 0>, 512},
    {(const void*)k_leaf_tree<512, 1>, 512},
    {(const void*)k_leaf_tree<256, 1>, 256},
    {(const void*)k_leaf_tree<1024, 1>, 1024},
    // diagnostic (wrong results): 4 = no memory reads, 5 = no compression
    {(const void*)k_leaf_tree<512, 2>, 512},
    {(const void*)k_leaf_tree<512, 3>, 512},
    // 6, 7 diagnostic (wrong results): no in-tile tree; no tree and no loads
    {(const void*)k_leaf_tree<512, 1, 0>, 512},
    {(const void*)k_leaf_tree<512, 2, 0>, 512},
    // 8, 9: workgroups staggered by 1/3 and 1/2 of a tile
    {(const void*)k_leaf_tree<512, 1, 1, 3>, 512},
    {(const void*)k_leaf_tree<512, 1, 1, 2>, 512},
    // 10: ping-pong block loop; 11: tree waves at priority 1; 12: both
    {(const void*)k_leaf_tree<512, 4>, 512},
    {(const void*)k_leaf_tree<512, 1, 1, 0, 1>, 512},
    {(const void*)k_leaf_tree<512, 4, 1, 0, 1>, 512},
    // 13: non-temporal (streaming) message loads
    {(const void*)k_leaf_tree<512, 5>, 512},
    // 14-16: compact LDS (4 workgroups per CU); min waves/SIMD 8, 6; 16: no prefetch
    {(const void*)k_leaf_slim<512, 1, 8>, 512},
    {(const void*)k_leaf_slim<512, 1, 6>, 512},
    {(const void*)k_leaf_slim<512, 0, 8>, 512},
    // 17: prefetch distance two blocks; 18: 128-byte pair loads
    {(const void*)k_leaf_tree<512, 6>, 512},
    {(const void*)k_leaf_tree<512, 7>, 512},
    // 19, 20: compact LDS + leaf order by block count (6 waves/SIMD); the same without prefetch
    {(const void*)k_leaf_slim<512, 1, 6, 1>, 512},
    {(const void*)k_leaf_slim<512, 0, 6, 1>, 512},
    // 21, 22: quad layout (four chunks per lane, 2048-slot tiles); without prefetch
    {(const void*)k_leaf_quad<1>, 512, 1},
    {(const void*)k_leaf_quad<0>, 512, 1},
    // 23, 24: compact LDS + ping-pong message registers (no copies) under a
    // 6- and 5-wave register cap
    {(const void*)k_leaf_slim<512, 4, 6>, 512},
    {(const void*)k_leaf_slim<512, 4, 5>, 512},
    // 25: leaf order by block count (ballot ranks, no LDS atomics)
    {(const void*)k_leaf_tree<512, 1, 1, 0, 0, 1>, 512},
    // 26-28 diagnostic (wrong results), 25 with: no memory reads; no in-tile tree; neither
    {(const void*)k_leaf_tree<512, 2, 1, 0, 0, 1>, 512},
    {(const void*)k_leaf_tree<512, 1, 0, 0, 0, 1>, 512},
    {(const void*)k_leaf_tree<512, 2, 0, 0, 0, 1>, 512},
    // 29: 25 with tiles handed out by a global counter (dynamic schedule)
    {(const void*)k_leaf_tree<512, 1, 1, 0, 0, 1, 1>, 512},
    // 30-33: compact LDS with the dynamic schedule: 8 waves/SIMD; 6 + leaf
    // order; 8 + leaf order; 30 without prefetch
    {(const void*)k_leaf_slim<512, 1, 8, 0, 1>, 512},
    {(const void*)k_leaf_slim<512, 1, 6, 1, 1>, 512},
    {(const void*)k_leaf_slim<512, 1, 8, 1, 1>, 512},
    {(const void*)k_leaf_slim<512, 0, 8, 0, 1>, 512},
    // 34: 29 at 1024 threads per workgroup (one chunk per lane)
    {(const void*)k_leaf_tree<1024, 1, 1, 0, 0, 1, 1>, 1024},
    // 35-38: 29 without the leaf order; with ping-pong blocks; with tree
    // waves at priority 1; with prefetch distance two
    {(const void*)k_leaf_tree<512, 1, 1, 0, 0, 0, 1>, 512},
    {(const void*)k_leaf_tree<512, 4, 1, 0, 0, 1, 1>, 512},
    {(const void*)k_leaf_tree<512, 1, 1, 0, 1, 1, 1>, 512},
    {(const void*)k_leaf_tree<512, 6, 1, 0, 0, 1, 1>, 512},
    // 39-41 diagnostic (wrong results), 36 with: no in-tile tree; no memory
    // reads (block loop of 29); neither
    {(const void*)k_leaf_tree<512, 4, 0, 0, 0, 1, 1>, 512},
    {(const void*)k_leaf_tree<512, 2, 1, 0, 0, 1, 1>, 512},
    {(const void*)k_leaf_tree<512, 2, 0, 0, 0, 1, 1>, 512},
    // 42: 29 with 128-byte pair loads (a lane reads a whole L2 line at once)
    {(const void*)k_leaf_tree<512, 7, 1, 0, 0, 1, 1>, 512},
    // 43: 36 with both halves of a line loaded together, no prefetch
    {(const void*)k_leaf_tree<512, 8, 1, 0, 0, 1, 1>, 512},
};
constexpr int kNumLeafVariants = sizeof(kLeafVariants) / sizeof(kLeafVariants[0]);
constexpr int kDefaultLeafVariant = 43;

int leaf_variant_count() { return kNumLeafVariants; }

int leaf_variant() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("SDCAS_LEAF_VARIANT");
    v = e ? atoi(e) : kDefaultLeafVariant;
    if (v < 0 || v >= kNumLeafVariants) v = kDefaultLeafVariant;
  }
  return v;
}

int batch_grid(int device, int variant) {
  static int cached[64][64] = {{0}};
  if (device >= 0 && device < 64 && cached[device][variant]) return cached[device][variant];
  int cus = 256, per = 1;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kLeafVariants[variant].fn, kLeafVariants[variant].wg, 0);
  if (per < 1) per = 1;
  if (getenv("SDCAS_DEBUG_GRID")) fprintf(stderr, "leaf variant %d: %d workgroups/CU\n", variant, per);
  int g = cus * per;
  if (device >= 0 && device < 64) cached[device][variant] = g;
  return g;
}

hipError_t batch_hash(const BatchWorkspace& ws, const uint8_t* blob, const uint64_t* offs, const uint64_t* lens,
                      uint32_t n, uint8_t* out32, uint64_t* out_keys, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (n == 0) return hipSuccess;
  if (n > ws.cap_msgs) return hipErrorInvalidValue;
  const uint32_t tb = 256;
  hipError_t e;
  const uint32_t* perm = nullptr;
  if (ws.sort && n > 1 && ws.perm) {
    uint32_t* counts = ws.sort_keys;  // [256] bin sizes, [256] per-bin cursors
    if ((e = hipMemsetAsync(counts, 0, 2 * kShapeBins * sizeof(uint32_t), st))) return e;
    const uint32_t hb = std::min<uint32_t>((n + 255) / 256, 1024u);
    hipLaunchKernelGGL(k_shape_hist, dim3(hb), dim3(256), 0, st, lens, n, counts);
    hipLaunchKernelGGL(k_shape_scatter, dim3((n + kScatterPerWG - 1) / kScatterPerWG), dim3(256), 0, st, offs, lens,
                       n, counts, counts + kShapeBins, ws.perm, ws.soffs, ws.slens);
    offs = ws.soffs;
    lens = ws.slens;
    perm = ws.perm;
  }
  int v = ws.variant >= 0 && ws.variant < kNumLeafVariants ? ws.variant : leaf_variant();
  const bool quad = kLeafVariants[v].quad && (perm || n == 1);
  if (kLeafVariants[v].quad && !quad) v = 1;  // the quad layout needs the shape-sorted order
  size_t tmp = ws.scan_tmp_bytes;
  if (quad) {
    QuadIt qit(hipcub::CountingInputIterator<uint32_t>(0), QuadSlotsOp{lens, n});
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tmp, qit, ws.S, (int)n, st))) return e;
    hipLaunchKernelGGL(k_tile_first_q, dim3((n + tb - 1) / tb), dim3(tb), 0, st, lens, ws.S, n, ws.cap_slots,
                       ws.tile_first, ws.total);
  } else {
    hipcub::TransformInputIterator<uint64_t, ChunkCountOp, const uint64_t*> it(lens, ChunkCountOp());
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, tmp, it, ws.S, (int)n, st))) return e;
    hipLaunchKernelGGL(k_tile_first, dim3((n + tb - 1) / tb), dim3(tb), 0, st, lens, ws.S, n, ws.cap_slots,
                       ws.tile_first, ws.total);
  }
  if (ev0) (void)hipEventRecord(ev0, st);
  {
    int dev = 0;
    (void)hipGetDevice(&dev);
    const int grid = batch_grid(dev, v);
    void* args[] = {(void*)&blob,     (void*)&offs,          (void*)&lens,       (void*)&n,
                    (void*)&ws.S,     (void*)&ws.tile_first, (void*)&ws.total,   (void*)&ws.cap_slots,
                    (void*)&ws.nodes, (void*)&out32,         (void*)&out_keys,   (void*)&perm};
    hipError_t le = hipLaunchKernel(kLeafVariants[v].fn, dim3(grid), dim3(kLeafVariants[v].wg), args, 0, st);
    if (le != hipSuccess) return le;
  }
  if (ev1) (void)hipEventRecord(ev1, st);
  if (quad) {
    const uint64_t tiles = ws.cap_slots / kQTile + 1;
    hipLaunchKernelGGL(k_finish_t<kQTile>, dim3((uint32_t)((tiles + kFinishWG - 1) / kFinishWG)), dim3(kFinishWG), 0,
                       st, lens, n, ws.S, ws.tile_first, ws.total, ws.cap_slots, ws.nodes, perm, out32, out_keys);
  } else {
    const uint64_t tiles = ws.cap_slots / kTile + 1;
    hipLaunchKernelGGL(k_finish_t<kTile>, dim3((uint32_t)((tiles + kFinishWG - 1) / kFinishWG)), dim3(kFinishWG), 0,
                       st, lens, n, ws.S, ws.tile_first, ws.total, ws.cap_slots, ws.nodes, perm, out32, out_keys);
  }
  return hipGetLastError();
}

hipError_t piece_hash(const uint8_t* blob, const PieceDesc* pieces, uint32_t npieces, uint32_t* file_nodes,
                      hipStream_t st) {
  if (!npieces) return hipSuccess;
  // SDCAS_PIECE_VARIANT (A/B): 0 = plain block loop, 1 = block prefetch at 8 waves/SIMD,
  // 2 = 1 with tree tasks indexed directly (one barrier per level), 3 = 2 at 6 waves/SIMD,
  // 4, 5 = 2 with the ping-pong block loop at 6 / 8 waves/SIMD (4: default, +2 % on C4)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SDCAS_PIECE_VARIANT");
    v = e ? atoi(e) : 4;
  }
  if (v == 0) hipLaunchKernelGGL((k_piece_tree<0, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 2)
    hipLaunchKernelGGL((k_piece_tree<1, 8, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 3)
    hipLaunchKernelGGL((k_piece_tree<1, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 4)
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 5)
    hipLaunchKernelGGL((k_piece_tree<4, 8, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 6)  // 4 with both halves of a line loaded together
    hipLaunchKernelGGL((k_piece_tree<8, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 8)  // 4 with per-workgroup rotated chunk order
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 9)  // 6 with per-workgroup rotated chunk order
    hipLaunchKernelGGL((k_piece_tree<8, 6, 1, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else if (v == 10) {  // 4 as a persistent grid (resident workgroups loop over the pieces)
    static int grid = 0;
    if (!grid) {
      int dev = 0, cus = 0, per = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_piece_tree<4, 6, 1>, kWG, 0);
      grid = (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
    }
    hipLaunchKernelGGL((k_piece_tree<4, 6, 1>), dim3(std::min<uint32_t>(npieces, (uint32_t)grid)), dim3(kWG), 0, st,
                       blob, pieces, npieces, file_nodes);
  } else if (v == 7)  // DIAGNOSTIC (wrong digests): 4's loop without memory reads
    hipLaunchKernelGGL((k_piece_tree<2, 6, 1>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  else hipLaunchKernelGGL((k_piece_tree<1, 8>), dim3(npieces), dim3(kWG), 0, st, blob, pieces, npieces, file_nodes);
  return hipGetLastError();
}

hipError_t bigfile_finish(const FileDesc* files, uint32_t nfiles, const uint32_t* file_nodes, uint8_t* out32,
                          hipStream_t st) {
  if (!nfiles) return hipSuccess;
  hipLaunchKernelGGL(k_bigfile_finish, dim3(nfiles), dim3(kWG), 0, st, files, nfiles, file_nodes, out32);
  return hipGetLastError();
}

}  // namespace sdcas
