// dist_dedup.hip — device stages of the multi-GPU identifier group-by.
//
// The reference links file_paths to Objects by cas_id inside one process,
// 100 files at a time (core/src/object/file_identifier/mod.rs:149-254 over
// the chunks of file_identifier_job.rs:296-319). In canonical form (SURVEY.md
// §8a a7; dedup.hip) the whole job reduces to, per cas key X:
//   existing(X) = first Object in DB order carrying X   (mod.rs:181-238)
//   rep(X)      = lowest orphan ordinal carrying X      (mod.rs:246-254)
// and a per-file rule. Both are associative minima, so each rank first
// COMBINES its files to one (key, min ordinal) record per distinct key — a
// Zipf heavy hitter then costs one record per rank, not millions (C5) — the
// records travel to the key's owner rank (RCCL all-to-all, by the caller),
// the owner RESOLVES each key against its slice of existing Objects, and the
// answers travel back in send order for each rank to APPLY to its files.
//
// HBM-bound integer work, no sort anywhere: the combine is a compact hash
// table (each key's lowest file index) and an emit pass into owner ranges;
// the resolve is a hash table with 64-bit atomicMin per key.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "dist_dedup.h"

namespace sdcas {

namespace {

constexpr uint32_t TB = 256;
constexpr int64_t kLinkDeferred = INT64_MIN + 1;  // SDCAS_LINK_DEFERRED
inline uint32_t blocks(uint32_t n) { return (n + TB - 1) / TB; }
constexpr uint32_t kIdxEmpty = 0xFFFFFFFFu;
constexpr uint32_t kCountShards = 64;  // the apply's count pairs (a workgroup adds to blockIdx % 64)

// ---- the steps' positions (see dist_dedup.h, "the job's steps") -------------------

// The re-read list's coarse index (round 6): every keyed file counts the
// re-reads below two ordinals (its own and its key's first), a binary search
// of log2(re-reads) dependent loads each — with C5's 0.2 % I/O errors over 50 M
// files, ~20 per file, the apply 0.80 -> 1.35 ms. k_rr_index counts the
// re-reads below each of kRrBuckets ordinals b << s (s: the least shift that
// puts the last re-read below kRrBuckets << s), so a search covers one
// bucket's entries. ridx: [0] the stamp of the plan it was built for (the
// plan's word kPlanIndex holds the same; an apply uses the index only when
// the two agree and are nonzero, so a plan rebuilt elsewhere or never indexed
// falls back to the full search), [1] s, then kRrBuckets + 1 u32 counts.
constexpr uint32_t kRrBuckets = 4096;
constexpr uint32_t kRrWords = 2 + (kRrBuckets + 2) / 2;
constexpr uint32_t kRrMin = 64;  // shorter lists: the plain search is as short

struct PlanView {
  const uint64_t* rr;  // re-read ordinals, ascending (null: none)
  uint64_t nrr, limit;
  uint64_t loop, loop_reads;  // a row read by every step left (~0: none)
  const uint32_t* ri;         // the coarse index's counts (null: none)
  uint32_t rs;                // its shift
};

__device__ __forceinline__ PlanView plan_view(const uint64_t* plan, const uint64_t* ridx = nullptr) {
  if (!plan) return PlanView{nullptr, 0, ~0ull, ~0ull, 0, nullptr, 0};
  PlanView v{plan + kPlanHeader, plan[kPlanRereads], plan[kPlanLimit], plan[kPlanLoop], plan[kPlanLoopReads],
             nullptr, 0};
  const uint64_t stamp = plan[kPlanIndex];
  if (ridx && stamp != 0 && ridx[0] == stamp) {
    v.ri = reinterpret_cast<const uint32_t*>(ridx + 2);
    v.rs = (uint32_t)ridx[1];
  }
  return v;
}

// re-read ordinals below x
__device__ __forceinline__ uint64_t rr_below(const PlanView& pv, uint64_t x) {
  uint64_t lo = 0, hi = pv.nrr;
  if (pv.ri) {
    const uint64_t b = x >> pv.rs;
    if (b >= kRrBuckets) return pv.nrr;  // x >= kRrBuckets << s > the last re-read
    lo = pv.ri[b];
    hi = pv.ri[b + 1];
  }
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (pv.rr[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

enum : int { kFileKeyed = 0, kFileNoKey = 1, kFileDropped = 2 };

// identifier_job_step's outcome for one file over the job's steps
// (mod.rs:125-141, 202-254): r = the key's answer for a keyed file (-(db+1)
// existing Object, else the key's lowest ordinal)
__device__ __forceinline__ int64_t step_link(int kind, int64_t me, int64_t r, uint64_t cs, const PlanView& pv,
                                             unsigned long long& c, unsigned long long& l) {
  if ((uint64_t)me >= pv.loop) {  // the repeated row, and the rows no step reaches after it
    if ((uint64_t)me > pv.loop) return kLinkDeferred;
    if (kind == kFileDropped) return INT64_MIN;
    c += pv.loop_reads;  // a stays row: no cas_id, an Object per read
    return me;
  }
  uint64_t pos = (uint64_t)me;
  bool twice = false;
  if (pv.rr) {
    const uint64_t b = rr_below(pv, (uint64_t)me);
    pos += b;
    twice = b < pv.nrr && pv.rr[b] == (uint64_t)me;
  }
  if (pos >= pv.limit) return kLinkDeferred;  // no step the job runs reaches it
  if (kind == kFileDropped) return INT64_MIN;
  if (kind == kFileNoKey) {  // mod.rs:246-254: its own Object, per step that reads it
    c += 1 + (twice && pos + 1 < pv.limit ? 1 : 0);
    return me;
  }
  if (r < 0) {
    l += 1;
    return r;
  }
  // created in the key's first step: a file of that step creates its own
  // Object (mod.rs:246-254), files of later steps link to the first one
  const uint64_t rpos = pv.rr ? (uint64_t)r + rr_below(pv, (uint64_t)r) : (uint64_t)r;
  // the same step? (32-bit division when everything fits: a 64-bit one is a
  // long software sequence, paid by every keyed file)
  const bool same = ((pos | rpos | cs) >> 32) == 0 ? (uint32_t)pos / (uint32_t)cs == (uint32_t)rpos / (uint32_t)cs
                                                   : pos / cs == rpos / cs;
  if (same) {
    c += 1;
    return me;
  }
  l += 1;
  return r;
}

__device__ __forceinline__ void add_counts(unsigned long long c, unsigned long long l, unsigned long long* sc,
                                           unsigned long long* counts) {
  for (int off = 32; off > 0; off >>= 1) {
    c += __shfl_down(c, off);
    l += __shfl_down(l, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&sc[0], c);
    atomicAdd(&sc[1], l);
  }
  __syncthreads();
  if (threadIdx.x == 0 && counts) {
    atomicAdd(&counts[0], sc[0]);
    atomicAdd(&counts[1], sc[1]);
  }
}

__global__ void k_dd_apply(const uint64_t* __restrict__ ids, const uint32_t* __restrict__ slot, uint32_t n,
                           const int64_t* __restrict__ result, uint64_t cs, const uint64_t* __restrict__ plan,
                           int64_t* __restrict__ link, unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  const PlanView pv = plan_view(plan);
  // grid-stride over a bounded grid: one global atomic pair per workgroup
  // (thousands of workgroups adding to one address serialise in L2)
  unsigned long long c = 0, l = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = slot[i];
    const int kind = s == kSlotDropped ? kFileDropped : s == kSlotNoKey ? kFileNoKey : kFileKeyed;
    link[i] = step_link(kind, (int64_t)ids[i], kind == kFileKeyed ? result[s] : 0, cs, pv, c, l);
  }
  add_counts(c, l, sc, counts);
}

// k_dd_apply with R files per thread over a full grid, the counts into
// kCountShards pairs (as k_solo_apply_r; folded by k_counts_fold)
template <uint32_t R>
__global__ void __launch_bounds__(TB) k_dd_apply_r(const uint64_t* __restrict__ ids,
                                                   const uint32_t* __restrict__ slot, uint32_t n,
                                                   const int64_t* __restrict__ result, uint64_t cs,
                                                   const uint64_t* __restrict__ plan, int64_t* __restrict__ link,
                                                   unsigned long long* __restrict__ shard,
                                                   const uint64_t* __restrict__ ridx) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  const PlanView pv = plan_view(plan, ridx);
  const uint64_t i0 = (uint64_t)blockIdx.x * TB * R + threadIdx.x;
  uint32_t s[R];
  int64_t me[R], r[R];
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    s[k] = i < n ? slot[i] : kSlotDropped;
    me[k] = i < n ? (int64_t)ids[i] : 0;
  }
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) r[k] = s[k] < kSlotDropped && s[k] != kSlotNoKey ? result[s[k]] : 0;
  unsigned long long c = 0, l = 0;
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    if (i >= n) continue;
    const int kind = s[k] == kSlotDropped ? kFileDropped : s[k] == kSlotNoKey ? kFileNoKey : kFileKeyed;
    link[i] = step_link(kind, me[k], r[k], cs, pv, c, l);
  }
  add_counts(c, l, sc, shard ? shard + 2 * (blockIdx.x % kCountShards) : nullptr);
}

// Stays rows — their step leaves them orphans (file_identifier_job.rs:258-264)
// — in order (what hipcub::DeviceSelect::If gave, without its look-back
// scan): (1) each workgroup counts its 4096 rows' stays, (2) one
// workgroup turns the counts into offsets and writes the total, (3) only the
// workgroups that hold a stays row write their indices, in order. A batch
// with none (C3 / C5: every file has a key) costs two streaming passes over
// the flags and an empty third launch. C5: ~50 us -> ~15 us per call.
constexpr uint32_t kStayWG = 256, kStayR = 16, kStayPer = kStayWG * kStayR;

__device__ __forceinline__ bool stays_row(const uint8_t* __restrict__ has_key, const int32_t* __restrict__ status,
                                          uint64_t i) {
  return (status && status[i] != 0) || (has_key && !has_key[i]);
}

__global__ void __launch_bounds__(kStayWG) k_stays_count(const uint8_t* __restrict__ has_key,
                                                         const int32_t* __restrict__ status, uint32_t n,
                                                         uint32_t* __restrict__ bcnt) {
  __shared__ uint32_t ws[kStayWG / 64];
  const uint64_t lo = (uint64_t)blockIdx.x * kStayPer;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t r = 0; r < kStayR; ++r) {
    const uint64_t i = lo + r * kStayWG + threadIdx.x;
    c += i < n && stays_row(has_key, status, i);
  }
#pragma unroll
  for (uint32_t d = 32; d; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// one workgroup: bcnt[b] <- its exclusive prefix; *total <- the sum
__global__ void __launch_bounds__(1024) k_stays_scan(uint32_t* __restrict__ bcnt, uint32_t nb,
                                                     uint32_t* __restrict__ total) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += 1024) {
    const uint32_t i = base + tid;
    const uint32_t v = i < nb ? bcnt[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += ws[w];
    if (i < nb) bcnt[i] = before + inc - v;
    __syncthreads();
    if (tid == 1023) carry = before + inc;
    __syncthreads();
  }
  if (tid == 0) *total = carry;
}

__global__ void __launch_bounds__(kStayWG) k_stays_write(const uint8_t* __restrict__ has_key,
                                                         const int32_t* __restrict__ status, uint32_t n,
                                                         const uint32_t* __restrict__ boff,
                                                         const uint32_t* __restrict__ total,
                                                         uint32_t* __restrict__ out) {
  __shared__ uint32_t ws[kStayWG / 64];
  const uint32_t b = blockIdx.x;
  const uint32_t mine = (b + 1 < gridDim.x ? boff[b + 1] : *total) - boff[b];
  if (mine == 0) return;  // uniform over the workgroup
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lo = (uint64_t)b * kStayPer;
  uint32_t run = boff[b];
#pragma unroll 1
  for (uint32_t r = 0; r < kStayR; ++r) {
    const uint64_t i = lo + r * kStayWG + tid;
    const bool f = i < n && stays_row(has_key, status, i);
    const uint64_t bal = __ballot(f);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (lane == 0) ws[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = run, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kStayWG / 64; ++w) {
      if (w < wave) before += ws[w];
      all += ws[w];
    }
    __syncthreads();
    if (f) out[before + below] = (uint32_t)i;
    run += all;
  }
}

// the stays rows of [0, n) in order into w.stay_idx, their count into w.nstay
static hipError_t select_stays(DistWs& w, const uint8_t* has_key, const int32_t* status, uint32_t n,
                               hipStream_t st) {
  hipError_t e;
  const uint32_t nb = (n + kStayPer - 1) / kStayPer;
  if ((e = w.stay_idx.ensure(n)) || (e = w.stay_cnt.ensure(nb + 1))) return e;
  hipLaunchKernelGGL(k_stays_count, dim3(nb), dim3(kStayWG), 0, st, has_key, status, n, w.stay_cnt.p);
  hipLaunchKernelGGL(k_stays_scan, dim3(1), dim3(1024), 0, st, w.stay_cnt.p, nb, w.nstay.p);
  hipLaunchKernelGGL(k_stays_write, dim3(nb), dim3(kStayWG), 0, st, has_key, status, n, w.stay_cnt.p, w.nstay.p,
                     w.stay_idx.p);
  return hipGetLastError();
}

__global__ void k_stays_gather(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ m_p,
                               const uint64_t* __restrict__ ids, uint32_t cap, uint64_t* __restrict__ out,
                               int64_t* __restrict__ count) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t m = *m_p;
  if (j == 0 && count) *count = (int64_t)m;
  if (j < cap) out[j] = j < m ? ids[idx[j]] : ~0ull;
}

// One wave walks the stays ordinals in order. Ordinal p ends a step — and is
// read again by the next — when its position p + r is the step's last,
// (p + r) % cs == cs - 1, r being the re-reads before it; the job's last
// orphan is never read again by a step inside the batch. 64 candidates at a
// time: the first lane whose test holds is a re-read; the lanes after it
// test again with r + 1. Two cases repeat a row for every step left (the
// reference re-reads it while its cursor stays put): chunks of one row
// (each step's only row is its last), and steps the job may still run after
// its last row when that row stays an orphan (only with max_steps above
// what the rows need).
__global__ __launch_bounds__(64) void k_plan_walk(const uint64_t* __restrict__ stays, const uint32_t* __restrict__ idx,
                                                  const uint64_t* __restrict__ ids, uint32_t cap,
                                                  const uint32_t* __restrict__ m_p, uint64_t n_total, uint64_t cs,
                                                  uint64_t max_steps, uint32_t more, uint64_t* __restrict__ plan,
                                                  const uint32_t* __restrict__ tile_cnt = nullptr, uint32_t ntiles = 0) {
  const int lane = (int)threadIdx.x;
  uint32_t m;
  if (tile_cnt) {  // the tiled insert's per-tile stays counts: their sum
    uint32_t s = 0;
    for (uint32_t t = (uint32_t)lane; t < ntiles; t += 64) s += tile_cnt[t];
#pragma unroll
    for (int d = 32; d; d >>= 1) s += __shfl_xor(s, d);
    m = min(s, cap);
  } else {
    m = m_p ? min(*m_p, cap) : cap;
  }
  uint64_t* rr = plan + kPlanHeader;
  uint64_t r = 0;
  uint64_t first = ~0ull, last_stay = ~0ull;  // smallest / largest valid stays ordinal
  // kWalkU batches of 64 ordinals are loaded together (a batch's ordinal is
  // two dependent loads, ids[idx[j]]: one memory round trip per 64 * kWalkU
  // ordinals) and their residues p % cs computed together; then each batch
  // is walked in order. Between two re-reads r is constant, so the next
  // re-read is the first candidate whose residue is the target
  // (cs - 1 - r) mod cs: a batch without it costs one compare and one
  // ballot, and each re-read moves the target down by one.
  constexpr uint32_t kWalkU = 16;
  const bool small = cs < (1ull << 32);
  uint64_t target = cs - 1;  // (cs - 1 - r) mod cs
  bool done = false;
  for (uint32_t base = 0; base < m && !done; base += 64 * kWalkU) {
    uint64_t pv[kWalkU], pm[kWalkU];
#pragma unroll
    for (uint32_t u = 0; u < kWalkU; ++u) {
      const uint32_t j = base + 64 * u + (uint32_t)lane;
      pv[u] = j < m ? (idx ? ids[idx[j]] : stays[j]) : ~0ull;
    }
    uint32_t pad = 0;  // batches holding a padding entry (sorted: padding from there on)
#pragma unroll
    for (uint32_t u = 0; u < kWalkU; ++u) {
      const uint32_t j = base + 64 * u + (uint32_t)lane;
      const uint64_t p = pv[u];
      const bool cand = cs > 1 && n_total && p < n_total - 1;  // the job's last orphan is never re-read
      pm[u] = !cand ? ~0ull : small && p < (1ull << 32) ? (uint64_t)((uint32_t)p % (uint32_t)cs) : p % cs;
      if (__ballot(j < m && p >= n_total)) pad |= 1u << u;
    }
    // the valid range: the first entry of all, the last before padding or m
    const uint64_t p00 = __shfl(pv[0], 0);
    if (base == 0 && m && p00 < n_total) first = p00;
    // every batch of the group is walked (no early exit: the register
    // arrays must stay fully unrolled); batches past the end or past padding
    // hold no candidate and move nothing
    const uint32_t nu = min(kWalkU, (m - base + 63) / 64);
    const uint32_t upad = pad ? (uint32_t)__builtin_ctz(pad) : kWalkU;  // first batch with padding
    const uint32_t ulast = min(nu - 1, upad);                          // the last batch holding valid entries
#pragma unroll
    for (uint32_t u = 0; u < kWalkU; ++u) {
      if (u == ulast) {
        const uint32_t j = base + 64 * u + (uint32_t)lane;
        const unsigned long long inm = __ballot(j < m && pv[u] < n_total);
        if (inm) last_stay = __shfl(pv[u], 63 - __clzll((long long)inm));
        else if (u) last_stay = __shfl(pv[u - 1], 63);
      }
      unsigned long long mask = __ballot(pm[u] == target);
      while (mask) {
        const int f = __ffsll((long long)mask) - 1;
        if (lane == f) rr[r] = pv[u];
        ++r;
        target = target == 0 ? cs - 1 : target - 1;
        mask = __ballot(pm[u] == target && lane > f);
      }
    }
    if (pad || base + 64 * kWalkU >= m) done = true;
  }
  if (lane == 0) {
    const uint64_t T = max_steps ? max_steps : (n_total + cs - 1) / cs;
    uint64_t loop = ~0ull, reads = 0, steps, limit, rows = 0;
    if (cs == 1 && first != ~0ull && first < T) {
      // one-row steps: the first stays row is read by every step from its own on
      loop = first;
      reads = T - first;
      steps = T;
      limit = first;  // positions below the loop row are ordinary steps
      rows = first + 1;
    } else {
      const uint64_t E = n_total + r;  // positions the rows take
      const uint64_t avail = more ? E / cs : (E + cs - 1) / cs;
      steps = avail < T ? avail : T;
      limit = steps * cs;
      if (steps) {
        // the ordinal at the last position run: P minus the second reads at or before it
        const uint64_t P = (limit < E ? limit : E) - 1;
        uint64_t lo = 0, hi = r;  // second reads sit at rr[k] + k + 1
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (rr[mid] + mid + 1 <= P) lo = mid + 1;
          else hi = mid;
        }
        rows = P - lo + 1;
      }
      if (!more && T > avail && n_total && last_stay == n_total - 1) {
        loop = n_total - 1;  // steps left after the last row: each reads it again
        reads = 1 + (T - avail);
        steps = T;
      }
    }
    plan[kPlanLimit] = limit;
    plan[kPlanRereads] = r;
    plan[kPlanSteps] = steps;
    plan[kPlanRows] = rows;
    plan[kPlanNTotal] = n_total;
    plan[kPlanChunk] = cs;
    plan[kPlanLoop] = loop;
    plan[kPlanLoopReads] = reads;
    uint64_t run = 0;  // re-reads whose second read is a step the job runs
    {
      uint64_t lo = 0, hi = r;
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (rr[mid] + mid + 1 < limit) lo = mid + 1;
        else hi = mid;
      }
      run = lo;
    }
    plan[kPlanRereadsRun] = run + (loop != ~0ull ? reads - 1 : 0);
    plan[kPlanIndex] = plan[10] = plan[11] = 0;
  }
}

// the coarse index of plan's re-read list (above), one thread per count;
// lists shorter than kRrMin are left unindexed (the plan's stamp stays 0)
__global__ void k_rr_index(uint64_t* __restrict__ plan, uint64_t* __restrict__ ridx, uint64_t stamp) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nrr = plan[kPlanRereads];
  if (nrr < kRrMin || b > kRrBuckets) return;
  const uint64_t* rr = plan + kPlanHeader;
  const uint64_t top = rr[nrr - 1];
  uint32_t s = 0;
  while ((top >> s) >= kRrBuckets) ++s;
  auto* cnt = reinterpret_cast<uint32_t*>(ridx + 2);
  if (b == kRrBuckets) {
    cnt[b] = (uint32_t)nrr;
  } else {
    const uint64_t x = (uint64_t)b << s;  // b < 2^12, s <= 52: no overflow
    uint64_t lo = 0, hi = nrr;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (rr[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    cnt[b] = (uint32_t)lo;
  }
  if (b == 0) {
    ridx[0] = stamp;
    ridx[1] = s;
    plan[kPlanIndex] = stamp;
  }
}

// SDCAS_RR_INDEX=0: the applies search the whole re-read list (A/B), read per call
static bool rr_index_enabled() {
  const char* v = getenv("SDCAS_RR_INDEX");
  return !(v && strcmp(v, "0") == 0);
}

// index plan's re-read list for the applies of this workspace (after the
// walk that wrote it, on the same stream)
static hipError_t rr_index(DistWs& w, uint64_t* plan, hipStream_t st) {
  if (!rr_index_enabled()) return hipSuccess;
  static std::atomic<uint64_t> stamps{0};
  hipError_t e;
  if ((e = w.ridx.ensure(kRrWords))) return e;
  hipLaunchKernelGGL(k_rr_index, dim3((kRrBuckets + TB) / TB), dim3(TB), 0, st, plan, w.ridx.p, ++stamps);
  return hipGetLastError();
}

}  // namespace

void DistWs::release() {
  idx_a.release(); idx_b.release(); starts.release(); ocnt.release(); tkey.release(); tmin.release();
  tpos.release(); stay_idx.release(); nstay.release(); stay_cnt.release(); plan.release(); stay_sorted.release();
  bitmap.release(); flag.release(); shard.release(); ridx.release();
  shard_dirty = false;
}

// the combine up to its device outputs: rec, slot, w.starts[0..world] (n > 0)
// (defined with the bucket combine below)
static hipError_t combine_core(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                               const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                               hipStream_t st);

hipError_t dd_combine(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                      const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                      uint64_t* h_starts, uint64_t* h_u, hipStream_t st) {
  hipError_t e;
  if (n == 0) {
    for (uint32_t r = 0; r <= world; ++r) h_starts[r] = 0;
    *h_u = 0;
    return hipSuccess;
  }
  if ((e = combine_core(w, keys, has_key, status, ids, n, world, rec, slot, st))) return e;
  uint32_t hs[1025];
  uint32_t* hp = world + 1 <= 1025 ? hs : new uint32_t[world + 1];
  e = hipMemcpyAsync(hp, w.starts.p, sizeof(uint32_t) * (world + 1), hipMemcpyDeviceToHost, st);
  if (!e) e = hipStreamSynchronize(st);
  if (!e) {
    for (uint32_t r = 0; r <= world; ++r) h_starts[r] = hp[r];
    *h_u = hp[world];
  }
  if (hp != hs) delete[] hp;
  if (e) return e;
  return hipGetLastError();
}

hipError_t dd_combine_dev(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                          const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                          uint32_t* d_starts, hipStream_t st) {
  if (n == 0) return hipMemsetAsync(d_starts, 0, sizeof(uint32_t) * (world + 1), st);
  hipError_t e;
  if ((e = combine_core(w, keys, has_key, status, ids, n, world, rec, slot, st))) return e;
  // w.starts is the context's scratch: the next combine on it rewrites it
  return hipMemcpyAsync(d_starts, w.starts.p, sizeof(uint32_t) * (world + 1), hipMemcpyDeviceToDevice, st);
}

// ---- the combine into fixed-capacity owner buckets (no host sync) ---------------
//
// RCCL's all-to-all through torch needs every split size on the host, i.e.
// a synchronisation to learn how many records go to each owner. With buckets
// of a capacity the host picks in advance (dist_dedup.py: from the file
// count and the previous call's fill), every exchange has equal splits and
// nothing waits for the host; a bucket that would overflow raises a flag
// that travels with the final counts, and the caller then reruns the exact
// path. Record u of owner r goes to send[r * cap + (u - starts[r])].

// (defined with the world-of-one path below)
__global__ void k_solo_insert_idx(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ ekeys, uint32_t n,
                                  const uint8_t* __restrict__ has_key, const int32_t* __restrict__ status,
                                  const uint64_t* __restrict__ eids, uint32_t count, uint32_t base,
                                  uint32_t* __restrict__ tab, unsigned long long* __restrict__ emin, uint32_t mask,
                                  uint32_t shift, uint32_t* __restrict__ pos, uint32_t* __restrict__ stay_cnt,
                                  uint32_t* __restrict__ noncontig, uint32_t sticky, uint32_t plain = 0);

// ---- the combine through a hash table ----------------------------------------------
//
// One (key, min ordinal) record per distinct key in its owner's bucket (or,
// exact layout, its owner's range), each file's record position — from the
// compact table of the world-of-one path: insert (the lowest file
// index per key), then each key's lowest file emits the record into its
// owner's bucket at a position taken per workgroup (LDS counters, one global
// atomicAdd per owner present), then every file reads its key's position. No
// sort; the records of a bucket are in no particular order, which neither the
// exchange nor the owner's resolve needs.
constexpr uint32_t kEmitR = 16;           // files per thread: 4096 per workgroup
constexpr uint32_t kEmitMaxWorld = 1024;  // owners a workgroup counts in LDS (more: one global atomic per record)

// base null: the buckets — record p of owner r at r * cap + p, p < cap (a
// fuller owner raises *overflow); base set: the exact layout — owner r's
// records from base[r] on, no capacity. count_only: each owner's record
// count added to fill[], nothing written (the exact layout's first pass).
__global__ void __launch_bounds__(TB) k_cb_emit(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ ids,
                                                uint32_t n, const uint32_t* __restrict__ pos,
                                                const uint32_t* __restrict__ tab, uint32_t world, uint32_t cap,
                                                const uint32_t* __restrict__ base, uint32_t count_only,
                                                uint32_t* __restrict__ fill, uint64_t* __restrict__ send,
                                                uint32_t* __restrict__ bpos, uint32_t* __restrict__ overflow) {
  // positions are taken per workgroup: LDS counters per owner, then ONE
  // global atomicAdd per owner present in the workgroup (a wave-level
  // aggregate left ~ 8 atomics per wave on `world` addresses: 7.5 ms for
  // C5's 6.25 M files at world 8, profiles/r04_dedup_world.json)
  __shared__ uint32_t s_cnt[kEmitMaxWorld], s_base[kEmitMaxWorld];
  const bool lds = world <= kEmitMaxWorld;
  for (uint32_t t = threadIdx.x; lds && t < world; t += TB) s_cnt[t] = 0;
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * TB * kEmitR + threadIdx.x;
  uint32_t h[kEmitR], lp[kEmitR], rr[kEmitR];
#pragma unroll
  for (uint32_t k = 0; k < kEmitR; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    h[k] = i < n ? pos[i] : kSlotDropped;
  }
#pragma unroll
  for (uint32_t k = 0; k < kEmitR; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    // the key's lowest file carries its record
    lp[k] = h[k] < kSlotDropped && tab[h[k]] == (uint32_t)i ? 0u : ~0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kEmitR; ++k) {
    rr[k] = 0;
    if (lp[k] == ~0u) continue;
    rr[k] = dd_owner(keys[i0 + (uint64_t)k * TB], world);
    lp[k] = lds ? atomicAdd(&s_cnt[rr[k]], 1u) : atomicAdd(&fill[rr[k]], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; lds && t < world; t += TB)
    s_base[t] = s_cnt[t] ? atomicAdd(&fill[t], s_cnt[t]) : 0u;
  if (count_only) return;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kEmitR; ++k) {
    if (lp[k] == ~0u) continue;
    const uint64_t i = i0 + (uint64_t)k * TB;
    const uint32_t p = (lds ? s_base[rr[k]] : 0u) + lp[k];
    if (!base && p >= cap) {
      atomicOr(overflow, 1u);  // the caller reruns the exact stages
      bpos[i] = kSlotNoKey;
      continue;
    }
    const uint64_t q = base ? (uint64_t)base[rr[k]] + p : (uint64_t)rr[k] * cap + p;
    send[2 * q] = keys[i];
    send[2 * q + 1] = ids[i];
    bpos[i] = (uint32_t)q;
  }
}

// ---- round 6: the bucket combine without a rank-side hash table -------------------
//
// The bucket protocol's owner resolve takes the minimum over every record of
// a key (records of one key from several ranks, and now from several tiles
// of one rank), so the rank side need not reduce to one record per key: each
// workgroup pre-aggregates its own tile of kTileN files in LDS (the Zipf
// head's copies in a tile collapse to one record) and sends one (key, lowest
// ordinal in the tile) record per distinct key of the tile to its owner's
// bucket. One pass over the files, all of its probing in LDS, instead of the
// global table's clear, insert, emit and slot passes (C5 at world 8: 0.50 ms
// of one rank's 0.89 ms), for more records in the exchange and at the owner.
constexpr uint32_t kTileR = 8, kTileN = TB * kTileR;  // 2048 files per workgroup
constexpr uint32_t kTileSlots = 2 * kTileN;            // the LDS table's slots (local indices)

__device__ __forceinline__ uint32_t tile_hash(uint64_t key) {
  return ((uint32_t)(key ^ (key >> 32)) * 0x9E3779B1u) >> (32 - 12);  // 12 bits: kTileSlots
}
static_assert(kTileSlots == 1u << 12, "tile_hash takes 12 bits");

// fill[0..world] and the overflow flag zeroed in one launch (two memsets
// were two). The owners' valid counts come from k_cb_counts after the tiles:
// a last-workgroup-writes-them pattern measured 113 -> 540 us for the tile
// kernel on C5 at world 8 — every workgroup's device-scope release fence
// writes back its XCD's L2 (profiles/r06_dedup_world.json)
__global__ void k_cb_prep(uint32_t* __restrict__ fill, uint32_t world, uint32_t* __restrict__ overflow) {
  for (uint32_t t = threadIdx.x; t <= world; t += blockDim.x) fill[t] = 0;
  if (threadIdx.x == 0) *overflow = 0;
}

__global__ void __launch_bounds__(TB) k_cb_tile(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ has_key,
                                                const int32_t* __restrict__ status, const uint64_t* __restrict__ ids,
                                                uint32_t n, uint32_t world, uint32_t cap, uint32_t* __restrict__ fill,
                                                uint64_t* __restrict__ send, uint32_t* __restrict__ slot,
                                                uint32_t* __restrict__ overflow) {
  __shared__ uint64_t skey[kTileN];
  __shared__ uint32_t tab[kTileSlots];
  __shared__ uint32_t spos[kTileN];
  __shared__ uint32_t s_cnt[kEmitMaxWorld], s_base[kEmitMaxWorld];
  const uint32_t tid = threadIdx.x;
  const bool lds = world <= kEmitMaxWorld;
  for (uint32_t t = tid; lds && t < world; t += TB) s_cnt[t] = 0;
  for (uint32_t t = tid; t < kTileSlots; t += TB) tab[t] = kIdxEmpty;
  const uint64_t tile0 = (uint64_t)blockIdx.x * kTileN;
  // code: the file's LDS slot (keyed), or its slot code (no key / dropped)
  uint32_t code[kTileR];
#pragma unroll
  for (uint32_t k = 0; k < kTileR; ++k) {
    const uint32_t t = k * TB + tid;
    const uint64_t i = tile0 + t;
    code[k] = kSlotDropped;
    if (i < n) {
      const bool ok = status == nullptr || status[i] == 0;  // mod.rs:125-141
      const bool has = has_key == nullptr || has_key[i];    // mod.rs:83-86
      skey[t] = keys[i];
      code[k] = !ok ? kSlotDropped : !has ? kSlotNoKey : 0u;
    }
  }
  __syncthreads();
  // the tile's table: each key's slot holds its lowest local index (local
  // order is ordinal order), the key read back from skey
#pragma unroll
  for (uint32_t k = 0; k < kTileR; ++k) {
    if (code[k] != 0u) continue;
    const uint32_t t = k * TB + tid;
    const uint64_t key = skey[t];
    uint32_t h = tile_hash(key);
    for (;;) {
      uint32_t cur = tab[h];
      if (cur == kIdxEmpty) {
        const uint32_t prev = atomicCAS(&tab[h], kIdxEmpty, t);
        if (prev == kIdxEmpty) break;
        cur = prev;
      }
      if (skey[cur] == key) {
        if (cur > t) atomicMin(&tab[h], t);
        break;
      }
      h = (h + 1) & (kTileSlots - 1);
    }
    code[k] = h;
  }
  __syncthreads();
  // each key's lowest file of the tile carries the record: a position in its
  // owner's bucket per workgroup (LDS counters, one global atomic per owner)
  uint32_t lp[kTileR], own[kTileR];
#pragma unroll
  for (uint32_t k = 0; k < kTileR; ++k) {
    const uint32_t t = k * TB + tid;
    lp[k] = ~0u;
    own[k] = 0;
    if (code[k] < kTileSlots && tab[code[k]] == t) {
      own[k] = dd_owner(skey[t], world);
      lp[k] = lds ? atomicAdd(&s_cnt[own[k]], 1u) : atomicAdd(&fill[own[k]], 1u);
    }
  }
  __syncthreads();
  for (uint32_t t = tid; lds && t < world; t += TB) s_base[t] = s_cnt[t] ? atomicAdd(&fill[t], s_cnt[t]) : 0u;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kTileR; ++k) {
    if (lp[k] == ~0u) continue;
    const uint32_t t = k * TB + tid;
    const uint32_t p = (lds ? s_base[own[k]] : 0u) + lp[k];
    if (p >= cap) {
      atomicOr(overflow, 1u);  // the caller reruns the exact stages
      spos[t] = kSlotNoKey;
      continue;
    }
    const uint64_t q = (uint64_t)own[k] * cap + p;
    send[2 * q] = skey[t];
    send[2 * q + 1] = ids[tile0 + t];
    spos[t] = (uint32_t)q;
  }
  if (!slot) return;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kTileR; ++k) {
    const uint64_t i = tile0 + k * TB + tid;
    if (i < n) slot[i] = code[k] < kTileSlots ? spos[tab[code[k]]] : code[k];
  }
}

// one workgroup: starts[0..world] = the exclusive prefix of cnt[0..world)
__global__ void __launch_bounds__(1024) k_owner_starts(const uint32_t* __restrict__ cnt, uint32_t world,
                                                       uint32_t* __restrict__ starts) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < world; b += 1024) {
    const uint32_t i = b + tid;
    const uint32_t v = i < world ? cnt[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += ws[w];
    if (i < world) starts[i] = before + inc - v;
    __syncthreads();
    if (tid == 1023) carry = before + inc;
    __syncthreads();
  }
  if (tid == 0) starts[world] = carry;
}

__global__ void k_cb_slot(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ tab,
                          const uint32_t* __restrict__ bpos, uint32_t n, uint32_t* __restrict__ slot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t h = pos[i];
  slot[i] = h >= kSlotDropped ? h : bpos[tab[h]];
}

__global__ void k_cb_counts(const uint32_t* __restrict__ fill, uint32_t world, uint32_t cap,
                            int64_t* __restrict__ counts) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < world) counts[r] = fill[r] < cap ? fill[r] : cap;
}

// ---- resolve: per-key minima in an open-addressing hash table -----------------
//
// The owner needs, per key, the minimum DB index over the existing Objects'
// records and the minimum orphan ordinal over the files' records. Both are
// associative minima, so every record is inserted (linear probing, 64-bit
// CAS on the key) and min-folded into its entry (64-bit atomicMin); each file
// record then reads its entry. Three streaming passes over the records and
// no sort. The all-ones key (a legal cas key) owns the extra entry at `cap`.
constexpr uint64_t kEmptyKey = ~0ull;

// Home slot = the key bits just below the 12 that chose the owner rank
// (dd_owner; cas keys are BLAKE3 output, uniform): within one owner's share
// the table is ordered like the keys, so the key-sorted runs the owner
// receives (one per source rank) insert into neighbouring lines instead of
// scattering one line per record. (The owner bits themselves would crowd an
// owner's keys into 1/world of the table: at 8 ranks the probe runs grew
// until a resolve took 640 ms instead of under 1 ms.) A slot is read before
// it is CAS'd, and an entry's minimum before it is atomicMin'd (both only
// ever decrease from all-ones).
constexpr uint32_t kOwnerBits = 12;
__device__ __forceinline__ uint32_t ht_find(unsigned long long* __restrict__ tkey, uint64_t key, uint32_t mask,
                                            uint32_t shift) {
  if (key == kEmptyKey) return mask + 1;
  uint32_t h = (uint32_t)((key << kOwnerBits) >> shift) & mask;
  for (;;) {
    const unsigned long long cur = __hip_atomic_load(&tkey[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return h;
    if (cur == kEmptyKey) {
      const unsigned long long prev = atomicCAS(&tkey[h], (unsigned long long)kEmptyKey, (unsigned long long)key);
      if (prev == kEmptyKey || prev == key) return h;
    }
    h = (h + 1) & mask;
  }
}

// rec[2p] = key, rec[2p+1] = value; min-fold value into tmin[2 * entry + side]
__global__ void k_ht_insert(const uint64_t* __restrict__ rec, uint32_t n, unsigned long long* __restrict__ tkey,
                            unsigned long long* __restrict__ tmin, uint32_t mask, uint32_t shift, uint32_t side,
                            uint32_t* __restrict__ pos_out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t h = ht_find(tkey, rec[2 * (uint64_t)p], mask, shift);
  const unsigned long long v = rec[2 * (uint64_t)p + 1];
  unsigned long long* m = &tmin[2 * (uint64_t)h + side];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  if (pos_out) pos_out[p] = h;
}

__global__ void k_ht_answer(const uint32_t* __restrict__ pos, uint32_t nf, const uint64_t* __restrict__ tmin,
                            int64_t* __restrict__ result) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nf) return;
  const uint32_t h = pos[p];
  const uint64_t e = tmin[2 * (uint64_t)h + 1];
  // mod.rs:202-238: the first existing Object carrying the key; else the
  // key's first file (mod.rs:246-254)
  result[p] = e != ~0ull ? -(int64_t)e - 1 : (int64_t)tmin[2 * (uint64_t)h];
}

hipError_t dd_resolve(DistWs& w, const uint64_t* frec, uint32_t nf, const uint64_t* erec, uint32_t ne,
                      int64_t* result, hipStream_t st) {
  hipError_t e;
  if (nf == 0) return hipSuccess;  // nothing asks: existing records alone answer no one
  uint64_t cap = 1024;
  while (cap < 2 * ((uint64_t)nf + ne)) cap <<= 1;
  if (cap > (1ull << 31)) return hipErrorInvalidValue;
  if ((e = w.tkey.ensure(cap + 1)) || (e = w.tmin.ensure(2 * (cap + 1))) || (e = w.tpos.ensure(nf))) return e;
  const uint32_t mask = (uint32_t)(cap - 1);
  const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(cap);
  if ((e = hipMemsetAsync(w.tkey.p, 0xFF, sizeof(uint64_t) * (cap + 1), st)) ||
      (e = hipMemsetAsync(w.tmin.p, 0xFF, sizeof(uint64_t) * 2 * (cap + 1), st)))
    return e;
  auto* tk = reinterpret_cast<unsigned long long*>(w.tkey.p);
  auto* tm = reinterpret_cast<unsigned long long*>(w.tmin.p);
  if (ne) hipLaunchKernelGGL(k_ht_insert, dim3(blocks(ne)), dim3(TB), 0, st, erec, ne, tk, tm, mask, shift, 1u, nullptr);
  hipLaunchKernelGGL(k_ht_insert, dim3(blocks(nf)), dim3(TB), 0, st, frec, nf, tk, tm, mask, shift, 0u, w.tpos.p);
  hipLaunchKernelGGL(k_ht_answer, dim3(blocks(nf)), dim3(TB), 0, st, w.tpos.p, nf, w.tmin.p, result);
  return hipGetLastError();
}

// Resolve over received buckets: world buckets of `cap` records each, bucket
// r holding counts[r] valid records (the rest is padding, skipped).
constexpr uint32_t kNoEntry = 0xFFFFFFFFu;

__global__ void k_ht_insert_b(const uint64_t* __restrict__ rec, uint32_t cap, const int64_t* __restrict__ counts,
                              uint32_t total, unsigned long long* __restrict__ tkey,
                              unsigned long long* __restrict__ tmin, uint32_t mask, uint32_t shift, uint32_t side,
                              uint32_t* __restrict__ pos_out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t r = q / cap, p = q - r * cap;
  if ((int64_t)p >= counts[r]) {
    if (pos_out) pos_out[q] = kNoEntry;
    return;
  }
  const uint32_t h = ht_find(tkey, rec[2 * (uint64_t)q], mask, shift);
  const unsigned long long v = rec[2 * (uint64_t)q + 1];
  unsigned long long* m = &tmin[2 * (uint64_t)h + side];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  if (pos_out) pos_out[q] = h;
}

__global__ void k_ht_answer_b(const uint32_t* __restrict__ pos, uint32_t total, const uint64_t* __restrict__ tmin,
                              int64_t* __restrict__ result) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t h = pos[q];
  if (h == kNoEntry) return;  // padding: nobody reads its answer
  const uint64_t e = tmin[2 * (uint64_t)h + 1];
  result[q] = e != ~0ull ? -(int64_t)e - 1 : (int64_t)tmin[2 * (uint64_t)h];
}

// Round 5: the owner's table sized from the records that arrived, not from
// the buckets' capacity, in one 16-byte (key, files' minimum) entry per slot
// — an insert is one line (its CAS and its atomicMin), an answer one line —
// plus the existing Objects' minima in a side array only when some arrived.
// The valid counts live on the device (the exchange carried them), so a
// one-wave kernel turns them into the table's mask and shift (cfg) and the
// other kernels read those: no host synchronisation, and only the table
// that is used is cleared. C5 at world 8 before: world x cap = 7.03 M slots
// of records, 2^24 slots x 24 B = 402 MB cleared per call for 3.04 M valid
// records; now 2^23 x 16 B = 134 MB.
__global__ void k_rb_size(const int64_t* __restrict__ fcounts, const int64_t* __restrict__ ecounts, uint32_t world,
                          uint32_t* __restrict__ cfg) {
  const uint32_t lane = threadIdx.x;
  uint64_t s = 0;
  for (uint32_t r = lane; r < world; r += 64) s += (uint64_t)fcounts[r] + (ecounts ? (uint64_t)ecounts[r] : 0ull);
#pragma unroll
  for (int d = 32; d; d >>= 1) s += __shfl_xor(s, d);
  if (lane == 0) {
    uint64_t cap = 1024;
    while (cap < 2 * s) cap <<= 1;
    cfg[0] = (uint32_t)(cap - 1);
    cfg[1] = 64u - (uint32_t)__builtin_ctzll(cap);
  }
}

// entries 0..mask+1 (the all-ones key's extra entry included) of the table
// and of the existing minima (when present) to all ones
__global__ void k_rb_clear(ulonglong2* __restrict__ tab, unsigned long long* __restrict__ emin,
                           const uint32_t* __restrict__ cfg) {
  const uint64_t m = (uint64_t)cfg[0] + 2;
  const ulonglong2 ones = make_ulonglong2(~0ull, ~0ull);
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (uint64_t)gridDim.x * blockDim.x) {
    tab[q] = ones;
    if (emin) emin[q] = ~0ull;
  }
}

__global__ void k_rb_insert(const uint64_t* __restrict__ rec, uint32_t bcap, const int64_t* __restrict__ counts,
                            uint32_t total, unsigned long long* __restrict__ tab,
                            unsigned long long* __restrict__ emin, const uint32_t* __restrict__ cfg,
                            uint32_t* __restrict__ pos_out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t r = q / bcap, p = q - r * bcap;
  if ((int64_t)p >= counts[r]) {
    if (pos_out) pos_out[q] = kNoEntry;
    return;
  }
  const uint32_t mask = cfg[0], shift = cfg[1];
  const uint64_t key = rec[2 * (uint64_t)q];
  const unsigned long long v = rec[2 * (uint64_t)q + 1];
  uint32_t h = mask + 1;  // the all-ones key's own entry
  if (key != kEmptyKey) {
    h = (uint32_t)((key << kOwnerBits) >> shift) & mask;  // below the owner bits (ht_find)
    for (;;) {
      const unsigned long long cur =
          __hip_atomic_load(&tab[2 * (uint64_t)h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == key) break;
      if (cur == kEmptyKey) {
        const unsigned long long prev =
            atomicCAS(&tab[2 * (uint64_t)h], (unsigned long long)kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey || prev == key) break;
      }
      h = (h + 1) & mask;
    }
  }
  unsigned long long* m = emin ? &emin[h] : &tab[2 * (uint64_t)h + 1];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  if (pos_out) pos_out[q] = h;
}

__global__ void k_rb_answer(const uint32_t* __restrict__ pos, uint32_t total, const uint64_t* __restrict__ tab,
                            const uint64_t* __restrict__ emin, int64_t* __restrict__ result) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t h = pos[q];
  if (h == kNoEntry) return;  // padding: nobody reads its answer
  const uint64_t e = emin ? emin[h] : ~0ull;
  // mod.rs:202-238: the first existing Object carrying the key; else the
  // key's first file (mod.rs:246-254)
  result[q] = e != ~0ull ? -(int64_t)e - 1 : (int64_t)tab[2 * (uint64_t)h + 1];
}

// The owner's table in its compact form (the default): one u32 per slot, the
// index of the record that claimed the key (file records 0..nf, existing
// records nf + j), the key read back through it; the claim is the key's only
// atomic, and every other record of the key folds its value into a side
// minimum (vmin for files, emin for existing Objects) — one atomic per record
// instead of the claim's CAS plus its atomicMin, which put the 16-byte table
// at the chip's atomic rate (C5 at world 8: 6.1 M atomics, 269 us). The
// claimer's own value is its record's, read back by the others through the
// table (a claimer marks its slot in tpos and reads only the minimum). A
// plain store of the claimer's value beside the minima cost the insert more
// than it saved the answer (C5 at world 8: +50 / -4 us). Existing records
// are inserted first, so a key with any existing Object has one as its
// claimer.
// a file record's slot in tpos carries this bit when the record claimed it
// (slots stay below 2^31: the table takes at most 2^30 + 1 entries here)
constexpr uint32_t kPosClaimed = 1u << 31;

__device__ __forceinline__ const uint64_t* rb_rec(const uint64_t* frec, const uint64_t* erec, uint32_t nf,
                                                  uint32_t x) {
  return x < nf ? frec + 2 * (uint64_t)x : erec + 2 * (uint64_t)(x - nf);
}

__global__ void k_rb_insert_idx(const uint64_t* __restrict__ frec, const uint64_t* __restrict__ erec, uint32_t nf,
                                uint32_t bcap, const int64_t* __restrict__ counts, uint32_t total, uint32_t base,
                                uint32_t* __restrict__ tab, unsigned long long* __restrict__ vmin,
                                const uint32_t* __restrict__ cfg, uint32_t* __restrict__ pos_out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t r = q / bcap, p = q - r * bcap;
  if ((int64_t)p >= counts[r]) {
    if (pos_out) pos_out[q] = kNoEntry;
    return;
  }
  const uint32_t mask = cfg[0], shift = cfg[1];
  const uint32_t x = base + q;
  const uint64_t* me = rb_rec(frec, erec, nf, x);
  const uint64_t key = me[0];
  uint32_t h = mask + 1;  // the all-ones key's own entry
  bool claimed = false;
  if (key != kEmptyKey) {
    h = (uint32_t)((key << kOwnerBits) >> shift) & mask;  // below the owner bits (ht_find)
    for (;;) {
      uint32_t cur = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kIdxEmpty) {
        cur = atomicCAS(&tab[h], kIdxEmpty, x);
        if (cur == kIdxEmpty) {
          claimed = true;
          break;
        }
      }
      if (rb_rec(frec, erec, nf, cur)[0] == key) break;
      h = (h + 1) & mask;
    }
  } else {
    claimed = atomicCAS(&tab[h], kIdxEmpty, x) == kIdxEmpty;
  }
  if (!claimed) {
    const unsigned long long v = me[1];
    unsigned long long* m = &vmin[h];
    if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  }
  if (pos_out) pos_out[q] = h | (claimed ? kPosClaimed : 0u);
}

// Round 6 ("rec", the default): the other records of a key fold their value
// into the CLAIMING record's own value field (the received buckets are the
// protocol's scratch) instead of a side minimum per table slot, so there is
// no minima array to clear (C5 at world 8: cap u64 = 128 MiB per call) and the
// answer reads one record. A file record whose claimer is an existing Object
// folds nothing (the key's answer is the existing minimum); existing records
// are inserted first and fold into their existing claimer.
__global__ void k_rb_insert_rec(uint64_t* __restrict__ frec, uint64_t* __restrict__ erec, uint32_t nf, uint32_t bcap,
                                const int64_t* __restrict__ counts, uint32_t total, uint32_t base,
                                uint32_t* __restrict__ tab, const uint32_t* __restrict__ cfg,
                                uint32_t* __restrict__ pos_out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint32_t r = q / bcap, p = q - r * bcap;
  if ((int64_t)p >= counts[r]) {
    if (pos_out) pos_out[q] = kNoEntry;
    return;
  }
  const uint32_t mask = cfg[0], shift = cfg[1];
  const uint32_t x = base + q;
  const uint64_t* me = rb_rec(frec, erec, nf, x);
  const uint64_t key = me[0];
  uint32_t h = mask + 1;  // the all-ones key's own entry
  uint32_t cur = kIdxEmpty;
  if (key != kEmptyKey) {
    h = (uint32_t)((key << kOwnerBits) >> shift) & mask;  // below the owner bits (ht_find)
    for (;;) {
      cur = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kIdxEmpty) {
        cur = atomicCAS(&tab[h], kIdxEmpty, x);
        if (cur == kIdxEmpty) break;  // claimed
      }
      if (rb_rec(frec, erec, nf, cur)[0] == key) break;
      h = (h + 1) & mask;
    }
  } else {
    cur = atomicCAS(&tab[h], kIdxEmpty, x);
  }
  const bool claimed = cur == kIdxEmpty;
  // fold into the claimer's value (same domain only: files into a file
  // claimer, existing Objects into an existing claimer)
  if (!claimed && (cur >= nf) == (x >= nf)) {
    unsigned long long* m = reinterpret_cast<unsigned long long*>(
        const_cast<uint64_t*>(rb_rec(frec, erec, nf, cur)) + 1);
    const unsigned long long v = me[1];
    if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  }
  if (pos_out) pos_out[q] = h | (claimed ? kPosClaimed : 0u);
}

__global__ void k_rb_answer_rec(const uint32_t* __restrict__ pos, uint32_t nf, const uint64_t* __restrict__ frec,
                                const uint64_t* __restrict__ erec, const uint32_t* __restrict__ tab,
                                int64_t* __restrict__ result) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nf) return;
  const uint32_t hp = pos[q];
  if (hp == kNoEntry) return;  // padding: nobody reads its answer
  const uint32_t c = (hp & kPosClaimed) ? q : tab[hp & ~kPosClaimed];
  const uint64_t v = rb_rec(frec, erec, nf, c)[1];  // the claimer's value: the key's minimum
  // mod.rs:202-238: the first existing Object (an existing claimer); else
  // the key's first file (mod.rs:246-254)
  result[q] = c >= nf ? -(int64_t)v - 1 : (int64_t)v;
}

// the table's size from the valid counts (as k_rb_size, computed by every
// workgroup; workgroup 0 stores it in cfg for the inserts), then its clear:
// one launch
__global__ void k_rb_clear_tab(uint32_t* __restrict__ tab, const int64_t* __restrict__ fcounts,
                               const int64_t* __restrict__ ecounts, uint32_t world, uint32_t* __restrict__ cfg) {
  __shared__ uint64_t s_cap;
  if (threadIdx.x < 64) {
    uint64_t s = 0;
    for (uint32_t r = threadIdx.x; r < world; r += 64)
      s += (uint64_t)fcounts[r] + (ecounts ? (uint64_t)ecounts[r] : 0ull);
#pragma unroll
    for (int d = 32; d; d >>= 1) s += __shfl_xor(s, d);
    if (threadIdx.x == 0) {
      uint64_t cap = 1024;
      while (cap < 2 * s) cap <<= 1;
      s_cap = cap;
      if (blockIdx.x == 0) {
        cfg[0] = (uint32_t)(cap - 1);
        cfg[1] = 64u - (uint32_t)__builtin_ctzll(cap);
      }
    }
  }
  __syncthreads();
  const uint64_t m = s_cap + 1;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (uint64_t)gridDim.x * blockDim.x)
    tab[q] = kIdxEmpty;
}

__global__ void k_rb_answer_idx(const uint32_t* __restrict__ pos, uint32_t nf, const uint64_t* __restrict__ frec,
                                const uint64_t* __restrict__ erec, const uint32_t* __restrict__ tab,
                                const uint64_t* __restrict__ vmin, const uint64_t* __restrict__ emin,
                                int64_t* __restrict__ result) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nf) return;
  const uint32_t hp = pos[q];
  if (hp == kNoEntry) return;  // padding: nobody reads its answer
  const uint32_t h = hp & ~kPosClaimed;
  // the claimer knows its own value (a file claimer: no existing Object has
  // the key); another record reads the claimer's through the table
  const uint32_t c = (hp & kPosClaimed) ? q : tab[h];
  const uint64_t own = rb_rec(frec, erec, nf, c)[1];
  // mod.rs:202-238: the first existing Object carrying the key (a key with
  // one has an existing record as its claimer); else the key's first file
  // (mod.rs:246-254)
  if (c >= nf) {
    const uint64_t e = emin[h] < own ? emin[h] : own;
    result[q] = -(int64_t)e - 1;
  } else {
    result[q] = (int64_t)(vmin[h] < own ? vmin[h] : own);
  }
}

__global__ void k_rb_clear_idx(uint32_t* __restrict__ tab, unsigned long long* __restrict__ vmin,
                               unsigned long long* __restrict__ emin, const uint32_t* __restrict__ cfg) {
  const uint64_t m = (uint64_t)cfg[0] + 2;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (uint64_t)gridDim.x * blockDim.x) {
    tab[q] = kIdxEmpty;
    vmin[q] = ~0ull;
    if (emin) emin[q] = ~0ull;
  }
}

// SDCAS_RESOLVE: "idx" (the default, above), "kv" = round 5's 16-byte (key,
// files' minimum) entries sized on the device, "split" = round 4's key array
// + minima pairs sized from the buckets' capacity (A/B)
enum ResolveTable { kResolveIdx = 0, kResolveKv = 1, kResolveSplit = 2, kResolveRec = 3 };
static ResolveTable resolve_table() {
  const char* v = getenv("SDCAS_RESOLVE");
  if (v && strcmp(v, "split") == 0) return kResolveSplit;
  if (v && strcmp(v, "kv") == 0) return kResolveKv;
  if (v && strcmp(v, "idx") == 0) return kResolveIdx;
  return kResolveRec;
}

hipError_t dd_resolve_buckets(DistWs& w, const uint64_t* frec, uint32_t fcap, const int64_t* fcounts,
                              const uint64_t* erec, uint32_t ecap, const int64_t* ecounts, uint32_t world,
                              int64_t* result, hipStream_t st) {
  hipError_t e;
  const uint32_t nf = world * fcap, ne = world * ecap;
  if (nf == 0) return hipSuccess;
  uint64_t cap = 1024;
  while (cap < 2 * ((uint64_t)nf + ne)) cap <<= 1;
  if (cap > (1ull << 31)) return hipErrorInvalidValue;
  ResolveTable rt = resolve_table();
  if ((rt == kResolveIdx || rt == kResolveRec) && cap > (1ull << 30)) rt = kResolveKv;  // tpos' claimed bit: slots < 2^31
  if (rt == kResolveRec) {
    // the received buckets' value fields take the minima (sdcas.h: resolve_buckets)
    if ((e = w.tmin.ensure(cap / 2 + 1)) || (e = w.tpos.ensure(nf)) || (e = w.starts.ensure(2))) return e;
    auto* tab = reinterpret_cast<uint32_t*>(w.tmin.p);
    auto* fr = const_cast<uint64_t*>(frec);
    auto* er = const_cast<uint64_t*>(erec);
    const uint32_t cg = (uint32_t)std::min<uint64_t>((cap + 1 + TB - 1) / TB, 2048);
    hipLaunchKernelGGL(k_rb_clear_tab, dim3(cg), dim3(TB), 0, st, tab, fcounts, ne ? ecounts : nullptr, world,
                       w.starts.p);
    if (ne)
      hipLaunchKernelGGL(k_rb_insert_rec, dim3(blocks(ne)), dim3(TB), 0, st, fr, er, nf, ecap, ecounts, ne, nf, tab,
                         w.starts.p, (uint32_t*)nullptr);
    hipLaunchKernelGGL(k_rb_insert_rec, dim3(blocks(nf)), dim3(TB), 0, st, fr, er, nf, fcap, fcounts, nf, 0u, tab,
                       w.starts.p, w.tpos.p);
    hipLaunchKernelGGL(k_rb_answer_rec, dim3(blocks(nf)), dim3(TB), 0, st, w.tpos.p, nf, frec, erec, tab, result);
    return hipGetLastError();
  }
  if (rt == kResolveIdx) {
    // tmin holds the u32 table (cap + 1 u32 in its first cap + 1 u64) and
    // the existing minima; tkey the files' minima
    if ((e = w.tmin.ensure(2 * (cap + 1))) || (e = w.tkey.ensure(cap + 1)) || (e = w.tpos.ensure(nf)) ||
        (e = w.starts.ensure(2)))
      return e;
    auto* tab = reinterpret_cast<uint32_t*>(w.tmin.p);
    auto* vm = reinterpret_cast<unsigned long long*>(w.tkey.p);
    auto* em = ne ? reinterpret_cast<unsigned long long*>(w.tmin.p + (cap + 1)) : nullptr;
    hipLaunchKernelGGL(k_rb_size, dim3(1), dim3(64), 0, st, fcounts, ne ? ecounts : nullptr, world, w.starts.p);
    const uint64_t slots = cap + 1;
    const uint32_t cg = (uint32_t)std::min<uint64_t>((slots + TB - 1) / TB, 2048);
    hipLaunchKernelGGL(k_rb_clear_idx, dim3(cg), dim3(TB), 0, st, tab, vm, em, w.starts.p);
    if (ne)
      hipLaunchKernelGGL(k_rb_insert_idx, dim3(blocks(ne)), dim3(TB), 0, st, frec, erec, nf, ecap, ecounts, ne, nf,
                         tab, em, w.starts.p, (uint32_t*)nullptr);
    hipLaunchKernelGGL(k_rb_insert_idx, dim3(blocks(nf)), dim3(TB), 0, st, frec, erec, nf, fcap, fcounts, nf, 0u, tab,
                       vm, w.starts.p, w.tpos.p);
    hipLaunchKernelGGL(k_rb_answer_idx, dim3(blocks(nf)), dim3(TB), 0, st, w.tpos.p, nf, frec, erec, tab, w.tkey.p,
                       (const uint64_t*)em, result);
    return hipGetLastError();
  }
  if (rt == kResolveKv) {
    // cap bounds the table the valid counts ask for; allocate that, clear what they ask
    if ((e = w.tmin.ensure(2 * (cap + 1))) || (ne && (e = w.tkey.ensure(cap + 1))) || (e = w.tpos.ensure(nf)) ||
        (e = w.starts.ensure(2)))
      return e;
    auto* tab = reinterpret_cast<unsigned long long*>(w.tmin.p);
    auto* em = ne ? reinterpret_cast<unsigned long long*>(w.tkey.p) : nullptr;
    hipLaunchKernelGGL(k_rb_size, dim3(1), dim3(64), 0, st, fcounts, ne ? ecounts : nullptr, world, w.starts.p);
    const uint64_t slots = cap + 1;
    const uint32_t cg = (uint32_t)std::min<uint64_t>((slots + TB - 1) / TB, 2048);
    hipLaunchKernelGGL(k_rb_clear, dim3(cg), dim3(TB), 0, st, reinterpret_cast<ulonglong2*>(tab), em, w.starts.p);
    if (ne)
      hipLaunchKernelGGL(k_rb_insert, dim3(blocks(ne)), dim3(TB), 0, st, erec, ecap, ecounts, ne, tab, em, w.starts.p,
                         (uint32_t*)nullptr);
    hipLaunchKernelGGL(k_rb_insert, dim3(blocks(nf)), dim3(TB), 0, st, frec, fcap, fcounts, nf, tab,
                       (unsigned long long*)nullptr, w.starts.p, w.tpos.p);
    hipLaunchKernelGGL(k_rb_answer, dim3(blocks(nf)), dim3(TB), 0, st, w.tpos.p, nf, w.tmin.p,
                       ne ? w.tkey.p : nullptr, result);
    return hipGetLastError();
  }
  if ((e = w.tkey.ensure(cap + 1)) || (e = w.tmin.ensure(2 * (cap + 1))) || (e = w.tpos.ensure(nf))) return e;
  const uint32_t mask = (uint32_t)(cap - 1);
  const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(cap);
  if ((e = hipMemsetAsync(w.tkey.p, 0xFF, sizeof(uint64_t) * (cap + 1), st)) ||
      (e = hipMemsetAsync(w.tmin.p, 0xFF, sizeof(uint64_t) * 2 * (cap + 1), st)))
    return e;
  auto* tk = reinterpret_cast<unsigned long long*>(w.tkey.p);
  auto* tm = reinterpret_cast<unsigned long long*>(w.tmin.p);
  if (ne)
    hipLaunchKernelGGL(k_ht_insert_b, dim3(blocks(ne)), dim3(TB), 0, st, erec, ecap, ecounts, ne, tk, tm, mask, shift,
                       1u, nullptr);
  hipLaunchKernelGGL(k_ht_insert_b, dim3(blocks(nf)), dim3(TB), 0, st, frec, fcap, fcounts, nf, tk, tm, mask, shift, 0u,
                     w.tpos.p);
  hipLaunchKernelGGL(k_ht_answer_b, dim3(blocks(nf)), dim3(TB), 0, st, w.tpos.p, nf, w.tmin.p, result);
  return hipGetLastError();
}

// ---- a world of one: no exchange, hence no combine ---------------------------
//
// The combine exists to shrink what crosses the exchange and to group it by
// owner. With one rank there is nothing to exchange: every present file's
// (key, ordinal) and every existing Object's (key, DB index) go straight into
// the resolve table, and each file reads its answer from its own entry.

// The table: one 16-byte entry per slot, (key, minimum file ordinal), so an
// insert touches one line; the existing Objects' minima live in a side array
// (emin), allocated and read only when there are existing Objects.
__device__ __forceinline__ uint32_t ht_find_kv(unsigned long long* __restrict__ tab, uint64_t key, uint32_t mask,
                                               uint32_t shift) {
  if (key == kEmptyKey) return mask + 1;
  uint32_t h = (uint32_t)(key >> shift) & mask;
  for (;;) {
    const unsigned long long cur = __hip_atomic_load(&tab[2 * (uint64_t)h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return h;
    if (cur == kEmptyKey) {
      const unsigned long long prev =
          atomicCAS(&tab[2 * (uint64_t)h], (unsigned long long)kEmptyKey, (unsigned long long)key);
      if (prev == kEmptyKey || prev == key) return h;
    }
    h = (h + 1) & mask;
  }
}

// files (emin null): pos[i] = entry, or the slot code of a file without one;
// existing Objects (emin set): min-fold the DB index into emin[entry]
__global__ void k_solo_insert(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ has_key,
                              const int32_t* __restrict__ status, const uint64_t* __restrict__ ids, uint32_t n,
                              unsigned long long* __restrict__ tab, unsigned long long* __restrict__ emin,
                              uint32_t mask, uint32_t shift, uint32_t* __restrict__ pos) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool ok = status == nullptr || status[i] == 0;  // mod.rs:125-141
  const bool has = has_key == nullptr || has_key[i];    // mod.rs:83-86
  if (!(ok && has)) {
    if (pos) pos[i] = !ok ? kSlotDropped : kSlotNoKey;
    return;
  }
  const uint32_t h = ht_find_kv(tab, keys[i], mask, shift);
  const unsigned long long v = ids[i];
  unsigned long long* m = emin ? &emin[h] : &tab[2 * (uint64_t)h + 1];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  if (pos) pos[i] = h;
}

// k_dd_apply with the answer read from the file's own table entry
__global__ void k_solo_apply(const uint64_t* __restrict__ ids, const uint32_t* __restrict__ pos, uint32_t n,
                             const uint64_t* __restrict__ tab, const uint64_t* __restrict__ emin, uint64_t cs,
                             const uint64_t* __restrict__ plan, int64_t* __restrict__ link,
                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  const PlanView pv = plan_view(plan);
  unsigned long long c = 0, l = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t h = pos[i];
    const int kind = h == kSlotDropped ? kFileDropped : h == kSlotNoKey ? kFileNoKey : kFileKeyed;
    int64_t r = 0;
    if (kind == kFileKeyed) {
      // mod.rs:202-238: the first existing Object; else the key's first file
      const uint64_t e = emin ? emin[h] : ~0ull;
      r = e != ~0ull ? -(int64_t)e - 1 : (int64_t)tab[2 * (uint64_t)h + 1];
    }
    link[i] = step_link(kind, (int64_t)ids[i], r, cs, pv, c, l);
  }
  add_counts(c, l, sc, counts);
}

// The compact table of a world of one: one u32 per slot, the lowest index
// carrying the slot's key in a combined index space — file i is i, existing
// Object j is n + j — so 4 bytes a slot instead of 16, a table (and its
// clearing) a quarter of the kv table's that stays resident in the Infinity
// Cache (C5: 67 MB against 268 MB). A slot's key is read back through the
// index it holds, never stored: every index ever written to a slot carries
// the same key, so the slot's key never changes, and the atomicMin of later
// inserters leaves the lowest — a file whenever a file carries the key (ids
// are ascending, so the lowest file index has the lowest ordinal). Existing
// Objects fold their DB index into a u64 side array (emin) by slot, which
// exists only when there are existing Objects.

__device__ __forceinline__ uint64_t idx_key(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ ekeys,
                                            uint32_t n, uint32_t x) {
  return x < n ? keys[x] : ekeys[x - n];
}

// Rows per stays count of the world-of-one path: the files' insert counts each
// tile's stays rows (below), the clear zeroes, the stays writer sums and the
// plan walk reads exactly these tiles, so all four must take this one constant.
// Round 5's tile-shape experiment changed it to 2048 / 4096 while the insert
// still counted per literal 1024 rows (gpurun_out/r05dbg/seq_tile_*.log): the
// counts were allocated and zeroed for ceil(n / 2048) tiles while the insert
// filled ceil(n / 1024) (past the allocation), the writer placed tile b's rows
// after the counts of 1024-row tiles 0..b-1 (about half the rows before it, so
// tiles overwrote each other's entries), and the walk summed only the first
// ceil(n / 2048) counts; the stays list it walked held misplaced, unordered
// ordinals, so the plan took re-reads the job never makes and the batch's last
// rows fell past task_count's limit (file 29994 of 30000 came back
// SDCAS_LINK_DEFERRED instead of linked to 14).
constexpr uint32_t kStayTile = 1024;
static_assert(kStayTile % 64 == 0, "the insert's per-wave ballot add needs a wave's 64 rows in one tile");
static_assert(kStayTile % TB == 0, "k_stays_write_t walks a tile in whole workgroups");
// the tiles' counts are kept at two levels: per tile, and per group of
// kStayGroup tiles (after the tile counts), so that a writer's offset is at
// most nt / kStayGroup + kStayGroup - 1 counts (a plain sum over the tiles
// before it cost tiles^2 reads: 50 M files with stays in every tile, 48 828
// tiles: 433 us) and a batch without stays rows pays nothing
constexpr uint32_t kStayGroup = 64;
__host__ __device__ constexpr uint32_t stay_groups(uint32_t nt) { return (nt + kStayGroup - 1) / kStayGroup; }

// files (emin null, base 0): pos[i] = slot, or the code of a file without
// one; existing Objects (emin set, base n): min-fold eids[j] into emin[slot]
// (sticky = kIdxEmpty: slot mode) or into emin[j'] for the key's claiming
// Object j' (sticky = n: entry mode — the existing Objects' pass runs first,
// their claims stay, and a file finding one leaves it: the apply reads the
// minimum through the claim, from an array of ne entries instead of cap)
// stay_cnt (files, may be null): += the rows of each kStayTile-row tile that
// stay orphans, one atomicAdd per wave holding one
// noncontig (files, may be null; eids = the files' ordinals then): set when
// some file's ordinal is not eids[0] + its index (one atomicOr per wave
// that finds one), so that the apply can take a key's first ordinal from its
// index instead of reading it
__global__ void k_solo_insert_idx(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ ekeys, uint32_t n,
                                  const uint8_t* __restrict__ has_key, const int32_t* __restrict__ status,
                                  const uint64_t* __restrict__ eids, uint32_t count, uint32_t base,
                                  uint32_t* __restrict__ tab, unsigned long long* __restrict__ emin, uint32_t mask,
                                  uint32_t shift, uint32_t* __restrict__ pos, uint32_t* __restrict__ stay_cnt,
                                  uint32_t* __restrict__ noncontig, uint32_t sticky, uint32_t plain) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= count) return;
  const uint32_t x = base + q;
  if (!emin) {
    if (noncontig) {
      const uint64_t bad = __ballot(eids[q] != eids[0] + q);
      if (bad && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)bad) - 1)) atomicOr(noncontig, 1u);
    }
    const bool ok = status == nullptr || status[q] == 0;  // mod.rs:125-141
    const bool has = has_key == nullptr || has_key[q];    // mod.rs:83-86
    if (stay_cnt) {
      const uint64_t bal = __ballot(!(ok && has));
      if (bal && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)bal) - 1)) {
        // a wave's 64 rows share a tile; the tile's count, then its group's
        // (kStayGroup tiles, after the nt tile counts)
        const uint32_t nt = (count + kStayTile - 1) / kStayTile;
        atomicAdd(&stay_cnt[q / kStayTile], (uint32_t)__popcll(bal));
        atomicAdd(&stay_cnt[nt + q / (kStayTile * kStayGroup)], (uint32_t)__popcll(bal));
      }
    }
    if (!(ok && has)) {
      pos[q] = !ok ? kSlotDropped : kSlotNoKey;
      return;
    }
  }
  const uint64_t key = idx_key(keys, ekeys, n, x);
  uint32_t h = (uint32_t)(key >> shift) & mask;
  uint32_t x_claim = x;
  for (;;) {
    // plain: the probe as an ordinary load, which may hit a stale line in
    // this XCD's L2 — safe, as a slot only ever goes from empty to an index of
    // ONE key and then to lower indices of that key: a stale empty is
    // corrected by the CAS's answer, a stale index names the same key
    uint32_t cur = plain ? tab[h] : __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kIdxEmpty) {
      const uint32_t prev = atomicCAS(&tab[h], kIdxEmpty, x);
      if (prev == kIdxEmpty) break;
      cur = prev;
    }
    if (idx_key(keys, ekeys, n, cur) == key) {
      // an existing Object's claim is sticky (entry mode): files leave it
      if (cur > x && cur < sticky && !(emin && sticky != kIdxEmpty)) atomicMin(&tab[h], x);
      if (emin && sticky != kIdxEmpty) x_claim = cur;
      break;
    }
    h = (h + 1) & mask;
  }
  if (emin) {
    // slot mode: the DB index min-folds into emin[slot] (cap entries);
    // entry mode: into emin[claimer - n] (ne entries, the claimer fixed by
    // its CAS: existing Objects never lower a claim)
    unsigned long long* m = sticky != kIdxEmpty ? &emin[x_claim - n] : &emin[h];
    const unsigned long long v = eids[q];
    if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > v) atomicMin(m, v);
  } else {
    pos[q] = h;
  }
}

__global__ void k_solo_apply_idx(const uint64_t* __restrict__ ids, const uint32_t* __restrict__ pos, uint32_t n,
                                 const uint32_t* __restrict__ tab, const uint64_t* __restrict__ emin, uint64_t cs,
                                 const uint64_t* __restrict__ plan, int64_t* __restrict__ link,
                                 unsigned long long* __restrict__ counts, uint32_t ebase) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  const PlanView pv = plan_view(plan);
  unsigned long long c = 0, l = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t h = pos[i];
    const int kind = h == kSlotDropped ? kFileDropped : h == kSlotNoKey ? kFileNoKey : kFileKeyed;
    int64_t r = 0;
    if (kind == kFileKeyed) {
      // mod.rs:202-238: the first existing Object; else (mod.rs:246-254) the
      // key's first file — a file, as this one carries the key
      const uint32_t f = tab[h];
      // entry mode (ebase = n): a claim by existing Object f - n holds its minimum
      const uint64_t e = ebase != kIdxEmpty ? (f >= ebase ? emin[f - ebase] : ~0ull) : emin ? emin[h] : ~0ull;
      r = e != ~0ull ? -(int64_t)e - 1 : (int64_t)(f == i ? ids[i] : ids[f]);
    }
    link[i] = step_link(kind, (int64_t)ids[i], r, cs, pv, c, l);
  }
  add_counts(c, l, sc, counts);
}

// ---- round 5: the world-of-one path in fewer launches -----------------------------
//
// The files' insert also counts, per 1024-row tile, the rows that stay
// orphans (one atomicAdd per wave that holds one; C3 / C5 have none), so
// the stays pass loses its counting launch and its one-workgroup scan: the
// writer sums the counts of the tiles before its own, and the plan walk sums
// them all. One clear kernel empties the table, the existing Objects'
// minima and the tile counts. Five launches where round 4 had eight (C3:
// 0.181 -> 0.168 ms per call in the same process, profiles/r05_ab_dedup.json).
// Measured and not kept (same-process A/Bs, bit-identical links): tiles of
// 1024 / 4096 files issuing each probe phase for 4 or 16 files per thread
// together, and tiles that first group their files by key in LDS so that only
// a key's lowest file per tile touches the table (C5's 4096-file tiles hold
// 71 % distinct keys) — every shape was slower on C5, 0.43-0.67 ms against
// 0.40, the barrier a tile needs holding its workgroup until its slowest
// probe chain ends; and, without tiles, the files' insert taking 2 or 4
// files per thread with each probe phase issued for all of them (C5 insert
// 210 -> 467 us at 4, profiles/r05_ab_dedup_apply.json). The tile is
// kStayTile (defined above the insert, which counts per tile).


__global__ void k_local_clear(uint4* __restrict__ tab, uint64_t tab_q, uint4* __restrict__ em, uint64_t em_q,
                              uint32_t* __restrict__ cnt, uint32_t nt, uint32_t* __restrict__ flag) {
  const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t q = t0; q < tab_q; q += stride) tab[q] = ones;
  for (uint64_t q = t0; q < em_q; q += stride) em[q] = ones;
  for (uint64_t q = t0; q < nt; q += stride) cnt[q] = 0;
  if (flag && t0 == 0) *flag = 0;
}

// The apply with R files per thread, each phase's loads issued for all R
// before the next phase (slot, then the table's lowest index and the existing
// minimum, then the winner's ordinal) and a grid of one workgroup per TB * R
// files: full occupancy instead of 1024 workgroups walking their files one
// dependent chain at a time. The counts go to kCountShards pairs (workgroup
// b adds to pair b % kCountShards), folded into the caller's by
// k_counts_fold — thousands of workgroups adding to one address serialise.
template <uint32_t R>
__global__ void __launch_bounds__(TB) k_solo_apply_r(const uint64_t* __restrict__ ids,
                                                     const uint32_t* __restrict__ pos, uint32_t n,
                                                     const uint32_t* __restrict__ tab,
                                                     const uint64_t* __restrict__ emin, uint64_t cs,
                                                     const uint64_t* __restrict__ plan, int64_t* __restrict__ link,
                                                     unsigned long long* __restrict__ shard,
                                                     const uint32_t* __restrict__ noncontig, uint32_t ebase,
                                                     const uint64_t* __restrict__ ridx) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  const PlanView pv = plan_view(plan, ridx);
  // ordinals eids[0] + index (the insert found no other): a key's first
  // ordinal follows from its first file's index, no read
  const bool contig = noncontig && *noncontig == 0;
  const uint64_t i0 = (uint64_t)blockIdx.x * TB * R + threadIdx.x;
  uint32_t h[R], f[R];
  uint64_t e[R], r[R], me[R];
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    h[k] = i < n ? pos[i] : kSlotDropped;
    me[k] = i < n ? ids[i] : 0;
  }
  const bool entry = ebase != kIdxEmpty;  // existing minima by claiming Object (ne entries), not by slot
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const bool keyed = h[k] < kSlotDropped && h[k] != kSlotNoKey;
    f[k] = keyed ? tab[h[k]] : 0u;
    e[k] = keyed && emin && !entry ? emin[h[k]] : ~0ull;
  }
  if (entry) {
#pragma unroll
    for (uint32_t k = 0; k < R; ++k) {
      const bool keyed = h[k] < kSlotDropped && h[k] != kSlotNoKey;
      if (keyed && f[k] >= ebase) e[k] = emin[f[k] - ebase];
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    const bool keyed = h[k] < kSlotDropped && h[k] != kSlotNoKey;
    // mod.rs:202-238: the first existing Object; else (mod.rs:246-254) the
    // key's first file — a file, as this one carries the key
    r[k] = !keyed || e[k] != ~0ull || f[k] == (uint32_t)i ? me[k]
           : contig                                           ? me[k] - i + f[k]
                                                              : ids[f[k]];
  }
  unsigned long long c = 0, l = 0;
#pragma unroll
  for (uint32_t k = 0; k < R; ++k) {
    const uint64_t i = i0 + (uint64_t)k * TB;
    if (i >= n) continue;
    const int kind = h[k] == kSlotDropped ? kFileDropped : h[k] == kSlotNoKey ? kFileNoKey : kFileKeyed;
    const int64_t rk = kind != kFileKeyed ? 0 : e[k] != ~0ull ? -(int64_t)e[k] - 1 : (int64_t)r[k];
    link[i] = step_link(kind, (int64_t)me[k], rk, cs, pv, c, l);
  }
  add_counts(c, l, sc, shard ? shard + 2 * (blockIdx.x % kCountShards) : nullptr);
}

// the shards' sums added to the caller's counts (one wave); the shards are
// left zeroed for the next call (and zeroed when allocated: shard_counts)
__global__ void k_counts_fold(unsigned long long* __restrict__ shard, unsigned long long* __restrict__ counts) {
  unsigned long long c = shard[2 * threadIdx.x], l = shard[2 * threadIdx.x + 1];
  shard[2 * threadIdx.x] = 0;
  shard[2 * threadIdx.x + 1] = 0;
  for (int off = 32; off > 0; off >>= 1) {
    c += __shfl_down(c, off);
    l += __shfl_down(l, off);
  }
  if (threadIdx.x == 0) {
    atomicAdd(&counts[0], c);
    atomicAdd(&counts[1], l);
  }
}

// the stays rows of tile blockIdx.x (PER rows) in order, at the offset the
// tiles before it add up to (only tiles holding one do any work): cnt holds
// the gridDim.x tile counts and, after them, the counts of their groups of
// kStayGroup tiles (the insert fills both), so the offset is the groups
// before this tile's group plus the tiles before it in its group.
// out32: the rows' indices; or, with ids (out64), their ordinals ids[i]
// (the plan walk then reads a dense list, not ids[idx[j]])
template <uint32_t PER>
__global__ void __launch_bounds__(TB) k_stays_write_t(const uint8_t* __restrict__ has_key,
                                                      const int32_t* __restrict__ status, uint32_t n,
                                                      const uint32_t* __restrict__ cnt, uint32_t* __restrict__ out,
                                                      const uint64_t* __restrict__ ids = nullptr,
                                                      uint64_t* __restrict__ out64 = nullptr) {
  __shared__ uint32_t ws[TB / 64];
  const uint32_t b = blockIdx.x;
  if (cnt[b] == 0) return;  // uniform over the workgroup
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t g = b / kStayGroup;
  const uint32_t* gcnt = cnt + gridDim.x;
  uint32_t s = 0;
  for (uint32_t t = tid; t < g; t += TB) s += gcnt[t];
  for (uint32_t t = g * kStayGroup + tid; t < b; t += TB) s += cnt[t];
#pragma unroll
  for (uint32_t d = 32; d; d >>= 1) s += __shfl_xor(s, d);
  if (lane == 0) ws[wave] = s;
  __syncthreads();
  uint32_t run = 0;
#pragma unroll
  for (uint32_t w = 0; w < TB / 64; ++w) run += ws[w];
  __syncthreads();
  const uint64_t lo = (uint64_t)b * PER;
#pragma unroll 1
  for (uint32_t r = 0; r < PER / TB; ++r) {
    const uint64_t i = lo + r * TB + tid;
    const bool f = i < n && stays_row(has_key, status, i);
    const uint64_t bal = __ballot(f);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (lane == 0) ws[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = run, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < TB / 64; ++w) {
      if (w < wave) before += ws[w];
      all += ws[w];
    }
    __syncthreads();
    if (f) {
      if (out64) out64[before + below] = ids[i];
      else out[before + below] = (uint32_t)i;
    }
    run += all;
  }
}

// SDCAS_DEDUP_TABLE: "idx" (the default) = the compact u32 table, the
// world-of-one path in five launches (above); "idx4" = the same table
// behind round 4's eight launches; "kv" = round 3's 16-byte (key, minimum)
// table (A/B)
enum DedupTable { kTableIdx = 0, kTableIdx4 = 1, kTableKv = 2 };
static DedupTable dedup_table() {
  const char* v = getenv("SDCAS_DEDUP_TABLE");
  if (v && strcmp(v, "kv") == 0) return kTableKv;
  if (v && strcmp(v, "idx4") == 0) return kTableIdx4;
  return kTableIdx;
}

// SDCAS_APPLY_R: files per thread of the fused path's apply (1, 2, 4, 8;
// 0 = round 5's grid-stride apply over at most 1024 workgroups), read per
// call (A/B in one process)
static uint32_t apply_files_per_thread() {
  const char* v = getenv("SDCAS_APPLY_R");
  const int x = v ? atoi(v) : 4;
  return x == 0 || x == 1 || x == 2 || x == 4 || x == 8 ? (uint32_t)x : 4u;
}

// SDCAS_CONTIG=0: the world-of-one apply reads every first ordinal (A/B)
static bool contig_ordinals() {
  const char* v = getenv("SDCAS_CONTIG");
  return !(v && strcmp(v, "0") == 0);
}

// the applies' count shards: zeroed when allocated, and by k_counts_fold
// after every use; a call whose launches failed between the apply and the
// fold marks them dirty (sharded_done), and the next call zeroes them first
static hipError_t shard_counts(DistWs& w, hipStream_t st) {
  if (w.shard.cap >= 2 * kCountShards && !w.shard_dirty) return hipSuccess;
  hipError_t e = w.shard.ensure(2 * kCountShards);
  if (!e) e = hipMemsetAsync(w.shard.p, 0, 2 * kCountShards * sizeof(unsigned long long), st);
  if (!e) w.shard_dirty = false;
  return e;
}

// the end of a call that used the shards: any launch error leaves them dirty
static hipError_t sharded_done(DistWs& w, bool sharded) {
  const hipError_t e = hipGetLastError();
  if (e && sharded) w.shard_dirty = true;
  return e;
}

// a world of one's table: a power of two of at least `load` slots per item
// (SDCAS_DEDUP_LOAD, default 2: at most half full when every key differs)
static uint64_t local_cap(uint64_t items) {
  const char* v = getenv("SDCAS_DEDUP_LOAD");  // read per call (A/B in one process)
  const double x = v ? atof(v) : 2.0;
  const double load = x >= 1.05 && x <= 8.0 ? x : 2.0;
  uint64_t cap = 1024;
  while ((double)cap < load * (double)items) cap <<= 1;
  return cap;
}

// SDCAS_EXIST_MIN=slot: the existing Objects' minima by table slot (cap u64,
// round 5) instead of by claiming Object (ne u64; the default), read per call
// (A/B in one process)
static bool exist_min_by_entry() {
  const char* v = getenv("SDCAS_EXIST_MIN");
  return !(v && strcmp(v, "slot") == 0);
}

// SDCAS_PROBE=plain: the files' insert probes with ordinary loads instead of
// agent-scope atomic loads (k_solo_insert_idx), read per call (A/B)
static bool plain_probe() {
  const char* v = getenv("SDCAS_PROBE");
  return v && strcmp(v, "plain") == 0;
}

static hipError_t local_fused(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                              const uint64_t* ids, uint32_t n, const uint64_t* ekeys, const uint64_t* eids,
                              uint32_t ne, uint64_t cs, const StepWindow& win, int64_t* link,
                              unsigned long long* counts, uint64_t cap, hipStream_t st) {
  hipError_t e;
  const uint32_t nt = (n + kStayTile - 1) / kStayTile;
  const bool stays = has_key || status;
  const uint32_t mask = (uint32_t)(cap - 1);
  const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(cap);
  // the u32 table borrows tmin's storage (cap u32 = cap / 4 of its u64);
  // the existing Objects' minima live in tkey (cap u64), when there are any
  const uint32_t ar = apply_files_per_thread();
  const bool sharded = ar && counts;
  const bool contig = ar && contig_ordinals() && n > 0;
  const bool entry = ne && exist_min_by_entry();
  const uint32_t sticky = entry ? n : kIdxEmpty;  // k_solo_insert_idx / the applies: entry mode from index n
  if ((e = w.tmin.ensure(cap / 2 + 1)) || (e = w.tpos.ensure(n)) ||
      (ne && (e = w.tkey.ensure(entry ? (uint64_t)ne + 2 : cap + 1))) ||
      (e = w.stay_cnt.ensure(nt + stay_groups(nt) + 1)) || (stays && (e = w.stay_sorted.ensure(n))) ||
      (sharded && (e = shard_counts(w, st))) ||
      (contig && (e = w.flag.ensure(1))))
    return e;
  auto* tab = reinterpret_cast<uint32_t*>(w.tmin.p);
  auto* em = ne ? reinterpret_cast<unsigned long long*>(w.tkey.p) : nullptr;
  const uint64_t tab_q = cap / 4, em_q = !ne ? 0 : entry ? ((uint64_t)ne + 1) / 2 : cap / 2;  // uint4 stores
  const uint32_t cg = (uint32_t)std::min<uint64_t>((tab_q + em_q + TB - 1) / TB, 2048);
  hipLaunchKernelGGL(k_local_clear, dim3(cg), dim3(TB), 0, st, reinterpret_cast<uint4*>(tab), tab_q,
                     reinterpret_cast<uint4*>(em), em_q, w.stay_cnt.p, stays ? nt + stay_groups(nt) : 0u,
                     contig ? w.flag.p : (uint32_t*)nullptr);
  if (ne)
    hipLaunchKernelGGL(k_solo_insert_idx, dim3(blocks(ne)), dim3(TB), 0, st, keys, ekeys, n, (const uint8_t*)nullptr,
                       (const int32_t*)nullptr, eids, ne, n, tab, em, mask, shift, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, (uint32_t*)nullptr, sticky);
  hipLaunchKernelGGL(k_solo_insert_idx, dim3(blocks(n)), dim3(TB), 0, st, keys, ekeys, n, has_key, status,
                     contig ? ids : (const uint64_t*)nullptr, n, 0u, tab, (unsigned long long*)nullptr, mask, shift,
                     w.tpos.p, stays ? w.stay_cnt.p : (uint32_t*)nullptr, contig ? w.flag.p : (uint32_t*)nullptr,
                     sticky, plain_probe() ? 1u : 0u);
  // the stays rows' ordinals, dense, for the walk (stay_sorted: dd_plan's
  // buffer, free in a world of one); the walk's count is the groups' sum
  if (stays)
    hipLaunchKernelGGL(k_stays_write_t<kStayTile>, dim3(nt), dim3(TB), 0, st, has_key, status, n, w.stay_cnt.p,
                       w.stay_idx.p, ids, w.stay_sorted.p);
  hipLaunchKernelGGL(k_plan_walk, dim3(1), dim3(64), 0, st, (const uint64_t*)w.stay_sorted.p, (const uint32_t*)nullptr,
                     ids, stays ? n : 0u, (const uint32_t*)nullptr, win.n_total ? win.n_total : (uint64_t)n, cs,
                     win.max_steps, win.more, w.plan.p, stays ? w.stay_cnt.p + nt : (const uint32_t*)nullptr,
                     stay_groups(nt));
  if (stays && n >= kRrMin && (e = rr_index(w, w.plan.p, st))) return e;
  const uint64_t* emp = ne ? w.tkey.p : nullptr;
  auto apply = [&](auto kern, uint32_t r) {
    const uint32_t g = (uint32_t)(((uint64_t)n + (uint64_t)TB * r - 1) / ((uint64_t)TB * r));
    if (g) hipLaunchKernelGGL(kern, dim3(g), dim3(TB), 0, st, ids, w.tpos.p, n, tab, emp, cs, w.plan.p, link,
                              sharded ? w.shard.p : nullptr, contig ? (const uint32_t*)w.flag.p : nullptr, sticky,
                              (const uint64_t*)w.ridx.p);
  };
  switch (ar) {
    case 1: apply(k_solo_apply_r<1>, 1); break;
    case 2: apply(k_solo_apply_r<2>, 2); break;
    case 4: apply(k_solo_apply_r<4>, 4); break;
    case 8: apply(k_solo_apply_r<8>, 8); break;
    default:
      hipLaunchKernelGGL(k_solo_apply_idx, dim3(blocks(n) < 1024 ? blocks(n) : 1024), dim3(TB), 0, st, ids, w.tpos.p,
                         n, tab, emp, cs, w.plan.p, link, counts, sticky);
  }
  if (sharded) hipLaunchKernelGGL(k_counts_fold, dim3(1), dim3(kCountShards), 0, st, w.shard.p, counts);
  return sharded_done(w, sharded);
}

hipError_t dd_stays(DistWs& w, const uint8_t* has_key, const int32_t* status, const uint64_t* ids, uint32_t n,
                    uint32_t cap, uint64_t* out, int64_t* count, hipStream_t st) {
  hipError_t e;
  if ((e = w.nstay.ensure(1))) return e;
  if (n == 0 || (!has_key && !status)) {
    if ((e = hipMemsetAsync(w.nstay.p, 0, sizeof(uint32_t), st))) return e;
  } else {
    if ((e = select_stays(w, has_key, status, n, st))) return e;
  }
  const uint32_t g = cap ? cap : 1;
  hipLaunchKernelGGL(k_stays_gather, dim3(blocks(g)), dim3(TB), 0, st, w.stay_idx.p, w.nstay.p, ids, cap, out, count);
  return hipGetLastError();
}

// ---- the gathered stays list in order (dd_plan), without a library sort -------------
//
// Every rank's stays ordinals arrive concatenated; the plan walk needs them
// ascending. A list of at most kSortLds entries (the bucket protocol's
// 256 per rank) is sorted by one workgroup in LDS (bitonic); a longer one
// (the exact protocol with dense stays rows) becomes a bitmap over the
// job's ordinals [0, n_total) read back in order by the stays pass's own
// ordered compaction. Round 4 ran hipcub::DeviceRadixSort over the list.
constexpr uint32_t kSortLds = 4096;

__global__ void __launch_bounds__(1024) k_sort_small(const uint64_t* __restrict__ in, uint32_t m,
                                                     uint64_t* __restrict__ out) {
  __shared__ uint64_t v[kSortLds];
  const uint32_t tid = threadIdx.x;
  uint32_t P = 1;
  while (P < m) P <<= 1;
  for (uint32_t t = tid; t < P; t += 1024) v[t] = t < m ? in[t] : ~0ull;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = tid; t < P; t += 1024) {
        const uint32_t u = t ^ j;
        if (u > t) {
          const uint64_t a = v[t], b = v[u];
          if ((a > b) == ((t & k) == 0)) {
            v[t] = b;
            v[u] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t t = tid; t < m; t += 1024) out[t] = v[t];
}

__global__ void k_stays_bits(const uint64_t* __restrict__ in, uint32_t m, uint64_t n_total, uint32_t* __restrict__ bm) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint64_t p = in[j];
  if (p < n_total) atomicOr(&bm[p >> 5], 1u << (p & 31));
}

constexpr uint32_t kBitsR = 16, kBitsPer = TB * kBitsR;  // words per workgroup

__global__ void __launch_bounds__(TB) k_bits_count(const uint32_t* __restrict__ bm, uint64_t words,
                                                   uint32_t* __restrict__ bcnt) {
  __shared__ uint32_t ws[TB / 64];
  uint32_t c = 0;
#pragma unroll
  for (uint32_t r = 0; r < kBitsR; ++r) {
    const uint64_t w = (uint64_t)blockIdx.x * kBitsPer + r * TB + threadIdx.x;
    c += w < words ? (uint32_t)__popc(bm[w]) : 0u;
  }
#pragma unroll
  for (uint32_t d = 32; d; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// workgroup b's set bits, ascending, from the offset the workgroups before it
// add up to: thread t takes words [b * kBitsPer + t * kBitsR, + kBitsR)
__global__ void __launch_bounds__(TB) k_bits_write(const uint32_t* __restrict__ bm, uint64_t words,
                                                   const uint32_t* __restrict__ bcnt, uint64_t* __restrict__ out) {
  __shared__ uint32_t ws[TB / 64];
  const uint32_t b = blockIdx.x;
  if (bcnt[b] == 0) return;  // uniform over the workgroup
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t s = 0;
  for (uint32_t t = tid; t < b; t += TB) s += bcnt[t];
#pragma unroll
  for (uint32_t d = 32; d; d >>= 1) s += __shfl_xor(s, d);
  if (lane == 0) ws[wave] = s;
  __syncthreads();
  uint32_t run = ws[0] + ws[1] + ws[2] + ws[3];
  __syncthreads();
  const uint64_t w0 = (uint64_t)b * kBitsPer + (uint64_t)tid * kBitsR;
  uint32_t v[kBitsR], c = 0;
#pragma unroll
  for (uint32_t r = 0; r < kBitsR; ++r) {
    v[r] = w0 + r < words ? bm[w0 + r] : 0u;
    c += (uint32_t)__popc(v[r]);
  }
  uint32_t inc = c;  // the workgroup's exclusive prefix of c, in thread order
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(inc, d);
    if (lane >= d) inc += t;
  }
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  for (uint32_t w = 0; w < wave; ++w) run += ws[w];
  uint64_t at = run + inc - c;
#pragma unroll
  for (uint32_t r = 0; r < kBitsR; ++r) {
    uint32_t x = v[r];
    while (x) {
      const uint32_t bit = (uint32_t)__ffs(x) - 1;
      out[at++] = ((w0 + r) << 5) + bit;
      x &= x - 1;
    }
  }
}

hipError_t dd_plan(DistWs& w, const uint64_t* stays, uint32_t n_stays, uint64_t cs, const StepWindow& win,
                   uint64_t* plan, hipStream_t st) {
  hipError_t e;
  const uint64_t* sorted = stays;
  const uint32_t* tcnt = nullptr;
  uint32_t ntiles = 0;
  if (n_stays > 1 && win.n_total) {
    if ((e = w.stay_sorted.ensure(n_stays))) return e;
    if (n_stays <= kSortLds) {
      hipLaunchKernelGGL(k_sort_small, dim3(1), dim3(1024), 0, st, stays, n_stays, w.stay_sorted.p);
    } else {
      const uint64_t words = (win.n_total + 31) / 32;
      ntiles = (uint32_t)((words + kBitsPer - 1) / kBitsPer);
      if ((e = w.bitmap.ensure(words)) || (e = w.stay_cnt.ensure(ntiles + 1))) return e;
      if ((e = hipMemsetAsync(w.bitmap.p, 0, sizeof(uint32_t) * words, st))) return e;
      hipLaunchKernelGGL(k_stays_bits, dim3(blocks(n_stays)), dim3(TB), 0, st, stays, n_stays, win.n_total,
                         w.bitmap.p);
      hipLaunchKernelGGL(k_bits_count, dim3(ntiles), dim3(TB), 0, st, w.bitmap.p, words, w.stay_cnt.p);
      hipLaunchKernelGGL(k_bits_write, dim3(ntiles), dim3(TB), 0, st, w.bitmap.p, words, w.stay_cnt.p,
                         w.stay_sorted.p);
      tcnt = w.stay_cnt.p;
    }
    sorted = w.stay_sorted.p;
  }
  hipLaunchKernelGGL(k_plan_walk, dim3(1), dim3(64), 0, st, sorted, (const uint32_t*)nullptr,
                     (const uint64_t*)nullptr, n_stays, (const uint32_t*)nullptr, win.n_total, cs, win.max_steps,
                     win.more, plan, tcnt, ntiles);
  if (n_stays >= kRrMin && (e = rr_index(w, plan, st))) return e;
  return hipGetLastError();
}

hipError_t dd_local(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                    const uint64_t* ids, uint32_t n, const uint64_t* ekeys, const uint64_t* eids, uint32_t ne,
                    uint64_t chunk_size, const StepWindow& win, int64_t* link, unsigned long long* counts,
                    hipStream_t st) {
  hipError_t e;
  if (chunk_size == 0) chunk_size = 100;
  // the steps' plan from this batch's stays rows (all of the job's: a world of one)
  if ((e = w.nstay.ensure(1)) || (e = w.plan.ensure(kPlanHeader + (uint64_t)n + 1))) return e;
  const DedupTable table = dedup_table();
  if (n && table == kTableIdx) {
    const uint64_t cap = local_cap((uint64_t)n + ne);
    if (cap > (1ull << 31)) return hipErrorInvalidValue;
    return local_fused(w, keys, has_key, status, ids, n, ekeys, eids, ne, chunk_size, win, link, counts, cap, st);
  }
  if (n && (has_key || status)) {
    if ((e = select_stays(w, has_key, status, n, st))) return e;
  } else if ((e = hipMemsetAsync(w.nstay.p, 0, sizeof(uint32_t), st))) {
    return e;
  }
  hipLaunchKernelGGL(k_plan_walk, dim3(1), dim3(64), 0, st, (const uint64_t*)nullptr, w.stay_idx.p, ids, n,
                     w.nstay.p, win.n_total ? win.n_total : (uint64_t)n, chunk_size, win.max_steps, win.more, w.plan.p);
  if (n == 0) return hipGetLastError();
  const uint64_t cap = local_cap((uint64_t)n + ne);
  if (cap > (1ull << 31)) return hipErrorInvalidValue;
  if (table == kTableIdx4) {
    const uint32_t mask = (uint32_t)(cap - 1);
    const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(cap);
    // the u32 table borrows tmin's storage (cap u32 = cap / 4 of its u64);
    // the existing Objects' minima live in tkey (cap u64), when there are any
    if ((e = w.tmin.ensure(cap / 2 + 1)) || (e = w.tpos.ensure(n)) || (ne && (e = w.tkey.ensure(cap + 1)))) return e;
    auto* tab = reinterpret_cast<uint32_t*>(w.tmin.p);
    auto* em = ne ? reinterpret_cast<unsigned long long*>(w.tkey.p) : nullptr;
    if ((e = hipMemsetAsync(tab, 0xFF, sizeof(uint32_t) * cap, st)) ||
        (ne && (e = hipMemsetAsync(em, 0xFF, sizeof(uint64_t) * cap, st))))
      return e;
    if (ne)
      hipLaunchKernelGGL(k_solo_insert_idx, dim3(blocks(ne)), dim3(TB), 0, st, keys, ekeys, n,
                         (const uint8_t*)nullptr, (const int32_t*)nullptr, eids, ne, n, tab, em, mask, shift,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr, kIdxEmpty);
    hipLaunchKernelGGL(k_solo_insert_idx, dim3(blocks(n)), dim3(TB), 0, st, keys, ekeys, n, has_key, status,
                       (const uint64_t*)nullptr, n, 0u, tab, (unsigned long long*)nullptr, mask, shift, w.tpos.p,
                       (uint32_t*)nullptr, (uint32_t*)nullptr, kIdxEmpty);
    hipLaunchKernelGGL(k_solo_apply_idx, dim3(blocks(n) < 1024 ? blocks(n) : 1024), dim3(TB), 0, st, ids, w.tpos.p, n,
                       tab, ne ? w.tkey.p : nullptr, chunk_size, w.plan.p, link, counts, kIdxEmpty);
    return hipGetLastError();
  }
  // (key, file minimum) pairs in tmin, existing minima in tkey (when ne > 0)
  if ((e = w.tmin.ensure(2 * (cap + 1))) || (e = w.tpos.ensure(n)) || (ne && (e = w.tkey.ensure(cap + 1)))) return e;
  const uint32_t mask = (uint32_t)(cap - 1);
  const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(cap);
  if ((e = hipMemsetAsync(w.tmin.p, 0xFF, sizeof(uint64_t) * 2 * (cap + 1), st)) ||
      (ne && (e = hipMemsetAsync(w.tkey.p, 0xFF, sizeof(uint64_t) * (cap + 1), st))))
    return e;
  auto* tab = reinterpret_cast<unsigned long long*>(w.tmin.p);
  auto* em = ne ? reinterpret_cast<unsigned long long*>(w.tkey.p) : nullptr;
  if (ne)
    hipLaunchKernelGGL(k_solo_insert, dim3(blocks(ne)), dim3(TB), 0, st, ekeys, nullptr, nullptr, eids, ne, tab, em,
                       mask, shift, nullptr);
  hipLaunchKernelGGL(k_solo_insert, dim3(blocks(n)), dim3(TB), 0, st, keys, has_key, status, ids, n, tab,
                     (unsigned long long*)nullptr, mask, shift, w.tpos.p);
  hipLaunchKernelGGL(k_solo_apply, dim3(blocks(n) < 1024 ? blocks(n) : 1024), dim3(TB), 0, st, ids, w.tpos.p, n,
                     w.tmin.p, ne ? w.tkey.p : nullptr, chunk_size, w.plan.p, link, counts);
  return hipGetLastError();
}

hipError_t dd_apply(DistWs& w, const uint64_t* ids, const uint32_t* slot, uint32_t n, const int64_t* result,
                    uint64_t chunk_size, const uint64_t* plan, int64_t* link, unsigned long long* counts,
                    hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t cs = chunk_size ? chunk_size : 100;
  const uint32_t ar = apply_files_per_thread();
  hipError_t e;
  if (ar && counts && (e = shard_counts(w, st))) return e;
  unsigned long long* sh = ar && counts ? w.shard.p : nullptr;
  auto apply = [&](auto kern, uint32_t r) {
    const uint32_t g = (uint32_t)(((uint64_t)n + (uint64_t)TB * r - 1) / ((uint64_t)TB * r));
    hipLaunchKernelGGL(kern, dim3(g), dim3(TB), 0, st, ids, slot, n, result, cs, plan, link, sh,
                       (const uint64_t*)w.ridx.p);
  };
  switch (ar) {
    case 1: apply(k_dd_apply_r<1>, 1); break;
    case 2: apply(k_dd_apply_r<2>, 2); break;
    case 4: apply(k_dd_apply_r<4>, 4); break;
    case 8: apply(k_dd_apply_r<8>, 8); break;
    default:
      hipLaunchKernelGGL(k_dd_apply, dim3(blocks(n) < 1024 ? blocks(n) : 1024), dim3(TB), 0, st, ids, slot, n, result,
                         cs, plan, link, counts);
  }
  if (sh) hipLaunchKernelGGL(k_counts_fold, dim3(1), dim3(kCountShards), 0, st, sh, counts);
  return sharded_done(w, sh != nullptr);
}

// The compact table of the files' keys (each key's lowest file index) in
// w.idx_a, each file's slot in w.idx_b: the first step of both combines.
static hipError_t combine_table(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                                uint32_t n, uint32_t world, hipStream_t st) {
  uint64_t tcap = 1024;
  while (tcap < 2 * (uint64_t)n) tcap <<= 1;
  if (tcap > (1ull << 31)) return hipErrorInvalidValue;
  hipError_t e;
  if ((e = w.idx_a.ensure(tcap)) || (e = w.idx_b.ensure(n)) || (e = w.tpos.ensure(n)) ||
      (e = w.starts.ensure(world + 1)) || (e = w.ocnt.ensure(world + 1)))
    return e;
  const uint32_t mask = (uint32_t)(tcap - 1);
  const uint32_t shift = 64u - (uint32_t)__builtin_ctzll(tcap);
  if ((e = hipMemsetAsync(w.idx_a.p, 0xFF, sizeof(uint32_t) * tcap, st)) ||
      (e = hipMemsetAsync(w.ocnt.p, 0, sizeof(uint32_t) * (world + 1), st)))
    return e;
  hipLaunchKernelGGL(k_solo_insert_idx, dim3(blocks(n)), dim3(TB), 0, st, keys, (const uint64_t*)nullptr, n, has_key,
                     status, (const uint64_t*)nullptr, n, 0u, w.idx_a.p, (unsigned long long*)nullptr, mask, shift,
                     w.idx_b.p, (uint32_t*)nullptr, (uint32_t*)nullptr, kIdxEmpty);
  return hipGetLastError();
}

static uint32_t emit_grid(uint32_t n) { return (uint32_t)((n + TB * kEmitR - 1) / (TB * kEmitR)); }

// the exact layout (dd_combine): owner r's records at [starts[r],
// starts[r+1]) in no particular order, slot[i] = the record of file i's key.
// Round 5: the bucket combine's table and emit, the owners' record counts
// taken by a first emit pass, in place of round 4's stable radix sort and
// scans (hipCUB), the library's last CUB-API dependency with the stays sort
// (dd_plan)
static hipError_t combine_core(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                               const uint64_t* ids, uint32_t n, uint32_t world, uint64_t* rec, uint32_t* slot,
                               hipStream_t st) {
  hipError_t e;
  if ((e = combine_table(w, keys, has_key, status, n, world, st))) return e;
  hipLaunchKernelGGL(k_cb_emit, dim3(emit_grid(n)), dim3(TB), 0, st, keys, ids, n, w.idx_b.p, w.idx_a.p, world, ~0u,
                     (const uint32_t*)nullptr, 1u, w.ocnt.p, (uint64_t*)nullptr, (uint32_t*)nullptr,
                     (uint32_t*)nullptr);
  hipLaunchKernelGGL(k_owner_starts, dim3(1), dim3(1024), 0, st, w.ocnt.p, world, w.starts.p);
  if ((e = hipMemsetAsync(w.ocnt.p, 0, sizeof(uint32_t) * (world + 1), st))) return e;
  hipLaunchKernelGGL(k_cb_emit, dim3(emit_grid(n)), dim3(TB), 0, st, keys, ids, n, w.idx_b.p, w.idx_a.p, world, ~0u,
                     (const uint32_t*)w.starts.p, 0u, w.ocnt.p, rec, w.tpos.p, (uint32_t*)nullptr);
  if (slot) hipLaunchKernelGGL(k_cb_slot, dim3(blocks(n)), dim3(TB), 0, st, w.idx_b.p, w.idx_a.p, w.tpos.p, n, slot);
  return hipGetLastError();
}

// SDCAS_COMBINE=hash: the bucket combine through the rank's global table
// (round 5: one record per key) instead of the per-tile LDS pre-aggregation
// (the default), read per call (A/B in one process)
static bool combine_by_tile() {
  const char* v = getenv("SDCAS_COMBINE");
  return !(v && strcmp(v, "hash") == 0);
}

hipError_t dd_combine_buckets(DistWs& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                              const uint64_t* ids, uint32_t n, uint32_t world, uint32_t cap, uint64_t* send,
                              uint32_t* slot, int64_t* counts, uint32_t* overflow, hipStream_t st) {
  hipError_t e;
  if (n == 0) {
    if ((e = hipMemsetAsync(overflow, 0, sizeof(uint32_t), st))) return e;
    return hipMemsetAsync(counts, 0, sizeof(int64_t) * world, st);
  }
  if (combine_by_tile()) {
    if ((e = w.ocnt.ensure(world + 1))) return e;
    hipLaunchKernelGGL(k_cb_prep, dim3(1), dim3(TB), 0, st, w.ocnt.p, world, overflow);
    hipLaunchKernelGGL(k_cb_tile, dim3((n + kTileN - 1) / kTileN), dim3(TB), 0, st, keys, has_key, status, ids, n,
                       world, cap, w.ocnt.p, send, slot, overflow);
    hipLaunchKernelGGL(k_cb_counts, dim3(blocks(world)), dim3(TB), 0, st, w.ocnt.p, world, cap, counts);
    return hipGetLastError();
  }
  if ((e = hipMemsetAsync(overflow, 0, sizeof(uint32_t), st))) return e;
  if ((e = combine_table(w, keys, has_key, status, n, world, st))) return e;
  hipLaunchKernelGGL(k_cb_emit, dim3(emit_grid(n)), dim3(TB), 0, st, keys, ids, n, w.idx_b.p, w.idx_a.p, world, cap,
                     (const uint32_t*)nullptr, 0u, w.ocnt.p, send, w.tpos.p, overflow);
  hipLaunchKernelGGL(k_cb_counts, dim3(blocks(world)), dim3(TB), 0, st, w.ocnt.p, world, cap, counts);
  if (slot) hipLaunchKernelGGL(k_cb_slot, dim3(blocks(n)), dim3(TB), 0, st, w.idx_b.p, w.idx_a.p, w.tpos.p, n, slot);
  return hipGetLastError();
}

}  // namespace sdcas
