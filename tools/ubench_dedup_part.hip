// ubench_dedup_part.hip — the single-rank group-by's resolve (per key: the
// lowest file ordinal) two ways, on a C5-shaped key set (measurement tool,
// not product code):
//   table: what dd_local does — an open-addressing table of 2^k >= 2n
//          16-byte entries in HBM (memset, CAS insert + atomicMin, then every
//          file reads its entry);
//   part:  the records partitioned by their top key bits into LDS-sized
//          buckets (per-block histograms, a scan, a scatter), each bucket
//          resolved by one workgroup in an LDS table, answers written per
//          file.
// Prints the time of each and checks that both give every file the same
// answer.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr uint64_t kEmpty = ~0ull;

// ---- table ------------------------------------------------------------------
__global__ void k_tab_insert(const uint64_t* __restrict__ keys, uint32_t n, unsigned long long* __restrict__ tab,
                             uint32_t mask, uint32_t shift, uint32_t* __restrict__ pos) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  uint32_t h = (uint32_t)(key >> shift) & mask;
  for (;;) {
    const unsigned long long cur = __hip_atomic_load(&tab[2 * (uint64_t)h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) break;
    if (cur == kEmpty) {
      const unsigned long long prev = atomicCAS(&tab[2 * (uint64_t)h], kEmpty, (unsigned long long)key);
      if (prev == kEmpty || prev == key) break;
    }
    h = (h + 1) & mask;
  }
  unsigned long long* m = &tab[2 * (uint64_t)h + 1];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > i) atomicMin(m, (unsigned long long)i);
  pos[i] = h;
}
__global__ void k_tab_answer(const uint32_t* __restrict__ pos, uint32_t n, const uint64_t* __restrict__ tab,
                             int64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (int64_t)tab[2 * (uint64_t)pos[i] + 1];
}

// ---- part -------------------------------------------------------------------
constexpr int kG = 512;          // partition blocks
constexpr int kPT = 512;         // threads per partition block
constexpr int kMaxBits = 13;     // at most 8192 buckets (the block histogram lives in LDS)
constexpr int kTab = 2048;       // LDS table entries per bucket workgroup

__global__ void __launch_bounds__(kPT) k_part_count(const uint64_t* __restrict__ keys, uint32_t n, uint32_t bits,
                                                    uint32_t* __restrict__ M) {
  __shared__ uint32_t hist[1 << kMaxBits];
  const uint32_t nb = 1u << bits;
  for (uint32_t b = threadIdx.x; b < nb; b += kPT) hist[b] = 0;
  __syncthreads();
  const uint64_t per = (n + kG - 1) / kG;
  const uint64_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += kPT) atomicAdd(&hist[bits ? keys[i] >> (64 - bits) : 0], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += kPT) M[(uint64_t)b * kG + blockIdx.x] = hist[b];
}

__global__ void __launch_bounds__(kPT) k_part_scatter(const uint64_t* __restrict__ keys, uint32_t n, uint32_t bits,
                                                      const uint32_t* __restrict__ Ms, uint64_t* __restrict__ pkey,
                                                      uint32_t* __restrict__ pidx) {
  __shared__ uint32_t cur[1 << kMaxBits];
  const uint32_t nb = 1u << bits;
  for (uint32_t b = threadIdx.x; b < nb; b += kPT) cur[b] = Ms[(uint64_t)b * kG + blockIdx.x];
  __syncthreads();
  const uint64_t per = (n + kG - 1) / kG;
  const uint64_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += kPT) {
    const uint64_t k = keys[i];
    const uint32_t p = atomicAdd(&cur[bits ? k >> (64 - bits) : 0], 1u);
    pkey[p] = k;
    pidx[p] = (uint32_t)i;
  }
}

// one workgroup per bucket; keys of the bucket share their top `bits` bits,
// so the LDS home slot comes from the bits below them
__global__ void __launch_bounds__(256) k_part_bucket(const uint64_t* __restrict__ pkey, const uint32_t* __restrict__ pidx,
                                                     const uint32_t* __restrict__ Ms, uint32_t n, uint32_t bits,
                                                     int64_t* __restrict__ out, uint32_t* __restrict__ overflow) {
  __shared__ unsigned long long tk[kTab];
  __shared__ uint32_t tm[kTab];
  const uint32_t b = blockIdx.x, nb = 1u << bits;
  const uint32_t s0 = Ms[(uint64_t)b * kG], s1 = b + 1 < nb ? Ms[(uint64_t)(b + 1) * kG] : n;
  for (uint32_t t = threadIdx.x; t < kTab; t += 256) {
    tk[t] = kEmpty;
    tm[t] = 0xFFFFFFFFu;
  }
  __syncthreads();
  const uint32_t sh = 64 - bits - 11;  // 11 = log2(kTab)
  for (uint32_t p = s0 + threadIdx.x; p < s1; p += 256) {
    const uint64_t k = pkey[p];
    uint32_t h = (uint32_t)(k >> sh) & (kTab - 1);
    uint32_t probes = 0;
    for (;; h = (h + 1) & (kTab - 1)) {
      const unsigned long long c = tk[h];
      if (c == k) break;
      if (c == kEmpty) {
        const unsigned long long prev = atomicCAS(&tk[h], kEmpty, (unsigned long long)k);
        if (prev == kEmpty || prev == k) break;
      }
      if (++probes == kTab) {  // table full: flagged (the product would take another path)
        atomicOr(overflow, 1u);
        h = kTab;
        break;
      }
    }
    if (h < kTab) atomicMin(&tm[h], pidx[p]);
  }
  __syncthreads();
  for (uint32_t p = s0 + threadIdx.x; p < s1; p += 256) {
    const uint64_t k = pkey[p];
    uint32_t h = (uint32_t)(k >> sh) & (kTab - 1), probes = 0;
    while (tk[h] != k && ++probes < kTab) h = (h + 1) & (kTab - 1);
    out[pidx[p]] = tk[h] == k ? (int64_t)tm[h] : -1;
  }
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 6250000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  // C5-shaped: 40 % of the files distinct contents, 60 % drawn Zipf(1.1) over them
  std::mt19937_64 rng(5);
  const uint32_t distinct = (uint32_t)(n * 0.4);
  std::vector<double> cdf(distinct);
  double acc = 0;
  for (uint32_t c = 0; c < distinct; ++c) cdf[c] = (acc += 1.0 / std::pow((double)c + 1, 1.1));
  std::vector<uint64_t> h_keys(n);
  auto mix = [](uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; return x ^ (x >> 31);
  };
  std::uniform_real_distribution<double> U(0, acc);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t cid = i < distinct ? i : (uint64_t)(std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin());
    h_keys[i] = mix(cid + 0x5D0005);
  }
  std::shuffle(h_keys.begin(), h_keys.end(), rng);
  uint64_t* keys;
  CK(hipMalloc(&keys, 8ull * n));
  CK(hipMemcpy(keys, h_keys.data(), 8ull * n, hipMemcpyHostToDevice));
  // table
  uint64_t cap = 1024;
  while (cap < 2ull * n) cap <<= 1;
  unsigned long long* tab;
  uint32_t* pos;
  int64_t *out_t, *out_p;
  CK(hipMalloc(&tab, 16 * cap));
  CK(hipMalloc(&pos, 4ull * n));
  CK(hipMalloc(&out_t, 8ull * n));
  CK(hipMalloc(&out_p, 8ull * n));
  const uint32_t mask = (uint32_t)(cap - 1), shift = 64u - (uint32_t)__builtin_ctzll(cap);
  // part
  uint32_t bits = 0;
  while (bits < (uint32_t)kMaxBits && ((uint64_t)n >> bits) > 768) ++bits;
  const uint32_t nb = 1u << bits;
  uint32_t *M, *Ms, *pidx, *ovf;
  uint64_t* pkey;
  CK(hipMalloc(&M, 4ull * nb * kG));
  CK(hipMalloc(&Ms, 4ull * nb * kG));
  CK(hipMalloc(&pkey, 8ull * n));
  CK(hipMalloc(&pidx, 4ull * n));
  CK(hipMalloc(&ovf, 4));
  size_t tmp = 0;
  CK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, M, Ms, (int)(nb * kG)));
  void* dtmp;
  CK(hipMalloc(&dtmp, tmp + 256));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  std::vector<float> tt, tp;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipEventRecord(e0));
    CK(hipMemsetAsync(tab, 0xFF, 16 * cap));
    hipLaunchKernelGGL(k_tab_insert, dim3((n + 255) / 256), dim3(256), 0, 0, keys, n, tab, mask, shift, pos);
    hipLaunchKernelGGL(k_tab_answer, dim3((n + 255) / 256), dim3(256), 0, 0, pos, n, (const uint64_t*)tab, out_t);
    CK(hipEventRecord(e1));
    CK(hipMemsetAsync(ovf, 0, 4));
    hipLaunchKernelGGL(k_part_count, dim3(kG), dim3(kPT), 0, 0, keys, n, bits, M);
    size_t t2 = tmp;
    CK(hipcub::DeviceScan::ExclusiveSum(dtmp, t2, M, Ms, (int)(nb * kG)));
    hipLaunchKernelGGL(k_part_scatter, dim3(kG), dim3(kPT), 0, 0, keys, n, bits, Ms, pkey, pidx);
    hipLaunchKernelGGL(k_part_bucket, dim3(nb), dim3(256), 0, 0, pkey, pidx, Ms, n, bits, out_p, ovf);
    CK(hipEventRecord(e2));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    if (r) tt.push_back(a), tp.push_back(b);
  }
  std::vector<int64_t> ht(n), hp(n);
  CK(hipMemcpy(ht.data(), out_t, 8ull * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hp.data(), out_p, 8ull * n, hipMemcpyDeviceToHost));
  uint32_t o = 0;
  CK(hipMemcpy(&o, ovf, 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (uint32_t i = 0; i < n; ++i) bad += ht[i] != hp[i];
  std::sort(tt.begin(), tt.end());
  std::sort(tp.begin(), tp.end());
  printf("{\"n\": %u, \"buckets\": %u, \"table_ms_median\": %.4f, \"part_ms_median\": %.4f, \"mismatches\": %zu, "
         "\"overflow\": %u}\n", n, nb, tt[tt.size() / 2], tp[tp.size() / 2], bad, o);
  return bad || o ? 1 : 0;
}
