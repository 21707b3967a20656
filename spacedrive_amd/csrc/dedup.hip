// dedup.hip — cas_id -> Object group-by/link on the device.
//
// Replaces the per-chunk logic of core/src/object/file_identifier/mod.rs:
//   :149-154  unique_cas_ids HashSet
//   :181-198  existing Objects whose file_paths carry one of those cas_ids
//   :202-238  link each file to the FIRST such Object (linear find :214-224)
//   :246-254  every other file (None cas_id, or unseen cas_id — intra-chunk
//             duplicates included) gets a new Object
// applied over consecutive 100-file chunks (mod.rs:34,
// file_identifier_job.rs:296-319). Canonical form: the
// first Object of a key is the one created by its lowest-index file, so the
// sequential chunk loop collapses to a sort:
//   rep(X)    = lowest file index with key X
//   link(i)   = i              if i is in rep(X)'s chunk (created there)
//             = rep(X)         otherwise (a later chunk links to it)
//             = -(e+1)         if X is carried by existing Object e (first in DB order)
// HBM-bound integer work: one radix sort of (key, index) pairs plus streaming
// passes; no atomics.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdint.h>

#include "dedup.h"

namespace sdcas {

__global__ void k_dedup_prepare(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ has_key,
                                const int32_t* __restrict__ status, uint32_t n, uint8_t* __restrict__ valid,
                                int64_t* __restrict__ out_link, uint32_t* __restrict__ idx) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool ok = status == nullptr || status[i] == 0;
  const bool v = ok && has_key[i];
  valid[i] = v;
  idx[i] = i;
  // dropped files (mod.rs:125-141) and None cas_ids (mod.rs:83-86, :246-254)
  out_link[i] = ok ? (int64_t)i : INT64_MIN;
}

// After sorting valid (key, idx) pairs by key (stable: idx ascending inside a
// key run), mark run heads.
__global__ void k_dedup_heads(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ nvalid_p,
                              uint32_t* __restrict__ headpos) {
  const uint32_t nv = *nvalid_p;
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nv) return;
  headpos[p] = (p == 0 || skeys[p] != skeys[p - 1]) ? p : 0u;
}

// existing Objects: sorted (key, e) pairs, stable, so the first e of a key
// run is the first Object in DB order
__device__ __forceinline__ int64_t find_existing(const uint64_t* ekeys, const uint32_t* eidx, uint32_t ne,
                                                 uint64_t key) {
  uint32_t lo = 0, hi = ne;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (ekeys[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < ne && ekeys[lo] == key) ? (int64_t)eidx[lo] : -1;
}

__global__ void k_dedup_link(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ sidx,
                             const uint32_t* __restrict__ headscan, const uint32_t* __restrict__ nvalid_p,
                             const uint64_t* __restrict__ ekeys, const uint32_t* __restrict__ eidx, uint32_t ne,
                             uint32_t chunk_size, int64_t* __restrict__ out_link) {
  const uint32_t nv = *nvalid_p;
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nv) return;
  const uint32_t i = sidx[p];
  const uint32_t h = headscan[p];
  const uint32_t rep = sidx[h];
  const int64_t e = ne ? find_existing(ekeys, eidx, ne, skeys[p]) : -1;
  int64_t link;
  if (e >= 0) link = -(e + 1);
  else if (i / chunk_size == rep / chunk_size) link = (int64_t)i;
  else link = (int64_t)rep;
  out_link[i] = link;
}

__global__ void k_dedup_count(const int64_t* __restrict__ out_link, const uint8_t* __restrict__ valid, uint32_t n,
                              unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long sc[2];
  if (threadIdx.x < 2) sc[threadIdx.x] = 0;
  __syncthreads();
  // grid-stride over a bounded grid: one global atomic pair per workgroup
  // (thousands of workgroups adding to one address serialise in L2)
  unsigned long long c = 0, l = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int64_t v = out_link[i];
    if (v == (int64_t)i) c += 1;
    else if (v != INT64_MIN && valid[i]) l += 1;
  }
  // wave-level sums, then one LDS atomic per wave
  for (int off = 32; off > 0; off >>= 1) {
    c += __shfl_down(c, off);
    l += __shfl_down(l, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&sc[0], c);
    atomicAdd(&sc[1], l);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&counts[0], sc[0]);
    atomicAdd(&counts[1], sc[1]);
  }
}

__global__ void k_iota32(uint32_t* p, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

struct MaxOp {
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};

size_t DedupWorkspace::temp_bytes_for(uint32_t n) {
  size_t a = 0, b = 0, c = 0, d = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, a, (const uint64_t*)nullptr, (const uint8_t*)nullptr,
                                      (uint64_t*)nullptr, (uint32_t*)nullptr, (int)n);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, MaxOp(),
                                          (int)n);
  d = a > b ? a : b;
  return d > c ? d : c;
}

hipError_t dedup_run(DedupWorkspace& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                     uint32_t n, uint32_t chunk_size, const uint64_t* ekeys_sorted, const uint32_t* eidx_sorted,
                     uint32_t ne, int64_t* out_link, unsigned long long* d_counts, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint32_t tb = 256, nb = (n + tb - 1) / tb;
  hipError_t e;
  hipLaunchKernelGGL(k_dedup_prepare, dim3(nb), dim3(tb), 0, st, keys, has_key, status, n, w.valid, out_link,
                     w.idx_a);
  // compact valid entries (key, file index); the tail past nvalid keeps
  // UINT64_MAX keys so that sorting all n slots (nvalid is not known on the
  // host without a sync) leaves the real entries first: the radix sort is
  // stable and the fillers come after every real entry in input order.
  if ((e = hipMemsetAsync(w.key_a, 0xFF, sizeof(uint64_t) * n, st))) return e;
  size_t tmp = w.temp_bytes;
  if ((e = hipcub::DeviceSelect::Flagged(w.temp, tmp, keys, w.valid, w.key_a, w.nvalid, (int)n, st))) return e;
  tmp = w.temp_bytes;
  if ((e = hipcub::DeviceSelect::Flagged(w.temp, tmp, w.idx_a, w.valid, w.idx_b, w.nvalid, (int)n, st))) return e;
  // stable sort by key: file order is kept inside a key run
  tmp = w.temp_bytes;
  if ((e = hipcub::DeviceRadixSort::SortPairs(w.temp, tmp, w.key_a, w.key_b, w.idx_b, w.idx_a, (int)n, 0, 64,
                                              st)))
    return e;
  hipLaunchKernelGGL(k_dedup_heads, dim3(nb), dim3(tb), 0, st, w.key_b, w.nvalid, w.head);
  tmp = w.temp_bytes;
  if ((e = hipcub::DeviceScan::InclusiveScan(w.temp, tmp, w.head, w.head, MaxOp(), (int)n, st))) return e;
  hipLaunchKernelGGL(k_dedup_link, dim3(nb), dim3(tb), 0, st, w.key_b, w.idx_a, w.head, w.nvalid, ekeys_sorted,
                     eidx_sorted, ne, chunk_size, out_link);
  if (d_counts) {
    (void)hipMemsetAsync(d_counts, 0, 2 * sizeof(unsigned long long), st);
    hipLaunchKernelGGL(k_dedup_count, dim3(std::min<uint32_t>(nb, 1024)), dim3(tb), 0, st, out_link, w.valid, n,
                       d_counts);
  }
  return hipGetLastError();
}

hipError_t dedup_sort_existing(DedupWorkspace& w, const uint64_t* ekeys, uint32_t ne, uint64_t* ekeys_sorted,
                               uint32_t* eidx_sorted, hipStream_t st) {
  if (ne == 0) return hipSuccess;
  const uint32_t tb = 256;
  hipLaunchKernelGGL(k_iota32, dim3((ne + tb - 1) / tb), dim3(tb), 0, st, w.idx_b, ne);
  size_t tmp = w.temp_bytes;
  return hipcub::DeviceRadixSort::SortPairs(w.temp, tmp, ekeys, ekeys_sorted, w.idx_b, eidx_sorted, (int)ne, 0, 64,
                                            st);
}

}  // namespace sdcas
