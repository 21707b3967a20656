// Random-access rate of one MI355X: what a hash join like the identifier
// dedup (dist_dedup.hip) can be priced against. For tables of 16 MiB .. 1 GiB
// of u32 slots: (a) independent random 4-byte loads (a gather), (b) random
// 32-bit CAS with return (an insert's claim), (c) a load followed by a
// dependent load at the address it returned (an insert's read-back of the
// key through the index), (d) random no-return atomicMin; every thread one
// request (or chain) of 64 M, addresses from a mixing hash of the thread
// index (uniform, like BLAKE3 keys). Prints G requests/s per case.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_gather.hip -o tools/ubench_gather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(x ^ (x >> 31));
}

__global__ void k_gather(const uint32_t* __restrict__ t, uint32_t mask, uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = __hip_atomic_load(&t[mix(i) & mask], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_cas(uint32_t* __restrict__ t, uint32_t mask, uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = atomicCAS(&t[mix(i) & mask], 0xFFFFFFFFu, (uint32_t)i);
}

__global__ void k_chain(const uint32_t* __restrict__ t, uint32_t mask, uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = __hip_atomic_load(&t[mix(i) & mask], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  out[i] = t[mix(a + i) & mask];
}

__global__ void k_min(uint32_t* __restrict__ t, uint32_t mask, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicMin(&t[mix(i) & mask], (uint32_t)i);
}

__global__ void k_fill(uint32_t* t, uint64_t n, uint32_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = v ^ (uint32_t)i;
}

int main() {
  const uint64_t n = 64ull << 20;  // requests per launch
  uint32_t *t, *out;
  CK(hipMalloc(&t, 1ull << 30));
  CK(hipMalloc(&out, n * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((uint32_t)((n + 255) / 256)), b(256);
  std::printf("{\"requests_per_launch\": %llu, \"cases\": [\n", (unsigned long long)n);
  bool first = true;
  for (int lg = 22; lg <= 28; lg += 2) {
    const uint64_t slots = 1ull << lg;
    const uint32_t mask = (uint32_t)(slots - 1);
    const char* names[] = {"gather", "cas", "chain", "atomic_min"};
    for (int c = 0; c < 4; ++c) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, t, slots, c == 1 ? 0xFFFFFFFFu : 0x12345u);
        if (c == 1) CK(hipMemset(t, 0xFF, slots * 4));
        CK(hipEventRecord(e0));
        if (c == 0) hipLaunchKernelGGL(k_gather, g, b, 0, 0, t, mask, n, out);
        if (c == 1) hipLaunchKernelGGL(k_cas, g, b, 0, 0, t, mask, n, out);
        if (c == 2) hipLaunchKernelGGL(k_chain, g, b, 0, 0, t, mask, n, out);
        if (c == 3) hipLaunchKernelGGL(k_min, g, b, 0, 0, t, mask, n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      const double reqs = (double)n * (c == 2 ? 2 : 1);
      std::printf("%s {\"table_mib\": %llu, \"case\": \"%s\", \"ms\": %.3f, \"g_requests_per_s\": %.1f}", first ? "" : ",\n",
                  (unsigned long long)(slots * 4 >> 20), names[c], best, reqs / best / 1e6);
      first = false;
    }
  }
  std::printf("\n]}\n");
  return 0;
}
