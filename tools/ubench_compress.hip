// ubench_compress.hip — BLAKE3 compression throughput on gfx950 with
// alternative instruction selections (measurement tool, not product code).
// Register-only: each lane runs dependent compressions (2 independent streams
// per lane), 8 waves per SIMD; prints G compressions/s per variant and checks
// every variant against the reference G (b3_device.h) bit-exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../spacedrive_amd/csrc/b3_device.h"

using namespace b3d;

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t xr(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t rot_shift(uint32_t x) {  // 3 full-rate ops
  uint32_t lo, hi, r;
  asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(lo) : "i"(N), "v"(x));
  asm volatile("v_lshlrev_b32 %0, %1, %2" : "=v"(hi) : "i"(32 - N), "v"(x));
  asm volatile("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t rot_align(uint32_t x) {
  return __builtin_amdgcn_alignbit(x, x, N);
}
// xor then rotate, the rotate's OR fused with... nothing: plain forms
template <int N>
__device__ __forceinline__ uint32_t xrot_shift_bitop(uint32_t d, uint32_t a) {
  // t = d ^ a; lo = t >> N; hi = t << (32-N); r = lo | hi  (4 full-rate ops)
  uint32_t t = d ^ a, lo, hi, r;
  asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(lo) : "i"(N), "v"(t));
  asm volatile("v_lshlrev_b32 %0, %1, %2" : "=v"(hi) : "i"(32 - N), "v"(t));
  asm volatile("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// VAR: 0 reference (add3 + alignbit); 1 add3 -> 2 adds; 2 rot12/rot7 by shifts;
// 3 all rotations by shifts; 4 = 1 + 2
template <int VAR>
__device__ __forceinline__ void G(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
  if (VAR == 1 || VAR == 4) a = add2(add2(a, b), x);
  else a = a + b + x;
  d = (VAR == 3) ? rot_shift<16>(d ^ a) : rot_align<16>(d ^ a);
  c = c + d;
  b = (VAR >= 2) ? rot_shift<12>(b ^ c) : rot_align<12>(b ^ c);
  if (VAR == 1 || VAR == 4) a = add2(add2(a, b), y);
  else a = a + b + y;
  d = (VAR == 3) ? rot_shift<8>(d ^ a) : rot_align<8>(d ^ a);
  c = c + d;
  b = (VAR >= 2) ? rot_shift<7>(b ^ c) : rot_align<7>(b ^ c);
}

#define RND(V, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  G<V>(v0, v4, v8, v12, m[s0], m[s1]);                                                  \
  G<V>(v1, v5, v9, v13, m[s2], m[s3]);                                                  \
  G<V>(v2, v6, v10, v14, m[s4], m[s5]);                                                 \
  G<V>(v3, v7, v11, v15, m[s6], m[s7]);                                                 \
  G<V>(v0, v5, v10, v15, m[s8], m[s9]);                                                 \
  G<V>(v1, v6, v11, v12, m[s10], m[s11]);                                               \
  G<V>(v2, v7, v8, v13, m[s12], m[s13]);                                                \
  G<V>(v3, v4, v9, v14, m[s14], m[s15]);

template <int V>
__device__ __forceinline__ void comp(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t ctr) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = ctr, v13 = 0, v14 = 64, v15 = 0;
  RND(V, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  RND(V, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
  RND(V, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1)
  RND(V, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6)
  RND(V, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4)
  RND(V, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7)
  RND(V, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13)
  cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}

template <int V, int STREAMS>
__global__ void __launch_bounds__(256) k_comp(uint32_t* out, int iters) {
  uint32_t cv[STREAMS][8];
  uint32_t m[16];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = t * 16 + i;
#pragma unroll
  for (int s = 0; s < STREAMS; ++s) {
    set_iv(cv[s]);
    cv[s][0] ^= t + s;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < STREAMS; ++s) comp<V>(cv[s], m, it);
    m[it & 15] ^= cv[0][1];
  }
  uint32_t x = 0;
#pragma unroll
  for (int s = 0; s < STREAMS; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= cv[s][i] * (i + 1);
  out[t] = x;
}

template <int V, int S>
void run(int cus, int wps, int iters, uint32_t* out, uint32_t* ref) {
  const int blocks = cus * wps;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_comp<V, S>), dim3(blocks), dim3(256), 0, 0, out, 4);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_comp<V, S>), dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  static uint32_t h[1 << 20], r[1 << 20];
  const int n = blocks * 256;
  hipMemcpy(h, out, 4 * n, hipMemcpyDeviceToHost);
  int bad = 0;
  if (ref) {
    hipMemcpy(r, ref, 4 * n, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i) bad += h[i] != r[i];
  }
  printf("variant %d streams %d waves/SIMD %d: %.1f G comp/s %s\n", V, S, wps,
         (double)blocks * 256 * iters * S / ms / 1e6, ref ? (bad ? "MISMATCH" : "ok") : "(ref)");
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t *out, *ref;
  hipMalloc(&out, 4 << 20);
  hipMalloc(&ref, 4 << 20);
  for (int w : {4, 8}) {
    run<0, 2>(cus, w, iters, ref, nullptr);
    run<0, 1>(cus, w, iters, out, nullptr);
    run<1, 2>(cus, w, iters, out, ref);
    run<2, 2>(cus, w, iters, out, ref);
    run<3, 2>(cus, w, iters, out, ref);
    run<4, 2>(cus, w, iters, out, ref);
  }
  return 0;
}
