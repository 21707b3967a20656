// ubench_compress.hip — BLAKE3 compression throughput on gfx950 with
// alternative instruction selections (measurement tool, not product code).
// Register-only: each lane runs dependent compressions (2 independent streams
// per lane), 8 waves per SIMD; prints G compressions/s per variant and checks
// every variant against the reference G (b3_device.h) bit-exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

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

// two-input xor issued as v_bitop3_b32 (truth table 0x3c = S0 ^ S1)
__device__ __forceinline__ uint32_t xr3(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %1 bitop3:0x3c" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t rot_align_asm(uint32_t x) {
  uint32_t r;
  asm volatile("v_alignbit_b32 %0, %1, %1, %2" : "=v"(r) : "v"(x), "i"(N));
  return r;
}

// one G as one asm block, dependent instructions back to back (no compiler
// scheduling, no hazard nops inside the block)
#define G_ASM_TEXT(R1, R2, R3, R4)                                                                   \
  "v_add3_u32 %0, %0, %1, %4\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, " #R1            \
  "\n v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, " #R2              \
  "\n v_add3_u32 %0, %0, %1, %5\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, " #R3         \
  "\n v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, " #R4 "\n"
__device__ __forceinline__ void g_asm(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
  asm volatile(G_ASM_TEXT(16, 12, 8, 7) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
}
// the same block with "s_nop 0" after chosen instruction kinds: NA after
// v_add3/v_add, NX after v_xor, NR after v_alignbit
#define G_NOP_TEXT(NA, NX, NR)                                                                                   \
  "v_add3_u32 %0, %0, %1, %4\n" NA "v_xor_b32 %3, %3, %0\n" NX "v_alignbit_b32 %3, %3, %3, 16\n" NR             \
  "v_add_u32 %2, %2, %3\n" NA "v_xor_b32 %1, %1, %2\n" NX "v_alignbit_b32 %1, %1, %1, 12\n" NR                  \
  "v_add3_u32 %0, %0, %1, %5\n" NA "v_xor_b32 %3, %3, %0\n" NX "v_alignbit_b32 %3, %3, %3, 8\n" NR              \
  "v_add_u32 %2, %2, %3\n" NA "v_xor_b32 %1, %1, %2\n" NX "v_alignbit_b32 %1, %1, %1, 7\n" NR
#define NOP "s_nop 0\n"
#define NOP1 "s_nop 1\n"
// alignbit nops chosen per rotation: R16, R12, R8, R7
#define G_ROT_TEXT(N16, N12, N8, N7)                                                                       \
  "v_add3_u32 %0, %0, %1, %4\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 16\n" N16              \
  "v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 12\n" N12                   \
  "v_add3_u32 %0, %0, %1, %5\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 8\n" N8                \
  "v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n" N7
template <int K>
__device__ __forceinline__ void g_nop(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
  if (K == 0) asm volatile(G_NOP_TEXT(NOP, NOP, NOP) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 1) asm volatile(G_NOP_TEXT("", NOP, NOP) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 2) asm volatile(G_NOP_TEXT("", "", NOP) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 3) asm volatile(G_NOP_TEXT("", NOP, "") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 4) asm volatile(G_NOP_TEXT(NOP, "", "") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 5) asm volatile(G_NOP_TEXT("", "", NOP1) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 6) asm volatile(G_ROT_TEXT("", NOP, "", NOP) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 7) asm volatile(G_ROT_TEXT(NOP, "", NOP, "") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
  if (K == 8) asm volatile(G_NOP_TEXT(NOP, NOP, "") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
}

// two G's interleaved instruction by instruction in one block
__device__ __forceinline__ void g2_asm(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y,
                                       uint32_t& e, uint32_t& f, uint32_t& g, uint32_t& h, uint32_t z, uint32_t w) {
  asm volatile(
      "v_add3_u32 %0, %0, %1, %8\n v_add3_u32 %4, %4, %5, %10\n"
      "v_xor_b32 %3, %3, %0\n v_xor_b32 %7, %7, %4\n"
      "v_alignbit_b32 %3, %3, %3, 16\n v_alignbit_b32 %7, %7, %7, 16\n"
      "v_add_u32 %2, %2, %3\n v_add_u32 %6, %6, %7\n"
      "v_xor_b32 %1, %1, %2\n v_xor_b32 %5, %5, %6\n"
      "v_alignbit_b32 %1, %1, %1, 12\n v_alignbit_b32 %5, %5, %5, 12\n"
      "v_add3_u32 %0, %0, %1, %9\n v_add3_u32 %4, %4, %5, %11\n"
      "v_xor_b32 %3, %3, %0\n v_xor_b32 %7, %7, %4\n"
      "v_alignbit_b32 %3, %3, %3, 8\n v_alignbit_b32 %7, %7, %7, 8\n"
      "v_add_u32 %2, %2, %3\n v_add_u32 %6, %6, %7\n"
      "v_xor_b32 %1, %1, %2\n v_xor_b32 %5, %5, %6\n"
      "v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %5, %5, %5, 7\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
      : "v"(x), "v"(y), "v"(z), "v"(w));
}

// 9..13 one asm block per G with s_nop 0 after: 9 every instruction, 10
// xor + alignbit, 11 alignbit, 12 xor, 13 add3/add
// VAR: 0 reference (add3 + alignbit); 1 add3 -> 2 adds; 2 rot12/rot7 by shifts;
// 3 all rotations by shifts; 4 = 1 + 2; 5 the four xors as v_bitop3_b32;
// 6 = 0 with every xor / alignbit as inline asm (same instructions as 5 but
// plain xor, to separate the asm-scheduling effect from the opcode)
template <int VAR>
__device__ __forceinline__ void G(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
  if (VAR == 7) {
    g_asm(a, b, c, d, x, y);
    return;
  }
  if (VAR >= 9 && VAR <= 17) {
    g_nop<VAR - 9>(a, b, c, d, x, y);
    return;
  }
  if (VAR == 5 || VAR == 6) {
    auto X = [](uint32_t p, uint32_t q) { return VAR == 5 ? xr3(p, q) : xr(p, q); };
    a = a + b + x;
    d = rot_align_asm<16>(X(d, a));
    c = c + d;
    b = rot_align_asm<12>(X(b, c));
    a = a + b + y;
    d = rot_align_asm<8>(X(d, a));
    c = c + d;
    b = rot_align_asm<7>(X(b, c));
    return;
  }
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

#define RND2(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15)            \
  g2_asm(v0, v4, v8, v12, m[s0], m[s1], v1, v5, v9, v13, m[s2], m[s3]);                         \
  g2_asm(v2, v6, v10, v14, m[s4], m[s5], v3, v7, v11, v15, m[s6], m[s7]);                       \
  g2_asm(v0, v5, v10, v15, m[s8], m[s9], v1, v6, v11, v12, m[s10], m[s11]);                     \
  g2_asm(v2, v7, v8, v13, m[s12], m[s13], v3, v4, v9, v14, m[s14], m[s15]);
#define RNDX(V, ...) \
  if (V == 8) {      \
    RND2(__VA_ARGS__) \
  } else {           \
    RND(V, __VA_ARGS__) \
  }

template <int V>
__device__ __forceinline__ void comp(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t ctr) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3, v12 = ctr, v13 = 0, v14 = 64, v15 = 0;
  RNDX(V, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  RNDX(V, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)
  RNDX(V, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1)
  RNDX(V, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6)
  RNDX(V, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4)
  RNDX(V, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7)
  RNDX(V, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13)
  cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}

template <int V, int STREAMS>
__global__ void __launch_bounds__(256) k_comp(uint32_t* out, int iters, uint64_t* stamps) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
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
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (stamps && (threadIdx.x & 63) == 0) {  // vector stores, one lane per wave
    const uint32_t w = t / 64;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

template <int V, int S>
void run(int cus, int wps, int iters, uint32_t* out, uint32_t* ref) {
  const int blocks = cus * wps;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  static uint64_t* stamps = nullptr;
  if (!stamps) hipMalloc(&stamps, 16 << 16);
  hipLaunchKernelGGL((k_comp<V, S>), dim3(blocks), dim3(256), 0, 0, out, 4, (uint64_t*)nullptr);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_comp<V, S>), dim3(blocks), dim3(256), 0, 0, out, iters, stamps);
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
  // in-kernel clock (MI355X_MICROARCH.md 'DVFS give-back' item 6): median over
  // waves of d(s_memtime) / d(s_memrealtime) x 100 MHz; cycles per compression
  // per SIMD from the same stamps
  static uint64_t hs[2 << 16];
  const int waves = n / 64;
  hipMemcpy(hs, stamps, 16 * waves, hipMemcpyDeviceToHost);
  static double clk[1 << 16], cyc[1 << 16];
  for (int w = 0; w < waves; ++w) {
    clk[w] = hs[2 * w + 1] ? (double)hs[2 * w] / (double)hs[2 * w + 1] * 0.1 : 0;
    cyc[w] = (double)hs[2 * w];
  }
  auto med = [&](double* v) {
    std::sort(v, v + waves);
    return v[waves / 2];
  };
  const double ghz = med(clk), wave_cycles = med(cyc);
  // a wave runs iters * S * 64 compressions; wps waves share a SIMD
  const double cyc_per_64 = wave_cycles / ((double)iters * S) / wps;
  printf("variant %d streams %d waves/SIMD %d: %.1f G comp/s, clock %.3f GHz, %.0f SIMD cycles per 64 compressions "
         "(%.2f per wave-instruction at 680) %s\n", V, S, wps,
         (double)blocks * 256 * iters * S / ms / 1e6, ghz, cyc_per_64, cyc_per_64 / 680.0,
         ref ? (bad ? "MISMATCH" : "ok") : "(ref)");
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t *out, *ref;
  hipMalloc(&out, 4 << 20);
  hipMalloc(&ref, 4 << 20);
  for (int w : {4, 6, 8}) {
    run<0, 2>(cus, w, iters, ref, nullptr);
    run<0, 1>(cus, w, iters, out, nullptr);
    run<6, 2>(cus, w, iters, out, ref);
    run<11, 2>(cus, w, iters, out, ref);
    run<12, 2>(cus, w, iters, out, ref);
    run<14, 2>(cus, w, iters, out, ref);
    run<15, 2>(cus, w, iters, out, ref);
    run<16, 2>(cus, w, iters, out, ref);
    run<17, 2>(cus, w, iters, out, ref);
    run<11, 1>(cus, w, iters, out, nullptr);
    run<0, 2>(cus, w, iters, out, ref);
  }
  return 0;
}
