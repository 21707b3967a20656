// ubench_valu.hip — VALU throughput of the BLAKE3 compression on gfx950 and of
// the instructions it is made of (measurement tool, not product code).
// Each lane runs ITERS dependent compressions on register data (4 independent
// streams per lane to give the scheduler ILP); grid = CUs x blocks; prints
// G compressions/s, effective int-ops/s and the in-kernel shader clock
// (s_memtime / s_memrealtime, MI355X_MICROARCH.md DVFS item 6).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../spacedrive_amd/csrc/b3_device.h"

using namespace b3d;

template <int STREAMS>
__global__ void __launch_bounds__(256) k_compress(uint32_t* out, int iters, uint64_t* clk) {
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
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < STREAMS; ++s) compress(cv[s], m, it, 64, 0);
    m[it & 15] ^= cv[0][1];
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
#pragma unroll
  for (int s = 0; s < STREAMS; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= cv[s][i];
  out[t] = x;
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// instruction-rate probes: 8 independent chains per lane, forced by inline asm
#define OP1(INS)                                                  \
  _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(INS : "+v"(a[i]) : "v"(b), "v"(c));
template <int OP>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, int iters) {
  uint32_t a[8];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = t * 7 + i;
  uint32_t b = t ^ 0x55, c = t * 3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (OP == 0) { OP1("v_add_u32 %0, %0, %1") }
      if (OP == 1) { OP1("v_xor_b32 %0, %0, %1") }
      if (OP == 2) { OP1("v_alignbit_b32 %0, %0, %0, 7") }
      if (OP == 3) { OP1("v_add3_u32 %0, %0, %1, %2") }
      if (OP == 4) { OP1("v_xad_u32 %0, %0, %1, %2") }
      if (OP == 5) { OP1("v_perm_b32 %0, %0, %0, %1") }
      if (OP == 6) { OP1("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") }
      if (OP == 7) { OP1("v_pk_add_u16 %0, %0, %1") }
      if (OP == 8) { OP1("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0") }
      if (OP == 9) { OP1("v_lshrrev_b32 %0, 7, %0") }
      if (OP == 10) { OP1("v_lshl_or_b32 %0, %0, 7, %1") }
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= a[i];
  out[t] = x;
}

__global__ void k_rot16_check(const uint32_t* in, uint32_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t d = in[2 * i], a = in[2 * i + 1];
    out[2 * i] = xor_rot16(d, a);
    out[2 * i + 1] = rotr(d ^ a, 16);
  }
}

int main(int argc, char** argv) {
  {
    const int n = 1 << 16;
    uint32_t *din, *dout;
    hipMalloc(&din, 8 * n);
    hipMalloc(&dout, 8 * n);
    uint32_t* h = (uint32_t*)malloc(8 * n);
    uint64_t x = 12345;
    for (int i = 0; i < 2 * n; ++i) { x = x * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(x >> 32); }
    hipMemcpy(din, h, 8 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rot16_check, dim3(n / 256), dim3(256), 0, 0, din, dout, n);
    hipMemcpy(h, dout, 8 * n, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += h[2 * i] != h[2 * i + 1];
    printf("xor_rot16 check: %d / %d mismatches (e.g. %08x vs %08x)\n", bad, n, h[0], h[1]);
  }
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t* out;
  uint64_t* clk;
  hipMalloc(&out, 64 << 20);
  hipMalloc(&clk, 2048 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wps = 1; wps <= 8; wps *= 2) {  // waves per SIMD
    const int blocks = cus * wps;           // 256-thread block = 4 waves = 1 per SIMD
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_compress<2>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      uint64_t h[2048];
      hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
      double ghz = 0;
      int nb = blocks < 1024 ? blocks : 1024;
      for (int b = 0; b < nb; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
      ghz /= nb;
      double comps = (double)blocks * 256 * iters * 2;
      if (rep)
        printf("compress streams=2 waves/SIMD=%d: %.3f ms  %.1f G comp/s  (%.1f T ops/s at 680/comp)  clock %.2f GHz\n",
               wps, ms, comps / ms / 1e6, comps * 680 / ms / 1e9, ghz);
    }
  }
  const char* names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_add3_u32", "v_xad_u32", "v_perm_b32",
                         "v_bitop3_b32", "v_pk_add_u16", "v_xor_b32_sdwa", "v_lshrrev_b32", "v_lshl_or_b32"};
  for (int op = 0; op < 11; ++op) {
    const int blocks = cus * 8;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (op == 0) hipLaunchKernelGGL(k_op<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 1) hipLaunchKernelGGL(k_op<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 2) hipLaunchKernelGGL(k_op<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 3) hipLaunchKernelGGL(k_op<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 4) hipLaunchKernelGGL(k_op<4>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 5) hipLaunchKernelGGL(k_op<5>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 6) hipLaunchKernelGGL(k_op<6>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 7) hipLaunchKernelGGL(k_op<7>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 8) hipLaunchKernelGGL(k_op<8>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 9) hipLaunchKernelGGL(k_op<9>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (op == 10) hipLaunchKernelGGL(k_op<10>, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double ops = (double)blocks * 256 * iters * 16 * 8;
      if (rep) printf("%-16s %.3f ms  %.1f T lane-ops/s\n", names[op], ms, ops / ms / 1e9);
    }
  }
  return 0;
}
