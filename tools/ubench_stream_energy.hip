// ubench_stream_energy.hip — does the SHAPE or CACHE POLICY of the message
// stream change the clock the card holds while it hashes? (measurement tool,
// not product code)
//
// The leaf kernel is held by the clock under the power limit, and the HBM
// stream costs ~16-19 % of that clock (profiles/r02_diag_hbm_energy.txt). Every
// variant here runs the SAME compressions (B3_G_ASM, 16 blocks per chunk, two
// chunks per lane, 512-thread workgroups at 6 waves/SIMD, one 1 MiB tile per
// workgroup, as k_leaf_tree) over the same 32 GiB and differs only in how the
// bytes reach the registers:
//   0  per-lane chunk lines (the leaf kernel's shape: each lane reads its own
//      chunk, a 128-byte line per step, 64 lines per wave-instruction group)
//   1  0 with non-temporal loads
//   2  coalesced: each wave-instruction reads 1 KiB of contiguous bytes (the
//      same bytes per wave, another order; the digests are meaningless)
//   3  2 with non-temporal loads
//   4  no loads (register values) — the compute-only clock
//   5  0 with every address folded into the first 2 MiB (served by L2)
//   6  global_load_lds_dwordx4 (LDS-DMA, coalesced 128-byte lines), then each
//      lane reads its own chunk's line from LDS (the correct layout)
// Prints ms, in-kernel clock (s_memtime / s_memrealtime), G compressions/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../spacedrive_amd/csrc/b3_device.h"

using namespace b3d;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}

__device__ __forceinline__ void put(uint32_t (&m)[16], int k, u32x4 v) {
  m[4 * k] = v.x; m[4 * k + 1] = v.y; m[4 * k + 2] = v.z; m[4 * k + 3] = v.w;
}

constexpr int WG = 512;
constexpr uint32_t TILE_BYTES = 1u << 20;  // 1024 chunks of 1 KiB, 2 per lane

template <int V>
__global__ void __launch_bounds__(WG, 6) k_stream(const uint8_t* __restrict__ buf, uint32_t* __restrict__ out,
                                                  uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[(V == 6) ? (WG / 64) * 4096 : 16];
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint8_t* tile = buf + (size_t)blockIdx.x * TILE_BYTES;
  uint32_t acc = 0;
  for (int s = 0; s < 2; ++s) {
    // chunk of this lane in this pass: wave w owns chunks [128 w, 128 w + 128)
    const uint32_t chunk = wave * 128 + s * 64 + lane;
    const uint8_t* cbase = tile + (size_t)chunk * 1024;
    // coalesced shape: the wave's 64 chunks are 64 KiB contiguous; step i reads
    // 8 KiB of it, 1 KiB per wave-instruction
    const uint8_t* wbase = tile + (size_t)(wave * 128 + s * 64) * 1024;
    uint32_t cv[8];
    set_iv(cv);
#pragma unroll 1
    for (uint32_t b = 0; b < 16; b += 2) {
      uint32_t m0[16], m1[16];
      if constexpr (V == 0 || V == 1 || V == 5) {
        const uint8_t* q = cbase + b * 64;
        if constexpr (V == 5) q = buf + (((size_t)(q - buf)) & ((2u << 20) - 1));
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m0, k, ld16<V == 1>(q + 16 * k));
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m1, k, ld16<V == 1>(q + 64 + 16 * k));
      } else if constexpr (V == 2 || V == 3) {
        const uint8_t* q = wbase + (size_t)(b / 2) * 8192 + lane * 16;
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m0, k, ld16<V == 3>(q + 1024 * k));
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m1, k, ld16<V == 3>(q + 4096 + 1024 * k));
      } else if constexpr (V == 4) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          m0[k] = chunk * 16 + k + b;
          m1[k] = chunk * 16 + k + b + 1;
        }
      } else if constexpr (V == 6) {
        // 4 LDS-DMA instructions per 64-byte half: instruction k fetches the
        // step's half-line of chunks 16k..16k+15 (4 lanes each); LDS holds them
        // in chunk order at wave base + chunk * 64 (4 KiB per wave, so three
        // workgroups fit a CU). The second half's DMA runs under the first
        // block's compression.
        uint8_t* wl = lds + wave * 4096;
        const uint32_t c16 = lane >> 2, piece = lane & 3;
        const u32x4* myl = reinterpret_cast<const u32x4*>(wl + lane * 64);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          __builtin_amdgcn_global_load_lds((const void*)(wbase + (size_t)(16 * k + c16) * 1024 + b * 64 + piece * 16),
                                           (__attribute__((address_space(3))) void*)(wl + k * 1024), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m0, k, myl[k]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k)
          __builtin_amdgcn_global_load_lds((const void*)(wbase + (size_t)(16 * k + c16) * 1024 + b * 64 + 64 + piece * 16),
                                           (__attribute__((address_space(3))) void*)(wl + k * 1024), 16, 0, 0);
        compress<2>(cv, m0, chunk, 64, b == 0 ? CHUNK_START : 0u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) put(m1, k, myl[k]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        compress<2>(cv, m1, chunk, 64, b + 2 == 16 ? CHUNK_END : 0u);
        continue;
      }
      compress<2>(cv, m0, chunk, 64, b == 0 ? CHUNK_START : 0u);
      compress<2>(cv, m1, chunk, 64, b + 2 == 16 ? CHUNK_END : 0u);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= cv[i] * (i + 1);
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    const uint32_t w = blockIdx.x * (WG / 64) + wave;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

__global__ void k_fill(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u;
    x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
    p[i] = x;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

struct Res {
  double ms, ghz;
};

template <int V>
Res run(const uint8_t* buf, uint32_t tiles, uint32_t* out, uint64_t* stamps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((k_stream<V>), dim3(tiles), dim3(WG), 0, 0, buf, out, stamps);
  CK(hipGetLastError());
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const size_t waves = (size_t)tiles * (WG / 64);
  std::vector<uint64_t> hs(2 * waves);
  CK(hipMemcpy(hs.data(), stamps, 16 * waves, hipMemcpyDeviceToHost));
  std::vector<double> clk;
  clk.reserve(waves);
  for (size_t w = 0; w < waves; ++w)
    if (hs[2 * w + 1]) clk.push_back((double)hs[2 * w] / (double)hs[2 * w + 1] * 0.1);
  std::sort(clk.begin(), clk.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return {ms, clk.empty() ? 0 : clk[clk.size() / 2]};
}

int main(int argc, char** argv) {
  const uint32_t gib = argc > 1 ? atoi(argv[1]) : 32;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t tiles = gib * 1024;
  uint8_t* buf;
  uint32_t* out;
  uint64_t* stamps;
  const size_t bytes = (size_t)tiles * TILE_BYTES;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMalloc(&out, (size_t)tiles * WG * 4));
  CK(hipMalloc(&stamps, (size_t)tiles * (WG / 64) * 16));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, bytes / 4);
  CK(hipDeviceSynchronize());
  const double comps = (double)tiles * 1024 * 16;  // 16 blocks per 1 KiB chunk
  const char* names[7] = {"lane-lines", "lane-lines nt", "coalesced", "coalesced nt", "no loads", "L2-folded",
                          "glds lines"};
  std::vector<std::vector<Res>> r(7);
  for (int it = 0; it < rounds + 1; ++it) {  // round 0 is warmup
    Res x[7] = {run<0>(buf, tiles, out, stamps), run<1>(buf, tiles, out, stamps), run<2>(buf, tiles, out, stamps),
                run<3>(buf, tiles, out, stamps), run<4>(buf, tiles, out, stamps), run<5>(buf, tiles, out, stamps),
                run<6>(buf, tiles, out, stamps)};
    if (it)
      for (int v = 0; v < 7; ++v) r[v].push_back(x[v]);
  }
  printf("{\"gib\": %u, \"rounds\": %d, \"compressions\": %.0f, \"variants\": [\n", gib, rounds, comps);
  for (int v = 0; v < 7; ++v) {
    auto ms = r[v];
    std::sort(ms.begin(), ms.end(), [](const Res& p, const Res& q) { return p.ms < q.ms; });
    const Res med = ms[ms.size() / 2];
    printf(" {\"v\": %d, \"name\": \"%s\", \"ms_median\": %.3f, \"ms_min\": %.3f, \"clock_ghz\": %.3f, "
           "\"gcomp_s\": %.2f, \"tb_s\": %.3f}%s\n",
           v, names[v], med.ms, ms[0].ms, med.ghz, comps / med.ms / 1e6, (double)bytes / med.ms / 1e9,
           v < 6 ? "," : "");
  }
  printf("]}\n");
  return 0;
}
