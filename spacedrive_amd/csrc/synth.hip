// synth.hip — device generators for the synthetic corpora of SURVEY.md §8d
// (include/sdcas_synth.h). Benchmark/test input plumbing, not the hot path:
// they write the bytes a file of (content key, size) would hand to
// generate_cas_id / file_checksum, straight into HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sdcas_synth.h"
#include "synth.h"

namespace sdcas {

// one workgroup per file; 16 message bytes per lane-iteration
__global__ void __launch_bounds__(256) k_synth_cas_messages(const uint64_t* __restrict__ keys,
                                                            const uint64_t* __restrict__ sizes,
                                                            const uint64_t* __restrict__ offs, uint32_t n,
                                                            uint8_t* __restrict__ blob) {
  const uint32_t f = blockIdx.x;
  if (f >= n) return;
  const uint64_t key = keys[f], size = sizes[f];
  const uint64_t len = sds_cas_msg_len(size);
  uint8_t* dst = blob + offs[f];
  const uint64_t groups = (len + 15) / 16;
  if (size <= SDS_MINIMUM_FILE_SIZE) {
    // message byte x = content byte x - 8 (x >= 8): group q = content words 2q-1, 2q
    for (uint64_t q = threadIdx.x; q < groups; q += blockDim.x) {
      const uint64_t lo = q == 0 ? size : sds_content_word(key, 2 * q - 1);
      const uint64_t hi = sds_content_word(key, 2 * q);
      reinterpret_cast<uint4*>(dst)[q] =
          make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    }
  } else {
    for (uint64_t q = threadIdx.x; q < groups; q += blockDim.x) {
      uint32_t w[4];
      for (int t = 0; t < 4; ++t) {
        uint32_t x = 0;
        for (int b = 0; b < 4; ++b) {
          const uint64_t pos = 16 * q + 4 * t + b;
          x |= (pos < len ? (uint32_t)sds_cas_msg_byte(key, size, pos) : 0u) << (8 * b);
        }
        w[t] = x;
      }
      reinterpret_cast<uint4*>(dst)[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// raw content bytes [start, start + len) of each stream (file_checksum input);
// start must be a multiple of 16
__global__ void __launch_bounds__(256) k_synth_content(const uint64_t* __restrict__ keys,
                                                       const uint64_t* __restrict__ starts,
                                                       const uint64_t* __restrict__ lens,
                                                       const uint64_t* __restrict__ offs, uint32_t n,
                                                       uint8_t* __restrict__ blob) {
  const uint32_t f = blockIdx.y * gridDim.x + blockIdx.x;
  if (f >= n) return;
  const uint64_t key = keys[f], w0 = starts[f] / 8;
  const uint64_t groups = (lens[f] + 15) / 16;
  uint4* dst = reinterpret_cast<uint4*>(blob + offs[f]);
  for (uint64_t q = threadIdx.x; q < groups; q += blockDim.x) {
    const uint64_t lo = sds_content_word(key, w0 + 2 * q), hi = sds_content_word(key, w0 + 2 * q + 1);
    dst[q] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

hipError_t synth_cas_messages(const uint64_t* keys, const uint64_t* sizes, const uint64_t* offs, uint32_t n,
                              uint8_t* blob, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_synth_cas_messages, dim3(n), dim3(256), 0, st, keys, sizes, offs, n, blob);
  return hipGetLastError();
}

hipError_t synth_content(const uint64_t* keys, const uint64_t* starts, const uint64_t* lens, const uint64_t* offs,
                         uint32_t n, uint8_t* blob, hipStream_t st) {
  if (!n) return hipSuccess;
  const uint32_t gx = n < 65535 ? n : 65535, gy = (n + gx - 1) / gx;
  hipLaunchKernelGGL(k_synth_content, dim3(gx, gy), dim3(256), 0, st, keys, starts, lens, offs, n, blob);
  return hipGetLastError();
}

}  // namespace sdcas
