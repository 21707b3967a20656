// synth.h — device generators for the synthetic corpora (bench/test plumbing).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdcas {
// cas_id messages (le64(size) || whole file, or the sampled 57,352-byte
// message) of synthetic files (keys[i], sizes[i]) at blob + offs[i]
// (16-byte aligned); bytes up to the next 16-byte boundary are filler.
hipError_t synth_cas_messages(const uint64_t* keys, const uint64_t* sizes, const uint64_t* offs, uint32_t n,
                              uint8_t* blob, hipStream_t st);
// content bytes [starts[i], starts[i] + lens[i]) of stream keys[i] at
// blob + offs[i]; starts[i] multiple of 16
hipError_t synth_content(const uint64_t* keys, const uint64_t* starts, const uint64_t* lens, const uint64_t* offs,
                         uint32_t n, uint8_t* blob, hipStream_t st);
}  // namespace sdcas
