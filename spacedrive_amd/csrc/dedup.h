// dedup.h — host interface of the device cas_id -> Object group-by.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdcas {

struct DedupWorkspace {
  uint64_t* key_a = nullptr;  // [cap]
  uint64_t* key_b = nullptr;  // [cap]
  uint32_t* idx_a = nullptr;  // [cap]
  uint32_t* idx_b = nullptr;  // [cap]
  uint32_t* head = nullptr;   // [cap]
  uint8_t* valid = nullptr;   // [cap]
  uint32_t* nvalid = nullptr; // [1]
  void* temp = nullptr;
  size_t temp_bytes = 0;
  uint32_t cap = 0;
  static size_t temp_bytes_for(uint32_t n);
};

// Sort existing Objects' keys (stable, so each key's first entry is the first
// Object in DB order). ekeys_sorted/eidx_sorted: [ne] device arrays.
hipError_t dedup_sort_existing(DedupWorkspace& w, const uint64_t* ekeys, uint32_t ne, uint64_t* ekeys_sorted,
                               uint32_t* eidx_sorted, hipStream_t st);

// All pointers device pointers. d_counts (optional): [created, linked].
hipError_t dedup_run(DedupWorkspace& w, const uint64_t* keys, const uint8_t* has_key, const int32_t* status,
                     uint32_t n, uint32_t chunk_size, const uint64_t* ekeys_sorted, const uint32_t* eidx_sorted,
                     uint32_t ne, int64_t* out_link, unsigned long long* d_counts, hipStream_t st);

}  // namespace sdcas
