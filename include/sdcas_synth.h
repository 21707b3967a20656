/*
 * sdcas_synth.h — definition of the synthetic corpora used by bench.py and the
 * parity tests (SURVEY.md §8d configs C2–C5). packages/test-files (config C1)
 * is empty in the reference snapshot, so every workload is generated from
 * (seed, file index, byte offset) with the functions below. They are written
 * once, as `static inline` C usable from host C/C++ and from HIP device code,
 * so the device generator and the CPU oracle read the exact same bytes.
 *
 * This is workload definition, not the hot path: nothing here touches BLAKE3.
 */
#ifndef SDCAS_SYNTH_H
#define SDCAS_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SDS_FN __host__ __device__ static inline
#else
#define SDS_FN static inline
#endif

/* constants fixed by the reference (core/src/object/cas.rs:10-15) */
#define SDS_SAMPLE_COUNT 4u
#define SDS_SAMPLE_SIZE 10240u
#define SDS_HEADER_OR_FOOTER_SIZE 8192u
#define SDS_MINIMUM_FILE_SIZE 102400u
/* le64(size) || header || 4 samples || footer */
#define SDS_SAMPLED_MSG_LEN (8u + 2u * SDS_HEADER_OR_FOOTER_SIZE + SDS_SAMPLE_COUNT * SDS_SAMPLE_SIZE)

/* per-config seeds */
#define SDS_SEED_C2 0x5D0002ull
#define SDS_SEED_C3 0x5D0003ull
#define SDS_SEED_C4 0x5D0004ull
#define SDS_SEED_C5 0x5D0005ull

SDS_FN uint64_t sds_mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* key of one content stream; `content_id` is what duplicate files share */
SDS_FN uint64_t sds_content_key(uint64_t seed, uint64_t content_id) {
  return sds_mix64(seed ^ (content_id * 0xD1B54A32D192ED03ull));
}

/* 8 content bytes at byte offset 8*w (little-endian packing) */
SDS_FN uint64_t sds_content_word(uint64_t key, uint64_t w) { return sds_mix64(key + w); }

SDS_FN uint8_t sds_content_byte(uint64_t key, uint64_t off) {
  return (uint8_t)(sds_content_word(key, off >> 3) >> ((off & 7u) * 8u));
}

/* C2: 1M files, size ~ Uniform{1024 .. 102400}, content_id = file index */
SDS_FN uint64_t sds_c2_size(uint64_t seed, uint64_t i) {
  return 1024u + sds_mix64(seed ^ 0xC2C2C2C2ull ^ (i << 20) ^ (i >> 44)) % (102400u - 1024u + 1u);
}

/* whole-file cas_id message length for a file of `size` bytes (cas.rs:25-29) */
SDS_FN uint64_t sds_cas_msg_len(uint64_t size) {
  return size <= SDS_MINIMUM_FILE_SIZE ? size + 8u : (uint64_t)SDS_SAMPLED_MSG_LEN;
}

/* Byte `x` of the cas_id message of a synthetic file (key, size): the
 * size prefix, then either the whole content or the six sampled windows
 * (cas.rs:25-58; seek_jump = (size - 16384) / 4, cas.rs:41). */
SDS_FN uint8_t sds_cas_msg_byte(uint64_t key, uint64_t size, uint64_t x) {
  if (x < 8u) return (uint8_t)(size >> (8u * x));
  uint64_t y = x - 8u;
  if (size <= SDS_MINIMUM_FILE_SIZE) return sds_content_byte(key, y);
  if (y < SDS_HEADER_OR_FOOTER_SIZE) return sds_content_byte(key, y);
  y -= SDS_HEADER_OR_FOOTER_SIZE;
  if (y < SDS_SAMPLE_COUNT * SDS_SAMPLE_SIZE) {
    uint64_t jump = (size - 2u * SDS_HEADER_OR_FOOTER_SIZE) / SDS_SAMPLE_COUNT;
    uint64_t k = y / SDS_SAMPLE_SIZE;
    return sds_content_byte(key, SDS_HEADER_OR_FOOTER_SIZE + k * jump + (y - k * SDS_SAMPLE_SIZE));
  }
  y -= SDS_SAMPLE_COUNT * SDS_SAMPLE_SIZE;
  return sds_content_byte(key, size - SDS_HEADER_OR_FOOTER_SIZE + y);
}

#endif /* SDCAS_SYNTH_H */
