// The host side of a small batch's slot plan (sdcas::batch_plan_host,
// spacedrive_amd/csrc/b3_batch.hip; no GPU call): against a slot-by-slot
// restatement of what the device scan and k_tile_first write — message m
// owns slots [S[m], S[m] + C[m]) with C = max(1, ceil(len / 1024)), tile t's
// first slot t * TILE belongs to tile_first[t], total = the slot count — and
// the "some message crosses a tile boundary" flag, over random and edge
// batches of 1-127 messages. TEST INFRASTRUCTURE.
#include <stdint.h>
#include <stdio.h>

#include <random>
#include <vector>

namespace sdcas {
uint64_t batch_plan_host(const uint64_t* lens, uint32_t n, uint32_t tile, uint64_t cap_slots, uint64_t* S,
                         uint32_t* tile_first, uint64_t* total, bool* crossing);
}

static int failures = 0;
#define CHECK(c, ...)                  \
  do {                                 \
    if (!(c)) {                        \
      fprintf(stderr, __VA_ARGS__);    \
      fprintf(stderr, "\n");           \
      ++failures;                      \
    }                                  \
  } while (0)

static void check_batch(const std::vector<uint64_t>& lens, uint32_t tile) {
  const uint32_t n = (uint32_t)lens.size();
  // the restatement: one owner per slot
  std::vector<uint32_t> owner;
  std::vector<uint64_t> want_S(n);
  bool want_cross = false;
  for (uint32_t m = 0; m < n; ++m) {
    const uint64_t C = lens[m] == 0 ? 1 : (lens[m] + 1023) / 1024;
    want_S[m] = owner.size();
    const uint64_t first_tile = owner.size() / tile;
    for (uint64_t k = 0; k < C; ++k) owner.push_back(m);
    want_cross = want_cross || (owner.size() - 1) / tile != first_tile;
  }
  const uint64_t slots = owner.size(), tiles = (slots + tile - 1) / tile;
  std::vector<uint64_t> S(n, ~0ull), total(4, ~0ull);
  std::vector<uint32_t> tf(tiles + 2, 0xFFFFFFFFu);
  bool cross = !want_cross;
  const uint64_t got_tiles = sdcas::batch_plan_host(lens.data(), n, tile, 1ull << 40, S.data(), tf.data(),
                                                    total.data(), &cross);
  CHECK(got_tiles == tiles, "n %u: tiles %llu, want %llu", n, (unsigned long long)got_tiles,
        (unsigned long long)tiles);
  CHECK(total[0] == slots && total[1] == 0 && total[2] == 0 && total[3] == 0, "n %u: total words", n);
  CHECK(cross == want_cross, "n %u: crossing %d, want %d", n, (int)cross, (int)want_cross);
  for (uint32_t m = 0; m < n; ++m) CHECK(S[m] == want_S[m], "n %u: S[%u]", n, m);
  for (uint64_t t = 0; t < tiles; ++t)
    CHECK(tf[t] == owner[t * tile], "n %u: tile_first[%llu] = %u, want %u", n, (unsigned long long)t, tf[t],
          owner[t * tile]);
  CHECK(tf[tiles] == 0xFFFFFFFFu, "n %u: wrote past the last tile", n);
}

int main() {
  std::mt19937_64 rng(128);
  const uint64_t edges[] = {0, 1, 63, 64, 1023, 1024, 1025, 2048, 127 * 1024, 128 * 1024 - 1, 128 * 1024,
                            128 * 1024 + 1, 300 * 1024 + 5};
  int batches = 0;
  for (uint64_t L : edges) {
    check_batch({L}, 128);
    ++batches;
  }
  for (int rep = 0; rep < 2000; ++rep) {
    const uint32_t n = 1 + (uint32_t)(rng() % 127);
    std::vector<uint64_t> lens(n);
    for (auto& L : lens) L = rng() % 3 ? rng() % (140 * 1024) : edges[rng() % (sizeof edges / sizeof edges[0])];
    check_batch(lens, 128);
    check_batch(lens, 1024);
    batches += 2;
  }
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("ALL OK (%d batches)\n", batches);
  return 0;
}
