// Dispatch latency of sdcas_io::WorkerPool (host only, no GPU): a context's
// path call hands the reads of a batch to the pool one or more times per
// call (once per upload part), so at the reference's 100-file steps the wake
// and join of the workers is part of every call.
//   ubench_pool THREADS ITEMS ITEM_US ROUNDS [GAP_US]
// runs ROUNDS dispatches of ITEMS items of ITEM_US busy work each, GAP_US of
// idle caller time between dispatches (the caller's GPU submit between two
// upload parts, or the time between calls), and prints the median / p90
// dispatch wall time and the ideal (ITEMS * ITEM_US / THREADS).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "../spacedrive_amd/host/cas_io.hpp"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void busy(double us) {
  const double t0 = now_us();
  while (now_us() - t0 < us) {
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s THREADS ITEMS ITEM_US ROUNDS [GAP_US]\n", argv[0]);
    return 2;
  }
  const uint32_t threads = (uint32_t)atoi(argv[1]);
  const size_t items = (size_t)atol(argv[2]);
  const double item_us = atof(argv[3]);
  const int rounds = atoi(argv[4]);
  const double gap_us = argc > 5 ? atof(argv[5]) : 0.0;
  sdcas_io::WorkerPool pool(threads);
  std::vector<double> t;
  std::vector<int> hit(items);
  for (int r = 0; r < rounds + 10; ++r) {
    if (gap_us > 0) busy(gap_us);
    const double t0 = now_us();
    pool.run(items, [&](size_t i) {
      busy(item_us);
      hit[i] = r;
    });
    const double dt = now_us() - t0;
    for (size_t i = 0; i < items; ++i)
      if (hit[i] != r) {
        fprintf(stderr, "item %zu not run in round %d\n", i, r);
        return 1;
      }
    if (r >= 10) t.push_back(dt);
  }
  std::sort(t.begin(), t.end());
  printf("{\"threads\": %u, \"items\": %zu, \"item_us\": %.1f, \"gap_us\": %.1f, "
         "\"median_us\": %.1f, \"p90_us\": %.1f, \"ideal_us\": %.1f}\n",
         threads, items, item_us, gap_us, t[t.size() / 2], t[t.size() * 9 / 10],
         items * item_us / std::min<size_t>(threads, items));
  return 0;
}
