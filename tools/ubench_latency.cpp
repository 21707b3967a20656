// ubench_latency.cpp — per-call wall time of sdcas_cas_ids at the C ABI (no
// Python in the timed region), for one library or several side by side
// (measurement tool; tools/latency_probe.py writes the files and runs it).
//
//   ubench_latency MANIFEST BATCHES CALLS LIB[@IO_THREADS]...
//
// MANIFEST: one "size path" line per file (files in the page cache). For each
// batch size B, CALLS calls over consecutive slices of the manifest (a call
// reads files its library has not just read, as the identifier's steps do);
// with several libraries each slice is hashed by all, the order rotating per
// call, and the keys must agree. Prints one JSON line per (library, B).
// "@N" sets the context's reader threads (sdcas_options.io_threads; default
// 0 = the library's 8); the same library may be named twice with different N.
// ",NAME=VALUE[,NAME=VALUE]" sets environment variables while the context is created
// (e.g. ",SDCAS_SMALL_SLOTS=0": that context never uses the small-batch
// kernel), so one library can be compared with itself under two settings.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../include/sdcas.h"

namespace {

struct Lib {
  std::string path;
  uint32_t io_threads = 0;
  void* h = nullptr;
  int (*init)(const sdcas_options*, sdcas_ctx**) = nullptr;
  void (*destroy)(sdcas_ctx*) = nullptr;
  int (*cas_ids)(sdcas_ctx*, const char* const*, const uint64_t*, size_t, uint64_t*, int32_t*) = nullptr;
  sdcas_ctx* ctx = nullptr;
  bool open(const std::string& spec_in) {
    path = spec_in;
    std::string spec = spec_in, env;
    const size_t comma = spec.find(',');
    if (comma != std::string::npos) {
      env = spec.substr(comma + 1);
      spec = spec.substr(0, comma);
    }
    const size_t at = spec.rfind('@');
    const std::string p = at == std::string::npos ? spec : spec.substr(0, at);
    if (at != std::string::npos) io_threads = (uint32_t)std::stoul(spec.substr(at + 1));
    h = dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) return fprintf(stderr, "dlopen %s: %s\n", p.c_str(), dlerror()), false;
    init = (decltype(init))dlsym(h, "sdcas_init");
    destroy = (decltype(destroy))dlsym(h, "sdcas_destroy");
    cas_ids = (decltype(cas_ids))dlsym(h, "sdcas_cas_ids");
    if (!init || !destroy || !cas_ids) return fprintf(stderr, "%s: missing symbols\n", p.c_str()), false;
    sdcas_options o = SDCAS_OPTIONS_INIT;
    o.device = 0;
    o.io_threads = io_threads;
    std::vector<std::string> names;  // ",A=1,B=2": several variables
    for (size_t pos = 0; !env.empty() && pos != std::string::npos;) {
      const size_t next = env.find(',', pos);
      const std::string kv = env.substr(pos, next == std::string::npos ? std::string::npos : next - pos);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos) {
        names.push_back(kv.substr(0, eq));
        setenv(names.back().c_str(), kv.substr(eq + 1).c_str(), 1);
      }
      pos = next == std::string::npos ? next : next + 1;
    }
    const bool ok = init(&o, &ctx) == SDCAS_OK;
    for (const auto& nm : names) unsetenv(nm.c_str());
    return ok;
  }
};

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}
double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[std::min(v.size() - 1, (size_t)(q * v.size()))];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s MANIFEST BATCHES CALLS LIB[@IO_THREADS]...\n", argv[0]);
    return 2;
  }
  std::vector<std::string> paths;
  std::vector<uint64_t> sizes;
  {
    std::ifstream f(argv[1]);
    uint64_t s;
    std::string p;
    while (f >> s >> p) sizes.push_back(s), paths.push_back(p);
  }
  std::vector<const char*> cp(paths.size());
  for (size_t i = 0; i < paths.size(); ++i) cp[i] = paths[i].c_str();
  std::vector<size_t> batches;
  {
    std::stringstream ss(argv[2]);
    std::string t;
    while (std::getline(ss, t, ',')) batches.push_back(std::stoul(t));
  }
  const size_t calls_max = std::stoul(argv[3]);
  std::vector<Lib> libs(argc - 4);
  for (size_t l = 0; l < libs.size(); ++l)
    if (!libs[l].open(argv[4 + l])) return 1;
  const size_t N = paths.size();
  std::vector<std::vector<uint64_t>> keys(libs.size(), std::vector<uint64_t>(N));
  std::vector<int32_t> st(N);
  // warm-up: contexts, reader pools, staging, page cache
  for (size_t l = 0; l < libs.size(); ++l)
    if (libs[l].cas_ids(libs[l].ctx, cp.data(), sizes.data(), N, keys[l].data(), st.data())) return 1;
  int bad = 0;
  for (size_t B : batches) {
    if (B > N) continue;
    const size_t calls = std::min(calls_max, N / B);
    std::vector<std::vector<double>> lat(libs.size());
    for (size_t c = 0; c < calls; ++c) {
      const size_t lo = c * B;
      for (size_t r = 0; r < libs.size(); ++r) {
        const size_t l = (r + c) % libs.size();
        const auto t0 = std::chrono::steady_clock::now();
        const int rc =
            libs[l].cas_ids(libs[l].ctx, cp.data() + lo, sizes.data() + lo, B, keys[l].data() + lo, st.data() + lo);
        lat[l].push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (rc) return fprintf(stderr, "call failed: %d\n", rc), 1;
        for (size_t i = lo; i < lo + B; ++i) bad += st[i] != 0;
      }
      for (size_t l = 1; l < libs.size(); ++l)
        for (size_t i = lo; i < lo + B; ++i) bad += keys[l][i] != keys[0][i];
    }
    for (size_t l = 0; l < libs.size(); ++l) {
      const double med = median(lat[l]);
      printf("{\"lib\": \"%s\", \"batch\": %zu, \"calls\": %zu, \"median_ms\": %.4f, \"p10_ms\": %.4f, "
             "\"p90_ms\": %.4f, \"files_per_s\": %.0f}\n",
             libs[l].path.c_str(), B, calls, med, pct(lat[l], 0.1), pct(lat[l], 0.9), B / (med * 1e-3));
    }
    fflush(stdout);
  }
  for (auto& L : libs) L.destroy(L.ctx);
  printf("{\"mismatches_or_errors\": %d}\n", bad);
  return bad != 0;
}
