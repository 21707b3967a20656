// CPU test of libsdcas's host file I/O (spacedrive_amd/host/cas_io.cpp) —
// built plain, with ASan + UBSan and with TSan (tests/cpp/Makefile
// `sanitize`). TEST INFRASTRUCTURE: the oracle (oracle/cas_ref.c,
// oracle/blake3_ref.c) is compiled in as the checker.
//
// Every file is read the way sdcas_cas_ids reads it (read_cas_message into a
// slot sized from the indexer's `size`, a retry in a bigger slot when the
// file grew) on 8 threads at once, and the message's cas key is compared
// with oracle_generate_cas_id's restatement of cas.rs:23-62 — whole files,
// sampled sparse files, files grown / shrunk since they were indexed,
// missing paths, directories, empty files. plan_batch (the staging-slot
// packing) is checked against its invariants on random sizes.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <atomic>
#include <vector>

#include "../../oracle/oracle.h"
#include "../../spacedrive_amd/host/cas_io.hpp"

static int failures = 0;
#define CHECK(cond, ...)                                        \
  do {                                                          \
    if (!(cond)) {                                              \
      ++failures;                                               \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
    }                                                           \
  } while (0)

struct Case {
  std::string path;
  uint64_t size;  // what the indexer saw (cas.rs's `size` argument)
};

static void write_file(const std::string& p, uint64_t n, std::mt19937_64& rng) {
  FILE* f = std::fopen(p.c_str(), "wb");
  std::vector<uint8_t> b(n);
  for (auto& x : b) x = (uint8_t)rng();
  if (n) std::fwrite(b.data(), 1, n, f);
  std::fclose(f);
}

// a sparse file of n bytes whose cas.rs windows hold data (the rest is a hole)
static void write_sparse(const std::string& p, uint64_t n, std::mt19937_64& rng) {
  int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
  if (ftruncate(fd, (off_t)n) != 0) std::perror("ftruncate");
  const uint64_t jump = (n - 16384) / 4;
  std::vector<std::pair<uint64_t, uint64_t>> w = {{0, 8192}, {n - 8192, 8192}};
  for (uint64_t k = 0; k < 4; ++k) w.push_back({8192 + k * jump, 10240});
  std::vector<uint8_t> b(10240);
  for (auto [off, len] : w) {
    for (auto& x : b) x = (uint8_t)rng();
    if (pwrite(fd, b.data(), len, (off_t)off) != (ssize_t)len) std::perror("pwrite");
  }
  close(fd);
}

// sdcas_cas_ids' use of read_cas_message: the slot the indexer's size
// predicts (+1 byte to tell a grown file), a retry in a bigger one
// mode 0: page-cache reads; 1: SDCAS_OPT_DIRECT_IO (O_DIRECT where the
// filesystem takes it); 2: the aligned (O_DIRECT) read logic on a plain
// descriptor, so that it is exercised whatever the filesystem
static int library_read(const Case& c, std::vector<uint8_t>& buf, uint64_t* len, int mode = 0) {
  const uint64_t want = (c.size <= 102400 ? c.size + 8 + 1 : 57352);
  uint64_t cap = sdcas_io::align_line(want);
  for (int round = 0; round < 4; ++round) {
    buf.assign(cap + 64, 0);
    uint64_t retry = 0;
    int st;
    if (mode == 2) {
      const int fd = open(c.path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) return errno;
      st = sdcas_io::read_cas_message_fd(fd, true, c.size, buf.data(), cap, len, &retry);
      close(fd);
    } else {
      st = sdcas_io::read_cas_message(c.path.c_str(), c.size, buf.data(), cap, len, &retry, mode == 1);
    }
    if (st || !retry) return st;
    cap = sdcas_io::align_line(retry);
  }
  return EAGAIN;
}

int main() {
  char tmpl[] = "/tmp/test_cas_io_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  if (!dir) return 2;
  std::mt19937_64 rng(12345);
  std::vector<Case> cases;
  auto path = [&](const std::string& n) { return std::string(dir) + "/" + n; };
  for (int i = 0; i < 240; ++i) {  // whole files (cas.rs:27-29), incl. the boundaries
    uint64_t n = i < 8 ? std::vector<uint64_t>{0, 1, 1016, 1017, 1023, 1024, 102399, 102400}[i] : rng() % 102401;
    write_file(path("w" + std::to_string(i)), n, rng);
    cases.push_back({path("w" + std::to_string(i)), n});
  }
  for (uint64_t n : {102401ull, 102402ull, 114688ull, (5ull << 20) + 3, (1ull << 30) + 3}) {  // cas.rs:30-59
    write_sparse(path("s" + std::to_string(n)), n, rng);
    cases.push_back({path("s" + std::to_string(n)), n});
  }
  write_file(path("grown"), 70000, rng);  // indexed at 5000 bytes, grew: fs::read takes it all
  cases.push_back({path("grown"), 5000});
  write_file(path("grown_big"), 300000, rng);  // indexed under 100 KiB, now past it
  cases.push_back({path("grown_big"), 100000});
  write_file(path("shrunk_whole"), 100, rng);  // indexed at 5000 bytes, now 100
  cases.push_back({path("shrunk_whole"), 5000});
  write_file(path("shrunk_sampled"), 50000, rng);  // sampled windows past EOF: UnexpectedEof
  cases.push_back({path("shrunk_sampled"), 300000});
  write_file(path("shrunk_tiny"), 5000, rng);  // not even a header
  cases.push_back({path("shrunk_tiny"), 300000});
  cases.push_back({path("missing"), 10});
  mkdir(path("adir").c_str(), 0755);
  cases.push_back({path("adir"), 4096});
  cases.push_back({path("adir"), 200000});

  // the oracle's answers
  std::vector<int> want_st(cases.size());
  std::vector<std::string> want_hex(cases.size());
  for (size_t i = 0; i < cases.size(); ++i) {
    char hex[17] = {0};
    want_st[i] = oracle_generate_cas_id(cases[i].path.c_str(), cases[i].size, hex);
    want_hex[i] = hex;
  }
  // the library's reads, 8 threads at once, ten times over (page cache,
  // O_DIRECT, aligned logic in turn): through parallel_for, then through one
  // WorkerPool reused for every run (as a context reuses its pool for every
  // staging slot)
  sdcas_io::WorkerPool pool(8);
  CHECK(pool.threads() == 8, "pool threads %u", pool.threads());
  for (int rep = 0; rep < 10; ++rep) {
    std::vector<int> st(cases.size());
    std::vector<std::string> hex(cases.size());
    auto one = [&](size_t i) {
      std::vector<uint8_t> buf;
      uint64_t len = 0;
      st[i] = library_read(cases[i], buf, &len, rep % 3);
      if (!st[i]) {
        char h[17];
        std::snprintf(h, sizeof h, "%016llx", (unsigned long long)oracle_cas_key_of_message(buf.data(), len));
        hex[i] = h;
      }
    };
    if (rep < 5) sdcas_io::parallel_for(8, cases.size(), one);
    else pool.run(cases.size(), one);
    for (size_t i = 0; i < cases.size(); ++i) {
      CHECK(st[i] == want_st[i], "%s: status %d, oracle %d", cases[i].path.c_str(), st[i], want_st[i]);
      if (!st[i] && !want_st[i])
        CHECK(hex[i] == want_hex[i], "%s: %s, oracle %s", cases[i].path.c_str(), hex[i].c_str(),
              want_hex[i].c_str());
    }
  }
  {  // many small jobs back to back on one pool: every item exactly once per
     // job, none after run() returned
    for (sdcas_io::WorkerPool* p : {&pool}) {
      std::vector<std::atomic<int>> hits(1000);
      for (int job = 0; job < 300; ++job) {
        const size_t n = 1 + (size_t)(job * 37 % 1000);
        p->run(n, [&](size_t i) { hits[i].fetch_add(1, std::memory_order_relaxed); });
        for (size_t i = 0; i < hits.size(); ++i) {
          const int h = hits[i].exchange(0, std::memory_order_relaxed);
          CHECK(h == (i < n ? 1 : 0), "job %d item %zu ran %d times", job, i, h);
        }
      }
    }
  }
  CHECK(want_st[cases.size() - 3] == ENOENT, "missing path: %d", want_st[cases.size() - 3]);
  CHECK(want_st[cases.size() - 2] == EISDIR, "directory: %d", want_st[cases.size() - 2]);

  // the big-file checksum reads: 1 MiB pieces with O_DIRECT (4 KiB-aligned
  // destination, the tail piece's length rounded up) where the filesystem
  // takes it, the page cache where it refuses; both give the file's bytes
  {
    const std::string bp = path("big_direct");
    const uint64_t n = (5ull << 20) + 123;
    write_file(bp, n, rng);
    std::vector<uint8_t> want(n);
    FILE* f = std::fopen(bp.c_str(), "rb");
    CHECK(std::fread(want.data(), 1, n, f) == n, "read back");
    std::fclose(f);
    for (bool direct : {false, true}) {
      bool is_direct = false;
      const int fd = sdcas_io::open_for_read(bp.c_str(), direct, &is_direct);
      CHECK(fd >= 0, "open_for_read %d", fd);
      CHECK(direct || !is_direct, "O_DIRECT without asking");
      if (direct && !is_direct) std::printf("(O_DIRECT refused by this filesystem: page-cache fallback)\n");
      void* buf = nullptr;
      if (posix_memalign(&buf, 4096, (1u << 20) + 4096) != 0) return 2;
      for (uint64_t off = 0; off < n; off += 1u << 20) {
        const uint64_t len = std::min<uint64_t>(1u << 20, n - off);
        const int st = is_direct ? sdcas_io::pread_direct(fd, (uint8_t*)buf, len, off)
                                 : sdcas_io::pread_exact(fd, (uint8_t*)buf, len, off);
        CHECK(st == 0 && std::memcmp(buf, want.data() + off, len) == 0, "piece at %llu (direct %d): %d",
              (unsigned long long)off, (int)is_direct, st);
      }
      // one piece more than the file holds: UnexpectedEof either way
      const int st = is_direct ? sdcas_io::pread_direct(fd, (uint8_t*)buf, 1u << 20, 5ull << 20)
                               : sdcas_io::pread_exact(fd, (uint8_t*)buf, 1u << 20, 5ull << 20);
      CHECK(st == sdcas_io::kUnexpectedEof, "past EOF: %d", st);
      std::free(buf);
      close(fd);
    }
    bool d = false;
    CHECK(sdcas_io::open_for_read(path("nope").c_str(), true, &d) == -ENOENT, "missing file");
  }

  // files opened relative to a cached directory descriptor (open_for_read):
  // within a path call the descriptor serves consecutive files of one
  // directory; a directory replaced between two calls (a new epoch) is looked
  // up again, so its new file is found; the error of a missing directory is
  // the full path's; a trailing slash and a bare name take the plain open
  {
    const std::string sub = path("sub"), moved = path("sub_old");
    CHECK(mkdir(sub.c_str(), 0755) == 0, "mkdir");
    write_file(sub + "/a", 10, rng);
    sdcas_io::new_path_epoch();
    bool d = false;
    int fd = sdcas_io::open_for_read((sub + "/a").c_str(), false, &d);
    CHECK(fd >= 0, "open in sub: %d", fd);
    if (fd >= 0) close(fd);
    CHECK(std::rename(sub.c_str(), moved.c_str()) == 0, "rename");
    CHECK(mkdir(sub.c_str(), 0755) == 0, "mkdir again");
    write_file(sub + "/b", 20, rng);
    sdcas_io::new_path_epoch();  // the next call
    fd = sdcas_io::open_for_read((sub + "/b").c_str(), false, &d);
    CHECK(fd >= 0, "the replaced directory's new file: %d", fd);
    struct stat sb;
    CHECK(fd >= 0 && fstat(fd, &sb) == 0 && sb.st_size == 20, "the new directory's file");
    if (fd >= 0) close(fd);
    CHECK(sdcas_io::open_for_read((sub + "/a").c_str(), false, &d) == -ENOENT, "the old file is gone from sub");
    CHECK(sdcas_io::open_for_read(path("no_dir/x").c_str(), false, &d) == -ENOENT, "missing directory");
    fd = sdcas_io::open_for_read((sub + "/").c_str(), false, &d);
    CHECK(fd >= 0, "trailing slash opens the directory");
    if (fd >= 0) close(fd);
    CHECK(sdcas_io::open_for_read("no_such_relative_file", false, &d) == -ENOENT, "bare name");
  }

  // plan_batch: items in order, line-aligned ascending offsets, within the
  // slot (the first item of a batch always taken), at most cap_n per batch
  std::vector<uint64_t> need(5000);
  std::vector<size_t> order(need.size());
  for (size_t i = 0; i < need.size(); ++i) {
    need[i] = rng() % 300000;
    order[i] = need.size() - 1 - i;
  }
  for (uint64_t cap : {1ull << 20, 256ull << 10, 4096ull}) {
    for (size_t cap_n : {(size_t)7, (size_t)100000}) {
      size_t p = 0, batches = 0;
      std::vector<uint64_t> offs;
      while (p < need.size()) {
        uint64_t used = 0;
        const size_t q = sdcas_io::plan_batch(need.data(), order.data(), p, need.size(), cap, cap_n, offs, &used);
        CHECK(q > p && q - p <= cap_n && offs.size() == q - p, "batch [%zu, %zu)", p, q);
        uint64_t u = 0;
        for (size_t k = 0; k < offs.size(); ++k) {
          CHECK(offs[k] == u && offs[k] % 128 == 0, "offset %zu", k);
          u += sdcas_io::align_line(need[order[p + k]]);
        }
        CHECK(u == used && (q - p == 1 || used <= cap), "used %llu", (unsigned long long)used);
        p = q;
        ++batches;
      }
      CHECK(batches > 0, "no batches");
    }
  }
  std::string rm = std::string("rm -rf ") + dir;
  if (std::system(rm.c_str()) != 0) std::fprintf(stderr, "cleanup failed\n");
  if (failures) {
    std::printf("%d FAILURES\n", failures);
    return 1;
  }
  std::printf("ALL OK (%zu files x 10 reps on 8 threads: page cache, O_DIRECT, aligned reads)\n", cases.size());
  return 0;
}
