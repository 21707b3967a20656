// cas_io.cpp — see cas_io.hpp. GPU-free; linked into libsdcas.so and into the
// sanitizer test builds of tests/cpp.
#include "cas_io.hpp"

#ifndef _GNU_SOURCE
#define _GNU_SOURCE  // O_DIRECT
#endif
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>

namespace sdcas_io {

// constants of core/src/object/cas.rs:10-15
constexpr uint64_t kSampleCount = 4, kSample = 10240, kHF = 8192, kMin = 102400;
constexpr uint64_t kSampledLen = 8 + 2 * kHF + kSampleCount * kSample;  // 57352

int pread_exact(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
  uint64_t got = 0;
  while (got < n) {
    ssize_t r = pread(fd, dst + got, n - got, (off_t)(off + got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) return kUnexpectedEof;
    got += (uint64_t)r;
  }
  return 0;
}

int pread_direct(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
  const uint64_t want = (n + kDirectAlign - 1) & ~(kDirectAlign - 1);
  uint64_t got = 0;
  while (got < want) {
    ssize_t r = pread(fd, dst + got, want - got, (off_t)(off + got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) break;
    got += (uint64_t)r;
    if (got % kDirectAlign) break;  // short of a block: the file ends here (another read would be unaligned)
  }
  return got >= n ? 0 : kUnexpectedEof;
}

namespace {
// Files are opened relative to their directory, whose descriptor a reader
// thread keeps while consecutive files share it (a batch lists a location's
// files directory by directory): openat(dir, name) walks one component
// where open(path) walks them all — on the GPU box's container filesystem
// the walk is most of an open (profiles/r05_job_read_side.json). A path call
// starts a new epoch (a directory replaced between calls is looked up
// again), and every thread drops its descriptor when its share of a pool run
// ends and when the path call ends (drop_dir_cache): an idle engine holds no
// directory open, so a volume it just indexed can be unmounted. SDCAS_DIRFD=0:
// open(path) (A/B).
std::atomic<uint64_t> g_epoch{1};
bool dirfd_enabled() {
  static const bool on = [] {
    const char* v = getenv("SDCAS_DIRFD");
    return !(v && strcmp(v, "0") == 0);
  }();
  return on;
}
struct DirCache {
  uint64_t epoch = 0;
  std::string dir;
  int fd = -1;
  void drop() {
    if (fd >= 0) close(fd);
    fd = -1;
  }
  ~DirCache() { drop(); }
};
thread_local DirCache t_dir;
// the descriptor to open `path` against, and the name to open there
int dir_of(const char* path, const char** name) {
  *name = path;
  const char* slash = strrchr(path, '/');
  // a name without a directory, a file in "/", a trailing slash: the plain open
  if (!slash || slash == path || !slash[1] || !dirfd_enabled()) return AT_FDCWD;
  DirCache& c = t_dir;
  const uint64_t e = g_epoch.load(std::memory_order_relaxed);
  const size_t dl = (size_t)(slash - path);
  if (c.epoch != e || c.fd < 0 || c.dir.size() != dl || memcmp(c.dir.data(), path, dl) != 0) {
    if (c.fd >= 0) close(c.fd);
    c.dir.assign(path, dl);
    c.fd = open(c.dir.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
    c.epoch = e;
    if (c.fd < 0) return AT_FDCWD;  // the full path then reports its own error
  }
  *name = slash + 1;
  return c.fd;
}
}  // namespace

void new_path_epoch() { g_epoch.fetch_add(1, std::memory_order_relaxed); }
void drop_dir_cache() { t_dir.drop(); }

int open_for_read(const char* path, bool direct, bool* is_direct) {
  *is_direct = false;
  const char* name = path;
  const int dir = dir_of(path, &name);
  if (direct) {
    int fd = openat(dir, name, O_RDONLY | O_CLOEXEC | O_DIRECT);
    if (fd >= 0) {
      *is_direct = true;
      return fd;
    }
    if (errno != EINVAL) return -errno;
  }
  int fd = openat(dir, name, O_RDONLY | O_CLOEXEC);
  return fd >= 0 ? fd : -errno;
}

int read_whole(int fd, uint8_t* dst, uint64_t cap, uint64_t expect, uint64_t* len, bool* overflow) {
  uint64_t got = 0;
  *overflow = false;
  for (;;) {
    if (got == cap) {
      *overflow = true;
      break;
    }
    ssize_t r = pread(fd, dst + got, cap - got, (off_t)got);
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) break;
    got += (uint64_t)r;
    if (got == expect) break;
  }
  *len = got;
  return 0;
}

namespace {
// a 4 KiB-aligned buffer per reader thread for O_DIRECT reads, grown on demand
struct Bounce {
  uint8_t* p = nullptr;
  size_t n = 0;
  ~Bounce() { free(p); }
};
uint8_t* bounce(size_t need) {
  thread_local Bounce b;
  if (b.n < need) {
    free(b.p);
    b.p = nullptr;
    b.n = 0;
    void* q = nullptr;
    if (posix_memalign(&q, kDirectAlign, need)) return nullptr;
    b.p = static_cast<uint8_t*>(q);
    b.n = need;
  }
  return b.p;
}

// read_exact (tokio) with either kind of read
int read_exact_any(int fd, bool aligned, uint8_t* dst, uint64_t n, uint64_t off) {
  if (!aligned) return pread_exact(fd, dst, n, off);
  uint64_t got = 0;
  const int st = read_span_direct(fd, dst, n, off, &got);
  return st ? st : (got < n ? kUnexpectedEof : 0);
}
}  // namespace

int read_span_direct(int fd, uint8_t* dst, uint64_t n, uint64_t off, uint64_t* got) {
  *got = 0;
  const uint64_t a = off & ~(kDirectAlign - 1), head = off - a;
  const uint64_t span = (head + n + kDirectAlign - 1) & ~(kDirectAlign - 1);
  uint8_t* b = bounce(span);
  if (!b) return ENOMEM;
  uint64_t r_total = 0;
  while (r_total < span) {
    ssize_t r = pread(fd, b + r_total, span - r_total, (off_t)(a + r_total));
    if (r < 0) {
      if (errno == EINTR) continue;
      return errno;
    }
    if (r == 0) break;
    r_total += (uint64_t)r;
    if (r_total % kDirectAlign) break;  // short of a block: the file ends here
  }
  const uint64_t avail = r_total > head ? std::min<uint64_t>(r_total - head, n) : 0;
  if (avail) memcpy(dst, b + head, avail);
  *got = avail;
  return 0;
}

int read_whole_any(int fd, bool aligned, uint8_t* dst, uint64_t cap, uint64_t expect, uint64_t* len,
                   bool* overflow) {
  if (!aligned) return read_whole(fd, dst, cap, expect, len, overflow);
  *overflow = false;
  const int st = read_span_direct(fd, dst, cap, 0, len);
  if (!st && *len == cap) *overflow = true;  // the file holds at least cap bytes
  return st;
}

int read_cas_message_fd(int fd, bool aligned, uint64_t size, uint8_t* dst, uint64_t cap, uint64_t* len,
                        uint64_t* retry_len) {
  *retry_len = 0;
  *len = 0;
  for (int i = 0; i < 8; ++i) dst[i] = (uint8_t)(size >> (8 * i));  // cas.rs:25
  int st = 0;
  if (size <= kMin) {
    // cas.rs:27-29: fs::read of the file as it is now
    uint64_t got = 0;
    bool over = false;
    st = read_whole_any(fd, aligned, dst + 8, cap - 8, size, &got, &over);
    if (!st && over) {
      struct stat sb;
      if (fstat(fd, &sb) == 0) *retry_len = 8 + (uint64_t)sb.st_size + 4096;
      else st = errno;
    }
    *len = 8 + got;
  } else {
    // cas.rs:35-58: header, 4 samples at 8192 + k*seek_jump, footer at EOF-8192
    uint8_t* p = dst + 8;
    st = read_exact_any(fd, aligned, p, kHF, 0);
    p += kHF;
    const uint64_t seek_jump = (size - kHF * 2) / kSampleCount;
    for (uint64_t k = 0; !st && k < kSampleCount; ++k) {
      st = read_exact_any(fd, aligned, p, kSample, kHF + k * seek_jump);
      p += kSample;
    }
    if (!st) {
      struct stat sb;
      if (fstat(fd, &sb) != 0) st = errno;
      else if ((uint64_t)sb.st_size < kHF) st = EINVAL;  // seek(End(-8192)) before byte 0
      else st = read_exact_any(fd, aligned, p, kHF, (uint64_t)sb.st_size - kHF);
    }
    *len = kSampledLen;
  }
  return st;
}

int read_cas_message(const char* path, uint64_t size, uint8_t* dst, uint64_t cap, uint64_t* len,
                     uint64_t* retry_len, bool direct) {
  *retry_len = 0;
  *len = 0;
  bool is_direct = false;
  const int fd = open_for_read(path, direct, &is_direct);
  if (fd < 0) return -fd;
  const int st = read_cas_message_fd(fd, is_direct, size, dst, cap, len, retry_len);
  close(fd);
  return st;
}

int read_file_metadata(const char* path, bool direct, uint8_t* dst, uint64_t cap, uint64_t* len,
                       uint64_t* retry_len, uint64_t* size, bool* is_dir) {
  *len = 0;
  *retry_len = 0;
  *size = 0;
  *is_dir = false;
  bool aligned = false;
  const int fd = open_for_read(path, direct, &aligned);
  struct stat sb;
  if (fd < 0) {
    if (stat(path, &sb) != 0) return errno;  // fs::metadata fails (mod.rs:63-65)
    *size = (uint64_t)sb.st_size;
    *is_dir = S_ISDIR(sb.st_mode);
    return *is_dir || sb.st_size == 0 ? 0 : -fd;  // generate_cas_id's open fails (mod.rs:78-82)
  }
  if (fstat(fd, &sb) != 0) {
    const int e = errno;
    close(fd);
    return e;
  }
  *size = (uint64_t)sb.st_size;
  *is_dir = S_ISDIR(sb.st_mode);
  int st = 0;
  if (!*is_dir && *size) {  // mod.rs:67-70, 78-86: no cas_id for a directory or an empty file
    const uint64_t need = (*size <= kMin ? 8 + *size + 1 : kSampledLen);
    if (need > cap) *retry_len = need;
    else st = read_cas_message_fd(fd, aligned, *size, dst, cap, len, retry_len);
  }
  close(fd);
  return st;
}

size_t plan_batch(const uint64_t* need, const size_t* order, size_t p, size_t end, uint64_t cap, size_t cap_n,
                  std::vector<uint64_t>& offs, uint64_t* used) {
  offs.clear();
  uint64_t u = 0;
  size_t q = p;
  while (q < end && q - p < cap_n) {
    const uint64_t nb = align_line(need[order ? order[q] : q]);
    if (q > p && u + nb > cap) break;
    offs.push_back(u);
    u += nb;
    ++q;
  }
  *used = u;
  return q;
}

WorkerPool::WorkerPool(uint32_t threads) {
  for (uint32_t t = 1; t < threads; ++t) workers_.emplace_back([this] { loop(); });
}

WorkerPool::~WorkerPool() {
  {
    std::lock_guard<std::mutex> g(m_);
    stop_ = true;
  }
  go_.notify_all();
  for (auto& t : workers_) t.join();
}

void WorkerPool::drain() {
  for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < n_;) (*fn_)(i);
}

void WorkerPool::dispatch(size_t n, const std::function<void(size_t)>* fn) {
  {
    std::lock_guard<std::mutex> g(m_);
    fn_ = fn;
    n_ = n;
    next_.store(0, std::memory_order_relaxed);
    active_ = workers_.size();
    ++gen_;
  }
  go_.notify_all();
  drain();  // the calling thread is one of the workers
  drop_dir_cache();
  std::unique_lock<std::mutex> g(m_);
  done_.wait(g, [this] { return active_ == 0; });
  fn_ = nullptr;
}

void WorkerPool::loop() {
  uint64_t seen = 0;
  std::unique_lock<std::mutex> g(m_);
  for (;;) {
    go_.wait(g, [&] { return stop_ || gen_ != seen; });
    if (stop_) return;
    seen = gen_;
    g.unlock();
    drain();
    drop_dir_cache();  // no directory descriptor held while the pool idles
    g.lock();
    if (--active_ == 0) done_.notify_one();
  }
}

}  // namespace sdcas_io
